"""bench.py's N-GPU launch path on the CPU (MDG_BENCH_DRYRUN=1: the workers rendezvous over gloo
and time a fixed sleep instead of the model): `bench.py --gpus 2` with no launcher spawns the
ranks itself, under torch.distributed.run each launched process starts its own rank's worker,
either way ONE JSON line with n_gpus 2 and a train_dp object comes out on stdout; a WORLD_SIZE
that disagrees with --gpus is refused; a train_dp leg whose rank dies is reported as failed
while the inference line stands (VERDICT r05 "next" 1)."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MDG_BENCH_DRYRUN="1", MASTER_ADDR="127.0.0.1", **kw)
    return env


def _lines(stdout):
    return [ln for ln in stdout.splitlines() if ln.strip()]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _check(line, launch):
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["leg"] == "infer", d
    assert d["train_dp"]["n_gpus"] == 2 and d["train_dp"]["leg"] == "train_dp", d
    assert launch in d["launch"], d
    return d


def test_self_launch_two_ranks_one_line():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], "self-launched")


def test_torchrun_two_ranks_one_line():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), BENCH, "--gpus", "2",
                        "--steps", "3", "--warmup", "1"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in _lines(r.stdout) if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    _check(lines[0], "torch.distributed.run")


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="3"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
    assert not _lines(r.stdout)


def test_failed_train_dp_leg_reported_inference_line_stands():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1", "--train-dp-timeout", "20"],
                       env=_env(MDG_BENCH_DRYRUN_FAIL="train_dp"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["leg"] == "infer"
    assert d["train_dp"]["status"] == "failed" and 3 in d["train_dp"]["worker_exit"], d["train_dp"]
