"""Training-step throughput: the GVP flow-matching step of the default model
(5 layers, C=384) at T=1000, L=4, B per GPU, on this process's GPU (or N ranks under
torch.distributed.run: DDP over RCCL).  Prints one JSON line from rank 0.

    python tools/train_bench.py --batch 8 --steps 5 --warmup 2 [--precision bf16-mixed]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mdgen_finetune_amd.parsing import parse_train_args  # noqa: E402
from mdgen_finetune_amd.train import Trainer, setup_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--crop", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default="32-true")
    ap.add_argument("--bucket_cap_mb", type=int, default=32)
    ap.add_argument("--train_backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--hip_dtype", default="bf16", choices=["bf16", "f32"])
    a = ap.parse_args()
    rank, world, dev = setup_distributed()
    args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb",
                             "--num_frames", str(a.frames), "--crop", str(a.crop), "--batch_size", str(a.batch),
                             "--synthetic_size", str(a.batch * world), "--precision", a.precision,
                             "--bucket_cap_mb", str(a.bucket_cap_mb),
                             "--train_backend", a.train_backend, "--hip_dtype", a.hip_dtype])
    torch.set_float32_matmul_precision("medium")
    tr = Trainer(args, rank, world, dev)
    batch = next(iter(tr.loader))
    for _ in range(a.warmup):
        loss, _ = tr.step([batch])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = tr.step([batch])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        print(json.dumps({
            "metric": "training frames/sec (GVP flow-matching step, forward+backward+Adam)",
            "value": round(world * a.batch * a.frames * a.steps / el, 1), "unit": "frames/s",
            "n_gpus": world, "ms_per_step": round(el / a.steps * 1e3, 2), "batch_per_gpu": a.batch,
            "frames": a.frames, "crop": a.crop, "precision": a.precision,
            "train_backend": a.train_backend, "hip_dtype": a.hip_dtype if a.train_backend == "hip" else None, "loss": float(loss),
            "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
