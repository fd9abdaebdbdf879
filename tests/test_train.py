"""Training path on the CPU: prep_batch against the reference's golden offsets, the
single-process trainer (steps, EMA, checkpoint round trip in the Lightning layout), and the
data-parallel path at world_size 2 over gloo (DDP's bucketed all-reduce must equal the mean of
the ranks' local gradients; replicas stay bit-identical after the optimizer step)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

SMALL = ["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames", "8", "--crop", "4",
         "--embed_dim", "32", "--mha_heads", "4", "--num_layers", "2", "--ipa_heads", "2", "--ipa_head_dim", "8",
         "--ipa_qk", "4", "--ipa_v", "4", "--batch_size", "2", "--synthetic_size", "8", "--print_freq", "1000"]


def _args(extra=(), tmp=None):
    from mdgen_finetune_amd.parsing import parse_train_args

    argv = list(SMALL) + list(extra)
    if tmp is not None:
        argv += ["--model_dir", str(tmp)]
    return parse_train_args(argv)


def _batch(args, B=2, seed=0):
    from mdgen_finetune_amd.data import SyntheticMDDataset, collate

    ds = SyntheticMDDataset(args.num_frames, args.crop, size=B, seed=seed)
    return collate([ds[i] for i in range(B)])


def test_prep_batch_matches_reference_golden(golden):
    """Offsets/sign fix/cond mask/x_cond vs the reference's get_offsets (utils.py:7-14) and the
    prep_batch glue (wrapper.py:283-365) — tests/golden/prep_batch.npz, oracle/gen_golden.py."""
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    d, cfg = golden("prep_batch")
    for tps in (False, True):
        extra = ["--tps_condition"] if tps else []
        a = _args(extra)
        a.sim_condition = not tps
        w = NewMDGenWrapper(a)
        batch = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("in_")}
        p = w.prep_batch(batch)
        sfx = "_tps" if tps else ""
        np.testing.assert_allclose(p["latents"].numpy(), d["out_latents" + sfx], rtol=0, atol=2e-6)
        np.testing.assert_array_equal(p["loss_mask"].numpy(), d["out_loss_mask" + sfx])
        np.testing.assert_array_equal(p["model_kwargs"]["x_cond_mask"].numpy(), d["out_cond_mask" + sfx])


def test_trainer_steps_ema_and_checkpoint_roundtrip(tmp_path):
    from mdgen_finetune_amd.checkpoint import load_checkpoint, load_from_checkpoint
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--ema", "--ema_decay", "0.9", "--max_steps", "3", "--epochs", "1"], tmp_path)
    tr = Trainer(a)
    w0 = {k: v.clone() for k, v in tr.wrapper.model.state_dict().items()}
    tr.fit()
    assert tr.global_step == 3
    changed = [k for k, v in tr.wrapper.model.state_dict().items() if not torch.equal(v, w0[k])]
    assert len(changed) > 10
    ema = tr.wrapper.ema.state_dict()["params"]
    k = "layers.0.mha_t.attn.q_proj.weight"
    assert not torch.equal(ema[k], tr.wrapper.model.state_dict()[k])
    files = sorted(os.listdir(tmp_path))
    assert files and files[-1].endswith(".ckpt")
    ck = load_checkpoint(os.path.join(tmp_path, files[-1]))
    assert set(ck) >= {"state_dict", "hyper_parameters", "optimizer_states", "ema", "epoch", "global_step"}
    assert all(key.startswith("model.") for key in ck["state_dict"])
    w2 = load_from_checkpoint(os.path.join(tmp_path, files[-1]))
    for key, v in tr.wrapper.model.state_dict().items():
        assert torch.equal(v, w2.model.state_dict()[key]), key
    assert torch.equal(w2.ema.state_dict()["params"][k], ema[k])
    # resume continues the step counter and the optimizer state
    a2 = _args(["--ema", "--max_steps", "4", "--epochs", "2", "--ckpt", os.path.join(tmp_path, files[-1])], tmp_path)
    tr2 = Trainer(a2)
    assert tr2.global_step == 3 and len(tr2.optimizer.state) > 0
    tr2.fit()
    assert tr2.global_step == 4


def test_loss_decreases_on_fixed_batch():
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--lr", "1e-3"])
    tr = Trainer(a)
    b = _batch(a)
    torch.manual_seed(0)
    first = [tr.step([b])[0].item() for _ in range(3)]
    for _ in range(30):
        tr.step([b])
    last = [tr.step([b])[0].item() for _ in range(3)]
    assert np.mean(last) < np.mean(first)


def test_grad_accumulation_equals_big_batch():
    """accumulate_grad=2 over two halves == one step over the whole batch (same noise)."""
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--grad_clip", "0"])
    b = _batch(a, B=4)
    halves = [{k: (v[:2] if torch.is_tensor(v) else v[:2]) for k, v in b.items()},
              {k: (v[2:] if torch.is_tensor(v) else v[2:]) for k, v in b.items()}]
    grads = []
    for mb in ([b], halves):
        tr = Trainer(a)
        noise = torch.Generator().manual_seed(5)
        x0 = torch.randn(4, 8, 4, 21, generator=noise)
        t = torch.rand(4, generator=noise)
        it = iter([(t[:2], x0[:2]), (t[2:], x0[2:])] if len(mb) == 2 else [(t, x0)])
        tr.wrapper.transport.sample = lambda x1, it=it: (lambda tx: (tx[0], tx[1], x1))(next(it))
        seen = []
        orig = tr.optimizer.step
        tr.optimizer.step = lambda *a_, **k_: (seen.append(torch.cat([p.grad.flatten().clone() for p in
                                                                      tr.wrapper.model.parameters()
                                                                      if p.grad is not None])), orig())[1]
        tr.step(mb)
        grads.append(seen[0])
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-5, atol=1e-6)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    from mdgen_finetune_amd import synthetic

    r, w, dev = setup_distributed()
    dist._DEFAULT_FIRST_BUCKET_BYTES = 50 * 1024  # DDP's first bucket would hold this whole small model
    a = _args(["--grad_clip", "0", "--bucket_cap_mb", "0.05", "--cond_allgather", "0"])
    tr = Trainer(a, r, w, dev)
    synthetic.fill_module_(tr.wrapper.model, 21)  # non-zero gradients everywhere (zero-init layers pass none)
    b = _batch(a, B=2, seed=100 + rank)
    # local gradient without communication, from the same (t, x0) draw
    g = torch.Generator().manual_seed(7 + rank)
    x0, t = torch.randn(2, 8, 4, 21, generator=g), torch.rand(2, generator=g)
    tr.wrapper.transport.sample = lambda x1: (t, x0, x1)
    # record the order in which DDP launches bucket all-reduces and autograd finishes gradients
    from torch.distributed.algorithms.ddp_comm_hooks.default_hooks import allreduce_hook

    events = []

    def hook(state, bucket):
        events.append(("bucket", bucket.index()))
        return allreduce_hook(None, bucket)

    tr.model.register_comm_hook(None, hook)
    for n, p in tr.wrapper.model.named_parameters():
        p.register_post_accumulate_grad_hook(lambda p, n=n: events.append(("grad", n)))
    prep = tr.wrapper.prep_batch(b)
    loss = tr.wrapper.transport.training_losses(tr.wrapper.model, prep["latents"], mask=prep["loss_mask"],
                                                model_kwargs=prep["model_kwargs"])["loss"].mean()
    local = torch.autograd.grad(loss, [p for p in tr.wrapper.model.parameters()], allow_unused=True)
    local = torch.cat([(x if x is not None else torch.zeros_like(p)).flatten()
                       for x, p in zip(local, tr.wrapper.model.parameters())])
    ref = local.clone()
    dist.all_reduce(ref)
    ref /= w
    # the DDP path (bucketed all-reduce during backward)
    # DDP does not bucket its first iterations (one all-reduce after backward; with static_graph
    # the buckets are rebuilt in backward order after iteration 2), so measure on the third
    for _ in range(2):
        tr.wrapper.general_step(b, model=tr.model).backward()
        tr.optimizer.zero_grad(set_to_none=True)
    events.clear()
    loss = tr.wrapper.general_step(b, model=tr.model)
    loss.backward()
    kinds = [k for k, _ in events]
    n_buckets = len({i for k, i in events if k == "bucket"})
    first_bucket = kinds.index("bucket") if "bucket" in kinds else len(kinds)
    last_grad = len(kinds) - 1 - kinds[::-1].index("grad") if "grad" in kinds else -1
    ddp = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).flatten()
                     for p in tr.wrapper.model.parameters()])
    tr.optimizer.step()
    params = torch.cat([p.detach().flatten() for p in tr.wrapper.model.parameters()])
    gathered = [torch.zeros_like(params) for _ in range(w)]
    dist.all_gather(gathered, params)
    out[rank] = (float((ddp - ref).abs().max()), float(ref.abs().max()),
                 float((gathered[0] - gathered[1]).abs().max()), float((local - ref).abs().max()),
                 n_buckets, first_bucket, last_grad)
    dist.destroy_process_group()


def test_ddp_world2_gloo_allreduce_matches_local_mean():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_ddp_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        err, scale, drift, spread, n_buckets, first_bucket, last_grad = out[r]
        assert err <= 1e-6 * max(1.0, scale), (r, err, scale)
        assert drift == 0.0
        assert spread > 0.0  # the ranks really had different data
        # overlap: several buckets, and the first bucket's all-reduce was launched while
        # backward was still producing gradients (before the last parameter's grad landed)
        assert n_buckets >= 2, n_buckets
        assert first_bucket < last_grad, (first_bucket, last_grad)


def _bucket_worker(rank, world, port, out):
    """grad_buckets.BucketedAllReduce (the graphed step's in-capture all-reduce) run eagerly over
    gloo: the order recorded from one backward, the buckets launched from the hooks."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mdgen_finetune_amd.grad_buckets import BucketedAllReduce, record_grad_order
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    from mdgen_finetune_amd import synthetic

    r, w, dev = setup_distributed()
    a = _args(["--grad_clip", "0", "--cond_allgather", "0"])
    tr = Trainer(a, r, w, dev)
    m = tr.wrapper.model
    synthetic.fill_module_(m, 21)  # non-zero gradients everywhere
    params = [p for p in m.parameters() if p.requires_grad]
    b = _batch(a, B=2, seed=100 + rank)
    g = torch.Generator().manual_seed(7 + rank)
    x0, t = torch.randn(2, 8, 4, 21, generator=g), torch.rand(2, generator=g)
    tr.wrapper.transport.sample = lambda x1: (t, x0, x1)

    def backward():
        m.zero_grad(set_to_none=True)
        tr.wrapper.general_step(b, model=m).backward()

    order, unhook = record_grad_order(params)
    backward()
    unhook()
    local = [p.grad.clone() if p.grad is not None else None for p in params]
    red = BucketedAllReduce(params, order, cap_bytes=40 * 1024, world=w)
    red.attach()
    backward()
    red.finish()
    err, scale = 0.0, 0.0
    for p, lg in zip(params, local):
        if lg is None:
            assert p.grad is None
            continue
        ref = lg.clone()
        dist.all_reduce(ref)
        ref /= w
        err = max(err, float((p.grad - ref).abs().max()))
        scale = max(scale, float(ref.abs().max()))
    # a second step through the same reducer (hooks re-armed) gives the same averages
    g1 = red.flat.clone()
    red.attach()
    backward()
    red.finish()
    out[rank] = (err, scale, len(red.buckets), red.launch_log, len(order), float((red.flat - g1).abs().max()),
                 sum((p.numel() + 3) // 4 * 4 for p, lg in zip(params, local) if lg is not None) == red.flat.numel()
                 and all((v.data_ptr() - red.flat.data_ptr()) % 16 == 0 for v in red.views.values()))
    dist.destroy_process_group()


def test_bucketed_allreduce_world2_gloo_overlaps_and_averages():
    """The graphed step's bucketed all-reduce (grad_buckets.py), world 2 over gloo: every
    gradient equals the ranks' mean, the buckets follow backward's completion order, and the
    first bucket is reduced before backward has produced the last gradient (overlap)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        err, scale, nb, log, n_grads, drift, covers = out[r]
        assert err <= 1e-6 * max(1.0, scale), (r, err, scale)
        assert nb >= 3, nb
        assert [bi for bi, _ in log] == list(range(nb)), log  # launched in layout order
        assert log[0][1] < n_grads, (log, n_grads)  # before the last gradient landed
        assert drift == 0.0
        assert covers


def _bucket_order_worker(rank, world, port, out):
    """Rank agreement of grad_buckets.BucketedAllReduce: rank 1 records a PERMUTED completion order
    and fires its hooks in yet another order; the layout must still be rank 0's, the buckets must
    be reduced in layout order on both ranks, and every parameter averaged with itself.  Then a
    rank that reached a different gradient set, and a hook firing twice, must raise."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from mdgen_finetune_amd.grad_buckets import BucketedAllReduce

    sizes = [300, 17, 1024, 5, 640, 96, 2048, 33, 512, 7]
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    order0 = list(range(len(sizes)))
    perm = [7, 2, 9, 0, 4, 1, 8, 3, 6, 5]
    red = BucketedAllReduce(params, order0 if rank == 0 else perm, cap_bytes=4 * 1100, world=world)
    layouts = [None] * world
    dist.all_gather_object(layouts, red.buckets)
    red.attach()
    gen = torch.Generator().manual_seed(40 + rank)
    local = [torch.randn(n, generator=gen) for n in sizes]
    fire = order0 if rank == 0 else list(reversed(perm))  # rank 1 completes in another order still
    for i in fire:
        params[i].grad = local[i].clone()
        red._ready(i)
    red.finish()
    err = 0.0
    for p, lg in zip(params, local):
        ref = lg.clone()
        dist.all_reduce(ref)
        ref /= world
        err = max(err, float((p.grad - ref).abs().max()))
    res = dict(layouts=layouts, log=[bi for bi, _ in red.launch_log], nb=len(red.buckets), err=err)
    # a hook that fires twice in one backward
    red.attach()
    params[0].grad = local[0].clone()
    red._ready(0)
    try:
        red._ready(0)
        res["dup"] = "no error"
    except RuntimeError as e:
        res["dup"] = str(e)
    # drain the collectives rank 0's single fire may have launched (same sequence on both ranks)
    for i in order0[1:]:
        params[i].grad = local[i].clone()
        red._ready(i)
    red.finish()
    # a rank whose backward reached a different set of gradients
    try:
        BucketedAllReduce(params, order0 if rank == 0 else order0[:-1], cap_bytes=4 * 1100, world=world)
        res["mismatch"] = "no error"
    except RuntimeError as e:
        res["mismatch"] = str(e)
    # same numels, one parameter shaped differently on rank 1
    shaped = [torch.nn.Parameter(torch.zeros(32, 32) if (rank == 1 and n == 1024) else torch.zeros(n)) for n in sizes]
    try:
        BucketedAllReduce(shaped, order0, cap_bytes=4 * 1100, world=world)
        res["shape"] = "no error"
    except RuntimeError as e:
        res["shape"] = str(e)
    out[rank] = res
    dist.destroy_process_group()


def test_bucket_layout_agreed_across_ranks_world2_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_order_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0["layouts"][0] == r0["layouts"][1] == r1["layouts"][0]
    assert [i for b in r0["layouts"][0] for i in b] == list(range(10))  # rank 0's order
    for r in (r0, r1):
        assert r["nb"] >= 3
        assert r["log"] == list(range(r["nb"])), r["log"]
        assert r["err"] <= 1e-6, r["err"]
        assert "fired twice" in r["dup"], r["dup"]
        assert "different set of gradients" in r["mismatch"], r["mismatch"]
        assert "different shapes" in r["shape"], r["shape"]


def _cond_gather_worker(rank, world, port, out):
    """Replicated conditioning (cond_dist.py) under DDP, world 2 over gloo: every parameter's
    averaged gradient — the conditioning's from the all-gathered batch, the rest from DDP's
    all-reduce — equals the single-process gradient of the mean loss over both ranks' batches."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mdgen_finetune_amd.data import collate
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    from mdgen_finetune_amd import synthetic

    r, w, dev = setup_distributed()
    dist._DEFAULT_FIRST_BUCKET_BYTES = 50 * 1024
    a = _args(["--grad_clip", "0", "--bucket_cap_mb", "0.05"])
    tr = Trainer(a, r, w, dev)
    m = tr.wrapper.model
    # non-zero weights everywhere (a fresh model's zero-init adaLN / final layers pass no gradient
    # to anything upstream); DDP broadcast the old values at wrap time, so fill on every rank alike
    synthetic.fill_module_(m, 21)
    assert m._cond_gather is not None and len(tr.replicated) > 0
    batches = [_batch(a, B=2, seed=100 + k) for k in range(w)]
    noise = []
    for k in range(w):
        g = torch.Generator().manual_seed(7 + k)
        noise.append((torch.rand(2, generator=g), torch.randn(2, 8, 4, 21, generator=g)))
    t, x0 = noise[rank]
    tr.wrapper.transport.sample = lambda x1: (t, x0, x1)
    for _ in range(3):  # DDP buckets from its third iteration (static graph); measure the last
        tr.optimizer.zero_grad(set_to_none=True)
        with tr.cond_active():  # (the Trainer's own step sets this)
            tr.wrapper.general_step(batches[rank], model=tr.model).backward()
    got = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    # single-process reference: a fresh trainer (same seed = same weights), no gather, both batches
    a1 = _args(["--grad_clip", "0"])
    ref = Trainer(a1)
    rm = ref.wrapper.model
    synthetic.fill_module_(rm, 21)
    tt = torch.cat([n_[0] for n_ in noise])
    xx = torch.cat([n_[1] for n_ in noise])
    ref.wrapper.transport.sample = lambda x1: (tt, xx, x1)
    big = collate([{k: v[i] if torch.is_tensor(v) else v[i] for k, v in b.items()} for b in batches for i in range(2)])
    ref.wrapper.general_step(big, model=rm).backward()
    want = {n: p.grad for n, p in rm.named_parameters() if p.grad is not None}
    rep = {n for n, p in m.named_parameters() if id(p) in tr.replicated}
    worst, worst_rep = 0.0, 0.0
    nonzero = sum(1 for n in rep if n in want and float(want[n].abs().max()) > 0)
    assert nonzero > 20, nonzero
    for n, g in want.items():
        e = float((got[n] - g).abs().max()) / max(1e-12, float(g.abs().max()))
        worst = max(worst, e)
        if n in rep:
            worst_rep = max(worst_rep, e)
    out[rank] = (worst, worst_rep, len(rep), len(want), sorted(set(want) - set(got)))
    dist.destroy_process_group()


def test_replicated_conditioning_world2_gloo_equals_big_batch():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_cond_gather_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        worst, worst_rep, n_rep, n_all, missing = out[r]
        assert not missing, missing
        assert n_rep > 20 and n_all > n_rep
        assert worst <= 1e-4, (r, worst, worst_rep)


def _graph_path_worker(rank, world, port, tps, out):
    """The graphed step's data-parallel objects without the capture, world 2 over gloo: the
    replicated conditioning (cond_dist.CondGather, its own process group) and the bucketed
    all-reduce of every other gradient (grad_buckets.BucketedAllReduce), composed exactly as
    train.GraphedStep composes them.  Records the (op, numel, group) sequence of every collective
    both objects issue across forward + backward, and the resulting gradients."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mdgen_finetune_amd.data import collate
    from mdgen_finetune_amd.grad_buckets import BucketedAllReduce, record_grad_order
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    from mdgen_finetune_amd import synthetic

    r, w, dev = setup_distributed()
    extra = ["--grad_clip", "0"] + (["--tps_condition"] if tps else [])

    def targs():
        a_ = _args(extra)
        a_.sim_condition = not tps
        return a_

    a = targs()
    tr = Trainer(a, r, w, dev)
    m = tr.wrapper.model
    synthetic.fill_module_(m, 21)
    cg = m._cond_gather
    lat = 28 if tps else 21
    batches = [_batch(a, B=2, seed=100 + k) for k in range(w)]
    noise = []
    for k in range(w):
        g = torch.Generator().manual_seed(7 + k)
        noise.append((torch.rand(2, generator=g), torch.randn(2, 8, 4, lat, generator=g)))
    t, x0 = noise[rank]
    tr.wrapper.transport.sample = lambda x1: (t, x0, x1)
    params = [p for p in m.parameters() if p.requires_grad]

    def backward():
        m.zero_grad(set_to_none=True)
        with tr.cond_active():
            tr.wrapper.general_step(batches[rank], model=m).backward()

    order, unhook = record_grad_order(params)
    backward()
    unhook()
    order = [i for i in order if id(params[i]) not in tr.replicated]
    red = BucketedAllReduce(params, order, cap_bytes=40 * 1024, world=w)
    log = []
    cg.log = red.log = log
    seqs = []
    for _ in range(2):
        log.clear()
        red.attach()
        backward()
        red.finish()
        seqs.append(list(log))
    # outside the Trainer's step (an eval-style grad-enabled call on one rank): no collective
    log.clear()
    if rank == 1:
        m.zero_grad(set_to_none=True)
        tr.wrapper.general_step(batches[rank], model=m)
    outside = list(log)
    m.zero_grad(set_to_none=True)
    log.clear()
    red.attach()
    backward()
    red.finish()
    got = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    # single-process reference: same weights, both ranks' batches and noise in one batch
    ref = Trainer(targs())
    rm = ref.wrapper.model
    synthetic.fill_module_(rm, 21)
    tt = torch.cat([n_[0] for n_ in noise])
    xx = torch.cat([n_[1] for n_ in noise])
    ref.wrapper.transport.sample = lambda x1: (tt, xx, x1)
    big = collate([{k: v[i] if torch.is_tensor(v) else v[i] for k, v in b.items()} for b in batches for i in range(2)])
    ref.wrapper.general_step(big, model=rm).backward()
    want = {n: p.grad for n, p in rm.named_parameters() if p.grad is not None}
    worst = 0.0
    for n, g in want.items():
        worst = max(worst, float((got[n] - g).abs().max()) / max(1e-12, float(g.abs().max())))
    out[rank] = dict(seqs=seqs, outside=outside, worst=worst, missing=sorted(set(want) - set(got)),
                     n_rep=len(tr.replicated), own_group=cg.group is not None and cg.group != dist.group.WORLD)
    dist.destroy_process_group()


@pytest.mark.parametrize("tps", [False, True])
def test_graph_path_collective_sequence_world2_gloo(tps):
    """Both ranks issue the same (op, numel, group) sequence of collectives across forward and
    backward — the conditioning's all-gathers on their own group, the buckets' all-reduces in
    layout order on the default group — step after step; a grad-enabled call outside the
    Trainer's step issues none; and the composed gradients equal the big-batch step's (sim and
    TPS: VERDICT r05 missing 3, the TPS conditioning replicated too)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_graph_path_worker, args=(2, _free_port(), tps, out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0["seqs"][0] == r1["seqs"][0] == r0["seqs"][1] == r1["seqs"][1]
    seq = r0["seqs"][0]
    cond = [e for e in seq if e[2] == "cond"]
    assert len(cond) == 2, seq  # forward inputs, backward row gradients
    assert len([e for e in seq if e[2] == "buckets"]) >= 3, seq
    assert seq[0][2] == "cond"  # the inputs' gather comes first (forward)
    assert r0["outside"] == [] and r1["outside"] == []
    for r in (r0, r1):
        assert r["own_group"]
        assert not r["missing"], r["missing"]
        assert r["n_rep"] > 20
        assert r["worst"] <= 1e-4, r["worst"]


def _replica_worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    r, w, dev = setup_distributed()
    # a different seed per rank: the initial weights differ until the Trainer broadcasts rank 0's
    tr = Trainer(_args(["--seed", str(137 + rank), "--ema"]), r, w, dev)
    m = tr.wrapper.model
    flat = torch.cat([p.detach().flatten() for p in m.parameters()])
    both = [torch.empty_like(flat) for _ in range(w)]
    dist.all_gather(both, flat)
    res = dict(same_init=bool(torch.equal(both[0], both[1])))
    res["n0"] = tr.check_replicas()
    tr.step([_batch(tr.args, B=2, seed=100 + rank)])
    res["n_step"] = tr.check_replicas()
    if rank == 1:  # a replicated-conditioning weight drifts by one ulp on one rank
        with torch.no_grad():
            p = m.t_embedder.mlp[0].weight
            p.view(-1)[0] = torch.nextafter(p.view(-1)[0], torch.tensor(1e9))
    res["n_drift"] = tr.check_replicas()
    res["n_after"] = tr.check_replicas()
    flat = torch.cat([p.detach().flatten() for p in m.parameters()])
    dist.all_gather(both, flat)
    res["same_after"] = bool(torch.equal(both[0], both[1]))
    out[rank] = res
    dist.destroy_process_group()


def test_replicas_broadcast_and_checked_world2_gloo():
    """Rank 0's initial state reaches every rank (graph mode has no DDP to broadcast it, and DDP
    skips the replicated conditioning), and check_replicas finds a one-ulp drift of a replicated
    weight on one rank and repairs it from rank 0."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_replica_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        res = out[r]
        assert res["same_init"], res
        assert res["n0"] == 0 and res["n_step"] == 0, res
        assert res["n_drift"] >= 1, res
        assert res["n_after"] == 0 and res["same_after"], res


def _bench_worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    el = bench.max_over_ranks(1.0 + 0.5 * rank, world, torch.device("cpu"))  # rank r timed 1 + r/2 s
    out[rank] = (el, bench.job_value(world, 16, 1000, 49, 10, el))
    dist.destroy_process_group()


def test_bench_n_rank_reporting_world2_gloo():
    """bench.py's N-rank reduction: every rank sees the max-over-ranks time, and the reported
    value is the WHOLE-job frames (world x B x T x 49 x steps) over that time."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        el, value = out[r]
        assert el == 1.5
        assert value == 2 * 16 * 1000 * 49 * 10 / 1.5


def test_precision_strings_mapped_or_refused():
    from mdgen_finetune_amd.train import resolve_precision

    cpu = torch.device("cpu")
    assert resolve_precision("32-true", cpu) is None
    assert resolve_precision("bf16-mixed", cpu) == torch.bfloat16
    for bad in ("bf16-true", "16-true", "64", "mixed"):
        with pytest.raises(NotImplementedError):
            resolve_precision(bad, cpu)


def test_resume_mid_epoch_continues_same_epoch(tmp_path):
    """A --max_steps save lands mid-epoch: resuming finishes that epoch's remaining batches
    (Lightning's fit-loop semantics) instead of skipping to the next epoch."""
    from mdgen_finetune_amd.checkpoint import load_checkpoint
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--max_steps", "1", "--epochs", "1", "--synthetic_size", "8"], tmp_path)  # 4 batches / epoch
    tr = Trainer(a)
    tr.fit()
    path = os.path.join(tmp_path, sorted(os.listdir(tmp_path))[-1])
    ck = load_checkpoint(path)
    assert ck["loops"]["fit_loop"] == {"epoch_complete": False, "batches_done": 1}
    a2 = _args(["--epochs", "1", "--synthetic_size", "8", "--ckpt", path], tmp_path)
    tr2 = Trainer(a2)
    assert tr2.epoch == 0 and tr2.skip_batches == 1
    tr2.fit()
    assert tr2.global_step == 4  # 1 before the save + the epoch's 3 remaining batches


def test_hip_training_gate_by_head_dim_and_dropout():
    """_use_hip_layers (latent_model.py): head_dim 32..63 takes the HIP training kernels since
    ABI 23 (--embed_dim 256 --mha_heads 8), head_dim 64 and dropout > 0 are refused with one
    RuntimeWarning per reason and train eagerly (no GPU needed: the gate reads shapes / flags)."""
    import types
    import warnings

    from tests.conftest import build_model

    m, _ = build_model(dict(flags=["--embed_dim", "256", "--mha_heads", "8", "--num_layers", "1"], latent_dim=21, L=4,
                            T=4, tps=False, weights_seed=1), "cpu", T=4)
    m.train()
    dev = types.SimpleNamespace(is_cuda=True)  # stands in for a ROCm tensor
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert m._use_hip_layers(dev)  # head_dim 32
    m.args.mha_heads = 4  # head_dim 64
    with pytest.warns(RuntimeWarning, match="head_dim 64"):
        assert not m._use_hip_layers(dev)
    m.args.mha_heads, m.args.dropout = 8, 0.1
    with pytest.warns(RuntimeWarning, match="dropout"):
        assert not m._use_hip_layers(dev)
    m.eval()  # dropout only matters while training
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert m._use_hip_layers(dev)
