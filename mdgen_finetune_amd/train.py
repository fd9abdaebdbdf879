"""Data-parallel trainer: the drop-in for the reference's ``src/train.py`` (a Lightning
``Trainer.fit`` over ``NewMDGenWrapper``), rebuilt as one process per GPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m mdgen_finetune_amd.train --sim_condition --prepend_ipa --abs_pos_emb \
        --num_frames 1000 --crop 4 --batch_size 8 --synthetic

Per optimizer step (train.py:46-60 + wrapper.py:78-173 semantics):
  * each rank draws its own ``batch_size`` items (DistributedSampler shard of the epoch's
    permutation) and computes the GVP flow-matching loss (wrapper.general_step);
  * backward through ``DistributedDataParallel``: gradients are averaged over ranks by
    bucketed all-reduces that RCCL runs over xGMI while backward is still producing the
    earlier layers' gradients (``bucket_cap_mb``; static graph, buckets as grad views);
  * ``accumulate_grad`` micro-batches per step (the non-final ones under ``no_sync``, loss
    divided by the count as Lightning does);
  * global grad-norm clip (``grad_clip``, Lightning's default 'norm' algorithm), Adam/AdamW,
    then the EMA update (on_before_zero_grad);
  * every ``print_freq`` steps the logs are gathered from all ranks (wrapper.py:22-44) and
    rank 0 prints their means; every ``ckpt_freq`` epochs rank 0 writes a Lightning-layout
    checkpoint to MODEL_DIR (checkpoint.py).
Resuming (``--ckpt``) restores weights, optimizer, EMA, epoch and step.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from .checkpoint import load_checkpoint, model_state_dict, save_checkpoint
from .data import MDGenDataset, SyntheticMDDataset, collate
from .grad_buckets import BucketedAllReduce, record_grad_order
from .parsing import parse_train_args
from .wrapper import NewMDGenWrapper


def gather_log(log, world_size):
    """wrapper.py:22-29."""
    if world_size == 1:
        return log
    out = [None] * world_size
    dist.all_gather_object(out, log)
    merged = defaultdict(list)
    for lg in out:
        for k, v in lg.items():
            merged[k].extend(v)
    return dict(merged)


def get_log_mean(log):
    """wrapper.py:31-43 (numeric entries only)."""
    out = {}
    for k, v in log.items():
        try:
            out[k] = float(np.nanmean(v))
        except (TypeError, ValueError):
            pass
    return out


def setup_distributed():
    """Rank/world from the torch.distributed.run environment; RCCL on GPUs, gloo on CPU.
    MDG_SHARE_GPU=1 puts every rank on cuda:0 with gloo (rehearsing N ranks on a one-GPU box:
    RCCL refuses two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    share = os.environ.get("MDG_SHARE_GPU") == "1"
    device = torch.device("cuda", 0 if share else local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        nccl = use_cuda and not share
        dist.init_process_group("nccl" if nccl else "gloo", rank=rank, world_size=world,
                                **({"device_id": device} if nccl else {}))
    return rank, world, device


class Trainer:
    def __init__(self, args, rank=0, world=1, device=None, dataset=None):
        self.args, self.rank, self.world = args, rank, world
        self.device = device or torch.device("cpu")
        torch.manual_seed(args.seed)  # identical initial weights on every rank
        self.wrapper = NewMDGenWrapper(args).to(self.device)
        m = self.wrapper.model
        if self.device.type == "cuda":  # block forward + backward on the HIP kernels (train_hip.py)
            m.backend, m.train_backend = "hip", getattr(args, "train_backend", "hip")
            m.hip_dtype = getattr(args, "hip_dtype", "bf16")
        else:
            m.backend = "torch"
        torch.manual_seed(args.seed + 1 + 1000 * rank)  # independent (t, x0) draws per rank
        self.precision = resolve_precision(args.precision, self.device)
        self.scaler = torch.amp.GradScaler(self.device.type) if self.precision == torch.float16 else None
        # the graphed step (GraphedStep): ROCm device, HIP block stack, one micro-batch per step,
        # no loss scaler; gradients averaged by this class's flat all-reduce instead of DDP
        self.graph_mode = bool(self.device.type == "cuda" and int(getattr(args, "train_graph", 0))
                               and m.backend == "hip" and self.scaler is None and max(1, args.accumulate_grad) == 1)
        self._graphed = None
        self.model = self.wrapper.model
        # the conditioning on the ranks' global batch (cond_dist.py): its collectives must be capturable
        # in graph mode (RCCL; gloo's graphed path keeps every gradient in the flat all-reduce)
        self.replicated = set()
        if world > 1 and int(getattr(args, "cond_allgather", 1)):
            self.setup_cond_gather()
        if world > 1:  # rank 0's initial state on every rank (DDP's module-state sync; graph mode
            # has no DDP, and DDP skips the replicated conditioning's parameters)
            self.broadcast_state()
        if world > 1 and not self.graph_mode:
            self.model = DDP(self.wrapper.model, device_ids=[self.device.index] if self.device.type == "cuda" else None,
                             bucket_cap_mb=args.bucket_cap_mb, gradient_as_bucket_view=True, static_graph=True)
        self.optimizer = self.wrapper.configure_optimizers(capturable=self.graph_mode)
        self.epoch, self.global_step, self.skip_batches = 0, 0, 0
        self.valset = None
        if dataset is None:
            if args.synthetic:
                dataset = SyntheticMDDataset(args.num_frames, args.crop, size=args.synthetic_size, seed=args.seed)
            else:  # train.py:25-30: the reference's .npy trajectories (window draws per rank)
                dataset = MDGenDataset(args, split=args.train_split,
                                       rng=np.random.default_rng([args.seed, rank]))
                if not args.no_validate:
                    self.valset = dataset if args.overfit else MDGenDataset(
                        args, split=args.val_split, repeat=args.val_repeat,
                        rng=np.random.default_rng([args.seed, rank, 1]))
        self.dataset = dataset
        self.sampler = torch.utils.data.DistributedSampler(dataset, num_replicas=world, rank=rank, shuffle=True,
                                                           seed=args.seed, drop_last=True)
        # item loading is host work (memmap reads, geometry): worker processes overlap it with the
        # step (train.py:32-43); a worker's window draws continue the rank's generator
        nw = 0 if args.synthetic else int(getattr(args, "num_workers", 0) or 0)
        self.loader = torch.utils.data.DataLoader(dataset, batch_size=args.batch_size, sampler=self.sampler,
                                                  num_workers=nw, collate_fn=collate, drop_last=True,
                                                  worker_init_fn=_worker_init if nw else None,
                                                  persistent_workers=bool(nw))
        self.val_loader = None
        if self.valset is not None:
            vs = torch.utils.data.DistributedSampler(self.valset, num_replicas=world, rank=rank, shuffle=False)
            self.val_loader = torch.utils.data.DataLoader(self.valset, batch_size=args.batch_size, sampler=vs,
                                                          num_workers=0, collate_fn=collate)
        if args.ckpt:
            self.resume(args.ckpt)

    def setup_cond_gather(self):
        """Run the conditioning on the ranks' global batch (cond_dist.py) and take its parameters
        out of the gradient all-reduce.  Graph mode needs capturable collectives (RCCL).  The
        all-gathers get a process group of their own (a second communicator: they cannot queue
        behind the bucket all-reduces on the default group).  (Also called at world 1 for the
        RCCL capture rehearsal.)"""
        m = self.wrapper.model
        if self.graph_mode and not (dist.is_initialized() and dist.get_backend() == "nccl"):
            return False
        from .cond_dist import CondGather, replicated_params

        group = dist.new_group(list(range(self.world)), backend=dist.get_backend()) if dist.is_initialized() else None
        m._cond_gather = CondGather(self.world, self.rank, group=group)
        names = replicated_params(m)
        self.replicated = {id(p) for n, p in m.named_parameters() if n in names}
        if not self.graph_mode and self.world > 1:  # DDP leaves them alone (they arrive averaged)
            DDP._set_params_and_buffers_to_ignore_for_model(m, names)
        return True

    def cond_active(self):
        """Context of the Trainer's own training step: the replicated conditioning's collectives
        are issued only inside it (cond_dist.CondGather.active)."""
        return _CondActive(getattr(self.wrapper.model, "_cond_gather", None))

    # ------------------------------------------------------------------ replica state
    def _state_tensors(self, optimizer=False):
        m = self.wrapper.model
        ts = [p.data for p in m.parameters()] + [b for b in m.buffers()]
        if self.wrapper.ema is not None:
            ts += [v for v in self.wrapper.ema.params.values()]
        if optimizer:
            for st in self.optimizer.state.values():
                ts += [v for v in st.values() if torch.is_tensor(v)]
        return ts

    @torch.no_grad()
    def broadcast_state(self, optimizer=False):
        """Rank 0's parameters, buffers and EMA (and optimizer state) copied to every rank: one
        broadcast per dtype of the concatenated tensors (gloo: staged through the host)."""
        if self.world == 1 or not dist.is_initialized():
            return
        gloo = dist.get_backend() == "gloo"
        by_dtype = {}
        for t in self._state_tensors(optimizer):
            by_dtype.setdefault((t.dtype, t.device), []).append(t)
        for (dt, dev), ts in sorted(by_dtype.items(), key=lambda kv: str(kv[0])):
            flat = torch.cat([t.reshape(-1) for t in ts])
            buf = flat.cpu() if (gloo and flat.is_cuda) else flat
            dist.broadcast(buf, 0)
            if buf is not flat:
                flat.copy_(buf)
            off = 0
            for t in ts:
                t.copy_(flat[off:off + t.numel()].view_as(t))
                off += t.numel()

    @torch.no_grad()
    def check_replicas(self, resync=True):
        """Are the replicas identical?  Every rank all-gathers a fp64 checksum (sum and sum of
        squares) of each parameter and of the EMA; any difference across ranks is reported and,
        with ``resync``, repaired by re-broadcasting rank 0's parameters, EMA and optimizer state
        (the replicated conditioning is never all-reduced: a rank whose arithmetic differed would
        otherwise drift silently).  Returns the number of tensors that differed (0 = identical)."""
        if self.world == 1 or not dist.is_initialized():
            return 0
        ts = [t for t in self._state_tensors() if torch.is_floating_point(t)]
        sums = torch.stack([t.double().sum() for t in ts])
        sqs = torch.stack([t.double().square().sum() for t in ts])
        sig = torch.cat([sums, sqs])
        if dist.get_backend() == "gloo":
            sig = sig.cpu()
        allsig = [torch.empty_like(sig) for _ in range(self.world)]
        dist.all_gather(allsig, sig)
        diff = torch.zeros(len(ts), dtype=torch.bool)
        for other in allsig:
            d = (other != sig).cpu()
            diff |= d[:len(ts)] | d[len(ts):]
        # every rank decides alike: the per-rank results of the comparison are combined
        n = torch.tensor([int(diff.sum())], dtype=torch.int64, device=sig.device)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        n = int(n.item())
        if n and resync:
            if self.rank == 0:
                print(f"[train] replicas differ in {n} tensors: re-broadcasting rank 0's state", file=sys.stderr,
                      flush=True)
            self.broadcast_state(optimizer=True)
        return n

    # ------------------------------------------------------------------ checkpoint
    def resume(self, path):
        self._graphed = None  # static buffers / captured optimizer state are re-made from the restored state
        ck = load_checkpoint(path, map_location=self.device)
        self.wrapper.model.load_state_dict(model_state_dict(ck))
        if ck.get("optimizer_states"):
            self.optimizer.load_state_dict(ck["optimizer_states"][0])
        if self.scaler is not None and ck.get("MixedPrecision"):  # the loss-scale state (16-mixed)
            self.scaler.load_state_dict(ck["MixedPrecision"])
        if self.wrapper.ema is not None and "ema" in ck:
            self.wrapper.ema.load_state_dict(ck["ema"])
            self.wrapper.ema.to(self.device)
        loop = ck.get("loops", {}).get("fit_loop", {"epoch_complete": True, "batches_done": 0})
        self.global_step = int(ck["global_step"])
        if loop.get("epoch_complete", True):
            self.epoch, self.skip_batches = int(ck["epoch"]) + 1, 0
        else:  # saved mid-epoch (--max_steps): finish that epoch's remaining batches first
            self.epoch, self.skip_batches = int(ck["epoch"]), int(loop.get("batches_done", 0))

    def save(self, epoch_complete=True, batches_done=0):
        if self.rank != 0:
            return None
        path = os.path.join(self.args.model_dir, f"epoch={self.epoch}-step={self.global_step}.ckpt")
        save_checkpoint(path, self.wrapper, self.optimizer, self.epoch, self.global_step,
                        epoch_complete=epoch_complete, batches_done=batches_done,
                        grad_scaler=self.scaler.state_dict() if self.scaler is not None else None)
        return path

    # ------------------------------------------------------------------ one optimizer step
    def _to_device(self, batch):
        return {k: (v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in batch.items()}

    def step(self, micro_batches, log=True):
        """One optimizer step over ``len(micro_batches)`` accumulated micro-batches; returns the
        mean loss (rank-local) and the global grad norm before clipping.  In graph mode the step
        is a replay of GraphedStep's graphs with the batch copied into its static buffers."""
        if self.graph_mode and len(micro_batches) == 1:
            if self._graphed is None:
                self._graphed = GraphedStep(self, micro_batches[0])
            loss, gnorm = self._graphed.run(micro_batches[0], log=log)
            self.global_step += 1
            return loss, gnorm
        return self._eager_step(micro_batches, log=log)

    def allreduce_grads(self, flat=None):
        """Average the gradients over ranks (graph mode; DDP does it in the eager mode): one
        all-reduce of the flat fp32 buffer (RCCL over xGMI; gloo on CPU)."""
        if self.world == 1:
            return
        # (parameters averaged by the replicated conditioning stay out of the all-reduce)
        params = [p for p in self.wrapper.model.parameters() if p.requires_grad and id(p) not in self.replicated]
        own = flat is None
        if own:
            flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])
        if flat.is_cuda and dist.get_backend() == "gloo":
            # gloo (the world-2 on-one-GPU tests, MDG_SHARE_GPU) reduces host memory: stage the
            # buffer explicitly so no gloo worker thread touches the device between the graphs
            host = flat.cpu()
            dist.all_reduce(host)
            flat.copy_(host)
        else:
            dist.all_reduce(flat)
        flat.div_(self.world)
        if own:
            off = 0
            for p in params:
                n = p.numel()
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                p.grad.copy_(flat[off:off + n].view_as(p))
                off += n

    @torch.enable_grad()
    def _eager_step(self, micro_batches, log=True, update=True):
        a = self.args
        n = len(micro_batches)
        self.wrapper.train()
        losses = []
        autocast = (torch.autocast(self.device.type, dtype=self.precision) if self.precision is not None
                    else torch.autocast(self.device.type, enabled=False))
        for i, batch in enumerate(micro_batches):
            batch = self._to_device(batch)
            sync = (i == n - 1) or self.world == 1
            ctx = self.model.no_sync() if (not sync and isinstance(self.model, DDP)) else _null()
            with ctx, self.cond_active():
                with autocast:
                    out = self.wrapper.general_step(batch, "train", model=self.model, log=log)
                loss = out if log else out[0]
                scaled = loss / n
                (self.scaler.scale(scaled) if self.scaler is not None else scaled).backward()
            losses.append(loss.detach())
        if self.graph_mode:
            self.allreduce_grads()
        if self.scaler is not None:
            self.scaler.unscale_(self.optimizer)
        gnorm = torch.nn.utils.clip_grad_norm_(self.wrapper.model.parameters(), a.grad_clip) if a.grad_clip else None
        if self.scaler is not None:
            self.scaler.step(self.optimizer)
            self.scaler.update()
        else:
            self.optimizer.step()
        self.wrapper.on_before_zero_grad()
        self.optimizer.zero_grad(set_to_none=True)
        if update:
            self.global_step += 1
        return torch.stack(losses).mean(), gnorm

    def print_log(self, prefix="iter"):
        """wrapper.py:132-165."""
        w = self.wrapper
        log = {k: v for k, v in w._log.items() if k.startswith(prefix + "_")}
        log = gather_log(log, self.world)
        mean = get_log_mean(log)
        mean.update(epoch=self.epoch, trainer_step=self.global_step, iter_step=w.iter_step,
                    lr=self.optimizer.param_groups[0]["lr"])
        if self.rank == 0:
            print(json.dumps(mean), flush=True)
        for k in list(w._log):
            if k.startswith(prefix + "_"):
                del w._log[k]
        return mean

    @torch.no_grad()
    def validate(self):
        """wrapper.py:88-109: the GVP loss on the validation split (EMA weights when --ema), logged
        under ``val_`` and gathered over ranks at the end."""
        a, w = self.args, self.wrapper
        if w.ema is not None:
            w.load_ema_weights()
        w.eval()
        try:
            for bi, batch in enumerate(self.val_loader):
                if a.val_batches is not None and bi >= a.val_batches:
                    break
                w.general_step(self._to_device(batch), "val", model=w.model)
        finally:
            if w.ema is not None:
                w.restore_cached_weights()
            w.train()
        return self.print_log("val")

    def fit(self):
        a = self.args
        acc = max(1, a.accumulate_grad)
        while self.epoch < a.epochs:
            self.sampler.set_epoch(self.epoch)
            pending = []
            skip, self.skip_batches = self.skip_batches, 0
            for bi, batch in enumerate(self.loader):
                if a.train_batches is not None and bi >= a.train_batches:
                    break
                if bi < skip:  # resumed mid-epoch: these batches were consumed before the save
                    continue
                pending.append(batch)
                if len(pending) < acc:
                    continue
                self.step(pending)
                pending = []
                if self.global_step % a.print_freq == 0:
                    self.print_log("iter")
                    if self.world > 1 and int(getattr(a, "check_replicas", 1)):
                        self.check_replicas()
                if a.val_freq and self.val_loader is not None and (bi + 1) % a.val_freq == 0:
                    self.validate()  # Lightning's val_check_interval (train.py:52)
                if a.max_steps is not None and self.global_step >= a.max_steps:
                    self.save(epoch_complete=False, batches_done=bi + 1)
                    return
            self.print_log("train")
            if self.val_loader is not None and (self.epoch + 1) % max(1, a.val_epoch_freq) == 0:
                self.validate()
            if (self.epoch + 1) % a.ckpt_freq == 0:
                self.save()
            self.epoch += 1


class GraphedStep:
    r"""The optimizer step as hipGraph replays (Trainer.graph_mode).

    The eager step launches ~2 300 kernels from the host (the IPA / t-MLP / loss autograd, the
    per-layer weight packing, the HIP layer kernels): 33 ms of CPU against ~25 ms of GPU work per
    step on MI355X, so the device idles.  Here, after two warm-up steps on a side
    stream (autograd buffers, optimizer / EMA state, RoPE tables; the parameters, optimizer
    state and EMA are restored afterwards, so warm-up trains nothing), one capture records
      world 1: prep_batch -> GVP loss -> backward -> grad clip -> Adam (capturable) -> EMA
    and each step is: copy the batch into the static buffers, replay.  With world > 1 over RCCL
    (``--allreduce_overlap 1``, the default) the gradient all-reduce is captured too: the
    parameters' gradients are bucketed in the order backward completes them, and each bucket's
    RCCL all-reduce runs on a side-stream branch of the same graph as soon as its last gradient
    lands, overlapped with the rest of backward (grad_buckets.BucketedAllReduce, DDP's schedule
    inside the capture):
      prep_batch -> loss -> backward  -> join -> clip -> Adam -> EMA
                              \_ bucket k: cat -> all_reduce / world (side stream) _/
    Otherwise (gloo, which cannot be captured, or ``--allreduce_overlap 0``) the step is two
    graphs around an eager all-reduce of the flat gradient buffer (graph 1 ends by packing the
    gradients into it; graph 2's clip / Adam read them through views of it):
      graph 1: prep_batch -> loss -> backward -> cat(grads) | all_reduce(flat) / world |
      graph 2: clip -> Adam -> EMA.
    The (t, x0) draws come from the CUDA generator's graph-safe philox offsets, so every replay
    draws fresh noise, as the eager step does."""

    def __init__(self, tr, batch, warmup=2):
        self.tr = tr
        dev = tr.device
        self.static = {k: (v.to(dev).clone() if torch.is_tensor(v) else v) for k, v in batch.items()}
        self.params = [p for p in tr.wrapper.model.parameters() if p.requires_grad]
        # force_allreduce: run the reduction machinery at world 1 (a world-1 RCCL group: the GPU
        # tests' capture check on a one-GPU box)
        self.split = tr.world > 1 or bool(getattr(tr, "force_allreduce", False))
        self.overlap = bool(self.split and int(getattr(tr.args, "allreduce_overlap", 1)) and dist.is_initialized()
                            and dist.get_backend() == "nccl")
        self.reducer = None
        model = tr.wrapper.model
        # TPS: the relative frames come from a host eigh (relative_tensor7), which a capture
        # cannot contain; they are computed here per step and read from a static buffer
        self.rel7 = None
        if getattr(model, "tps", False):
            B, L = self.static["trans"].shape[0], self.static["trans"].shape[2]
            self.rel7 = torch.empty(2, B, L, 7, device=dev)
            self._stage_rel7(self.static)
            model._rel7_feed = self.rel7
        try:
            self._build(tr, model, dev, warmup)
        finally:
            model._rel7_feed = None

    def _stage_rel7(self, batch):
        from .model.latent_model import relative_tensor7

        rots, trans = batch["rots"].float(), batch["trans"].float()
        r0, t0, r1, t1 = rots[:, 0], trans[:, 0], rots[:, -1], trans[:, -1]
        self.rel7.copy_(torch.stack([relative_tensor7(r0, t0, r1, t1), relative_tensor7(r1, t1, r0, t0)]),
                        non_blocking=False)

    def _build(self, tr, model, dev, warmup):
        # warm-up trains nothing: snapshot everything it updates and put it back afterwards.
        # Optimizer state that exists before warm-up (a --ckpt resume) is restored as loaded;
        # state warm-up itself creates (a fresh run) is zeroed, i.e. "no step taken yet".
        snap = [p.detach().clone() for p in model.parameters()]
        opt_snap = {id(p): {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                    for p, st in tr.optimizer.state.items()}
        ema = tr.wrapper.ema
        ema_snap = {k: v.detach().clone() for k, v in ema.params.items()} if ema is not None else None
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        order, unhook = record_grad_order(self.params)  # the order backward completes gradients
        with torch.cuda.stream(side):
            for w in range(warmup):
                tr._eager_step([self.static], log=False, update=False)
                if w == 0:
                    unhook()
        unhook()
        if self.overlap:
            # parameters the replicated conditioning averages already (cond_dist.py) are not bucketed
            order = [i for i in order if id(self.params[i]) not in tr.replicated]
            self.reducer = BucketedAllReduce(self.params, order, int(tr.args.bucket_cap_mb * 2 ** 20), tr.world)
            with torch.cuda.stream(side):  # the communicator exists before the capture
                dist.all_reduce(torch.zeros(1, device=dev))
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.no_grad():
            for p, v in zip(model.parameters(), snap):
                p.copy_(v)
            for p, st in tr.optimizer.state.items():
                old = opt_snap.get(id(p))
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        continue
                    if old is not None and torch.is_tensor(old.get(k)):
                        v.copy_(old[k])  # in place: the capture below reads these very tensors
                    else:
                        v.zero_()
            if ema is not None:
                for k, v in ema_snap.items():
                    ema.params[k].copy_(v)
        tr.optimizer.zero_grad(set_to_none=True)
        # clip + Adam on the library's two-pass update (optim_hip.FusedClipAdam) instead of torch's
        # foreach norm / multiplies / fused Adam launches; MDG_TRAIN_FUSED_OPT=0 keeps torch's (A/B)
        from .optim_hip import FusedClipAdam
        self.fused_opt = None
        if os.environ.get("MDG_TRAIN_FUSED_OPT", "1") != "0" and FusedClipAdam.supported(tr.optimizer):
            self.fused_opt = FusedClipAdam(tr.optimizer, self.params, tr.args.grad_clip)
        # the split path's flat buffer holds the gradients the all-reduce averages: the replicated
        # conditioning's arrive averaged already and keep their own (graph-1) tensors
        self.red_params = [p for p in self.params if id(p) not in tr.replicated]
        n = sum(p.numel() for p in self.red_params)
        self.flat = self.reducer.flat if self.overlap else (torch.empty(n, device=dev) if self.split else None)
        # DP markers (bench.py's train_dp line): device timestamps inside the capture (mdg_stamp;
        # ROCm's torch refuses external timing events in a graph) at the step's start and
        # backward's end on the main stream, and after the last bucket's all-reduce on the side
        # stream; the last distance is the all-reduce time backward did not hide
        self.markers = None
        if self.overlap and getattr(tr, "dp_markers", False):
            from . import _lib

            khz = ctypes.c_int32()
            _lib.check(_lib.load().mdg_wall_clock_khz(ctypes.byref(khz)), "mdg_wall_clock_khz")
            self.clock_khz = khz.value
            self.markers = torch.zeros(3, dtype=torch.int64, device=dev)
            self.reducer.markers = self.stamp
        if self.fused_opt is not None:
            self.fused_opt.reserve()  # its tables outside the graph's private pool (optim_hip)
        self.g1 = torch.cuda.CUDAGraph()
        # thread-local capture: a process group's watchdog thread polls its events during the
        # capture (global mode would fail that query and abort the process)
        with torch.cuda.graph(self.g1, capture_error_mode="thread_local"):
            if self.overlap:
                self.reducer.attach()
            if self.markers is not None:
                self.stamp(0, torch.cuda.current_stream())
            self.loss, self.losses, self.t = self._fwd_bwd()
            if self.overlap:  # one graph: the bucket all-reduces are branches of it
                if self.markers is not None:
                    self.stamp(1, torch.cuda.current_stream())
                self.reducer.finish()
                self.gnorm = self._update()
            elif self.split:
                self.grads_g1 = [p.grad for p in self.params]  # graph-1 memory, kept referenced
                torch.cat([p.grad.reshape(-1) for p in self.red_params], out=self.flat)
            else:
                self.gnorm = self._update()
        if self.fused_opt is not None and not (self.split and not self.overlap):
            self.fused_opt.finish_capture()
        if self.split and not self.overlap:
            off = 0
            for p in self.red_params:  # graph 2 reads the averaged gradients in place
                p.grad = self.flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            self.g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g2, capture_error_mode="thread_local"):
                self.gnorm = self._update()
            if self.fused_opt is not None:
                self.fused_opt.finish_capture()

    def _fwd_bwd(self):
        tr = self.tr
        tr.wrapper.train()
        autocast = (torch.autocast("cuda", dtype=tr.precision) if tr.precision is not None
                    else torch.autocast("cuda", enabled=False))
        with torch.enable_grad(), tr.cond_active():
            with autocast:
                loss, losses, t = tr.wrapper.general_step(self.static, "train", model=tr.wrapper.model, log=False)
            loss.backward()
        return loss.detach(), losses.detach(), t.detach()

    def _update(self):
        tr = self.tr
        if self.fused_opt is not None:
            gnorm = self.fused_opt.step(capturing=True)
            tr.wrapper.on_before_zero_grad()
            return gnorm if tr.args.grad_clip else None
        gnorm = torch.nn.utils.clip_grad_norm_(self.params, tr.args.grad_clip) if tr.args.grad_clip else None
        tr.optimizer.step()
        tr.wrapper.on_before_zero_grad()
        return gnorm

    def stamp(self, slot, stream):
        from . import _lib

        _lib.check(_lib.load().mdg_stamp(self.markers.data_ptr(), slot, stream.cuda_stream), "mdg_stamp")

    def dp_times_ms(self):
        """(forward + backward, all-reduce exposed after backward's end) of the last replay in ms,
        from the in-graph markers (None without them)."""
        if self.markers is None:
            return None
        torch.cuda.synchronize()
        v = [int(x) for x in self.markers.cpu().tolist()]
        return (v[1] - v[0]) / self.clock_khz, max(0.0, (v[2] - v[1]) / self.clock_khz)

    def run(self, batch, log=True):
        for k, v in batch.items():
            if torch.is_tensor(v):
                self.static[k].copy_(v, non_blocking=True)
        if self.rel7 is not None:
            self._stage_rel7(batch)
        self.g1.replay()
        if self.split and not self.overlap:
            self.tr.allreduce_grads(self.flat)
            self.g2.replay()
        model = self.tr.wrapper.model  # the replayed Adam bumps no version counters: tell the engine
        model._weights_gen = getattr(model, "_weights_gen", 0) + 1
        if log:
            w = self.tr.wrapper
            w.stage = "train"
            w.iter_step += 1
            w.log("loss", self.losses)
            w.log("time", self.t)
        return self.loss, self.gnorm


# Lightning precision strings the reference passes to pl.Trainer(precision=...) (train.py:52)
_PRECISIONS = {"32-true": None, "32": None, "bf16-mixed": torch.bfloat16, "16-mixed": torch.float16}


def resolve_precision(precision, device):
    """autocast dtype for --precision (None = full fp32).  'bf16-true' / '16-true' (weights
    held in half precision) and unknown strings are refused instead of silently training fp32."""
    key = str(precision)
    if key not in _PRECISIONS:
        raise NotImplementedError(f"--precision {precision!r}: supported are {sorted(_PRECISIONS)}")
    dt = _PRECISIONS[key]
    if dt == torch.float16 and device.type != "cuda":
        raise NotImplementedError("--precision 16-mixed needs a GPU (fp16 autocast + GradScaler)")
    return dt


def _worker_init(worker_id):
    """A DataLoader worker's dataset copy draws from its own stream of the rank's generator."""
    info = torch.utils.data.get_worker_info()
    ds = info.dataset
    if hasattr(ds, "rng"):
        ds.rng = np.random.default_rng([int(ds.rng.integers(2 ** 31)), worker_id])


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class _CondActive:
    def __init__(self, cg):
        self.cg, self.prev = cg, False

    def __enter__(self):
        if self.cg is not None:
            self.prev, self.cg.active = self.cg.active, True
        return self

    def __exit__(self, *exc):
        if self.cg is not None:
            self.cg.active = self.prev
        return False


def main(argv=None):
    args = parse_train_args(argv)
    rank, world, device = setup_distributed()
    if device.type == "cuda":
        torch.set_float32_matmul_precision("medium")  # train.py:13
    tr = Trainer(args, rank, world, device)
    t0 = time.time()
    if args.validate:  # train.py:74-75: trainer.validate(model, ckpt_path=args.ckpt), no training
        if tr.val_loader is None:
            raise SystemExit("--validate needs a validation split (--val_split, not --no_validate / --synthetic)")
        tr.validate()
    else:
        tr.fit()
    if rank == 0:
        print(json.dumps({"done": True, "steps": tr.global_step, "wall_s": round(time.time() - t0, 2)}), flush=True)
    if world > 1:
        dist.barrier()
        # the captured step's graph holds RCCL collectives: release it before the communicator
        tr._graphed = None
        import gc

        gc.collect()
        if device.type == "cuda":
            torch.cuda.synchronize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1:])
