"""Bucketed gradient all-reduce overlapped with backward, usable inside a hipGraph capture.

The reference averages gradients with Lightning's DDP (``/root/reference/src/train.py:46-60``):
bucketed all-reduces that NCCL runs while backward is still producing the earlier layers'
gradients.  DDP's reducer cannot be captured (it synchronises with the host between
iterations), and the graphed optimizer step (train.GraphedStep) is what removes the eager
step's host-launch bound, so this class does DDP's job inside the capture:

* the parameters are laid out in a flat fp32 buffer in the order backward COMPLETES their
  gradients (recorded once from post-accumulate-grad hooks during warm-up), cut into buckets
  of ``cap_bytes``, so each bucket is one contiguous slice that becomes final at one moment;
* a post-accumulate-grad hook counts a bucket's parameters down; when the last one lands, the
  bucket's gradients are packed into its slice (one foreach copy on the producing stream; every
  gradient 16-B aligned in the buffer), an event
  forks a side stream, and the slice's all-reduce (RCCL over xGMI) + 1/world scale run there
  while backward continues on the main stream;
* ``finish()`` joins the side stream (graph-capture legal: event record / wait) and points
  every ``p.grad`` at its slice, so clip / Adam / EMA read the averaged values in place.

Rank agreement (DDP's rules, which this class must keep because the collectives are matched by
sequence): every rank builds its layout from RANK 0's recorded order (broadcast at construction)
and checks by an all-gather that all ranks hold the same parameter set, bucket sizes and the same
set of gradients reached by backward; and buckets are reduced strictly in layout order — a bucket
that completes early waits for its predecessors — so the collectives' sequence is the same on
every rank whatever order the local hooks fire in.  A hook that fires twice in one backward
(a reentrant re-run) is an error, not a silent early launch.

Inside a capture the collectives become graph nodes on the side stream's branch, interleaved
with the backward kernels (the replay keeps the overlap).  On CPU (gloo) the same object runs
eagerly with ``async_op`` all-reduces, which is how the world-2 CPU tests exercise it.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_MARK = os.environ.get("MDG_BUCKET_MARK") == "1"


def record_grad_order(params):
    """Register hooks that log the order in which backward completes each parameter's
    gradient; returns (order list of indices, remove())."""
    order, handles = [], []
    for i, p in enumerate(params):
        handles.append(p.register_post_accumulate_grad_hook(lambda _p, i=i: order.append(i)))

    def remove():
        for h in handles:
            h.remove()

    return order, remove


def agree_order(params, order, world, group=None):
    """Rank 0's completion order, broadcast to every rank, after checking that all ranks hold the
    same parameter shapes and reached the same set of gradients (raises RuntimeError otherwise).
    On world 1 (or without an initialised group) the local order is returned unchanged."""
    seen = list(dict.fromkeys(order))
    if world <= 1 or not dist.is_initialized():
        return seen
    dev = params[0].device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    n = len(params)
    # per-rank signature: parameter count, total elements, a position-weighted numel checksum,
    # then per parameter a code of its SHAPE (rank and every extent), then the reached set
    reached = torch.zeros(n, dtype=torch.int64)
    reached[seen] = 1
    numels = torch.tensor([p.numel() for p in params], dtype=torch.int64)
    shapes = torch.tensor([_shape_code(p.shape) for p in params], dtype=torch.int64)
    head = torch.tensor([n, int(numels.sum()), int((numels * torch.arange(1, n + 1)).sum())])
    sig = torch.cat([head, shapes, reached])
    sig = sig.to(dev)
    allsig = [torch.empty_like(sig) for _ in range(world)]
    dist.all_gather(allsig, sig, group=group)
    for r, other in enumerate(allsig):
        if not torch.equal(other, sig):
            o, mine = other.cpu(), sig.cpu()
            if not torch.equal(o[:3], mine[:3]):
                raise RuntimeError(f"gradient buckets: rank {r} holds different parameters (count / sizes "
                                   f"{o[:3].tolist()} vs {mine[:3].tolist()})")
            bad = (o[3:3 + n] != mine[3:3 + n]).nonzero().flatten().tolist()
            if bad:
                raise RuntimeError(f"gradient buckets: rank {r} holds parameters of different shapes "
                                   f"(parameters {bad[:8]}{'...' if len(bad) > 8 else ''})")
            diff = (o[3 + n:] != mine[3 + n:]).nonzero().flatten().tolist()
            raise RuntimeError(f"gradient buckets: rank {r} reached a different set of gradients in backward "
                               f"(parameters {diff[:8]}{'...' if len(diff) > 8 else ''} differ)")
    buf = torch.full((n,), -1, dtype=torch.int64)
    buf[:len(seen)] = torch.tensor(seen, dtype=torch.int64)
    buf = buf.to(dev)
    dist.broadcast(buf, 0, group=group)
    return [int(i) for i in buf.cpu().tolist() if i >= 0]


def _shape_code(shape):
    """An int63 code of a shape (its rank and extents, order-sensitive): equal shapes give equal
    codes on every rank; (3, 4) and (4, 3), or (12,) and (3, 4), do not collide."""
    h = len(shape) + 1
    for d in shape:
        h = (h * 1000003 + int(d) + 1) % (2 ** 61 - 1)
    return h


class BucketedAllReduce:
    """tail_bytes: the LAST bucket (the gradients backward completes last, which nothing overlaps)
    is cut further into pieces of at most this size (default cap / 4), so all but its final piece
    leave while backward is still running."""

    def __init__(self, params, order, cap_bytes, world, group=None, tail_bytes=None):
        self.params = list(params)
        self.world, self.group = world, group
        dev = self.params[0].device
        # parameters that backward never reached keep grad None (the optimizer skips them).
        # Layout from rank 0's order on every rank (DDP syncs its rebuilt buckets the same way)
        seen = agree_order(self.params, order, world, group)
        self.buckets, cur, size = [], [], 0
        for i in seen:
            nb = self.params[i].numel() * 4
            if cur and size + nb > cap_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += nb
        if cur:
            self.buckets.append(cur)
        tail = cap_bytes // 4 if tail_bytes is None else tail_bytes
        if self.buckets and tail > 0:
            last, pieces, cur, size = self.buckets.pop(), [], [], 0
            for i in last:
                nb = self.params[i].numel() * 4
                if cur and size + nb > tail:
                    pieces.append(cur)
                    cur, size = [], 0
                cur.append(i)
                size += nb
            self.buckets += pieces + [cur]
        # every gradient starts on a 16-B boundary (the library optimizer's float4 path); the pad
        # elements stay zero and are reduced along with the bucket
        pad4 = lambda v: (v + 3) // 4 * 4  # noqa: E731
        n = sum(pad4(self.params[i].numel()) for b in self.buckets for i in b)
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        self.slices, self.views, self.bucket_of, off = [], {}, {}, 0
        for bi, b in enumerate(self.buckets):
            start = off
            for i in b:
                p = self.params[i]
                self.views[i] = self.flat[off:off + p.numel()].view_as(p)
                self.bucket_of[i] = bi
                off += pad4(p.numel())
            self.slices.append(self.flat[start:off])
        self.cuda = dev.type == "cuda"
        self.side = torch.cuda.Stream(device=dev) if self.cuda else None
        self._handles = []
        self.markers = None
        self.log = None  # a list: (op, numel, group) of every collective issued (the CPU tests)
        self.launch_log = []  # (bucket, number of hooks fired so far) per launch: the overlap record

    # ---------------------------------------------------------------- per step
    def attach(self):
        """Arm the hooks for one backward pass."""
        self.detach()
        self._pending = [len(b) for b in self.buckets]
        self._works, self._fired = [], 0
        self._done, self._next = set(), 0  # fired parameter indices; next bucket to reduce
        self.launch_log = []
        for bi, b in enumerate(self.buckets):
            for i in b:
                self._handles.append(self.params[i].register_post_accumulate_grad_hook(
                    lambda _p, i=i: self._ready(i)))

    def detach(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def _ready(self, i):
        if i in self._done:
            raise RuntimeError(f"gradient buckets: parameter {i}'s gradient hook fired twice in one backward "
                               "(a reentrant re-run would reduce the bucket before its final gradients)")
        if i not in self.bucket_of:
            raise RuntimeError(f"gradient buckets: parameter {i} produced a gradient that warm-up never saw")
        self._done.add(i)
        self._fired += 1
        self._pending[self.bucket_of[i]] -= 1
        # reduce in layout order: the collectives' sequence must be the same on every rank
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        self.launch_log.append((bi, self._fired))
        sl = self.slices[bi]
        b = self.buckets[bi]
        torch._foreach_copy_([self.views[i] for i in b], [self.params[i].grad for i in b])
        if self.log is not None:
            self.log.append(("all_reduce", int(sl.numel()), "buckets"))
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(sl.device))
            self.side.wait_event(ev)
            with torch.cuda.stream(self.side):
                if _MARK:  # profiling: a one-kernel marker per bucket in the trace (tools/rccl_overlap_trace.py)
                    torch.cuda._sleep(1)
                dist.all_reduce(sl, group=self.group)
                if self.world > 1:
                    sl.div_(self.world)
        else:
            self._works.append((dist.all_reduce(sl, group=self.group, async_op=True), sl))

    def finish(self):
        """Join the reductions and point every gradient at its averaged slice."""
        if any(self._pending):
            missing = [bi for bi, n in enumerate(self._pending) if n]
            raise RuntimeError(f"gradient buckets {missing} never completed: backward skipped parameters "
                               "that produced gradients in warm-up")
        if self.cuda:
            if self.markers is not None:  # (train.GraphedStep's DP markers) the side branch is done
                self.markers(2, self.side)
            torch.cuda.current_stream(self.flat.device).wait_stream(self.side)
        else:
            for w, sl in self._works:
                w.wait()
                if self.world > 1:
                    sl.div_(self.world)
        for i, v in self.views.items():
            self.params[i].grad = v
        self.detach()
