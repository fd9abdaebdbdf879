"""Data-parallel training without an all-reduce for the conditioning's parameters.

In the reference's DDP step (``/root/reference/src/train.py:46-60``, Lightning's implicit DDP)
every parameter's gradient is all-reduced after backward.  The conditioning path of
``LatentMDGenModel`` — the t-embedding MLP, every adaLN linear and the IPA prepend
(latent_model.py:179-214, 252, 415-418; ~22 M of the 34 M parameters) — receives its gradients
at the very END of backward (its outputs enter the first block and the token embedding), so
its ~90 MB of fp32 gradients leave backward with nothing left to overlap them.  Yet the work is
tiny and depends on few inputs per sample: t [B], the first frame's mask, frames and amino
acids [B, L] (TPS: also the last frame's frames and the two relative 7-vectors of the
reference's ``a.invert().compose(b).to_tensor_7()``, latent_model.py:197-211).

``CondGather`` runs that path on the GLOBAL batch on every rank instead:
  forward   all-gather the ranks' conditioning inputs (one packed fp32 tensor per rank:
            [B, 1 + 14 L] sim, [B, 1 + 40 L] TPS), compute c, every adaLN row and the IPA
            prepend for all W*B samples, and keep the local rows (``local``);
  backward  ``local``'s backward all-gathers the ranks' gradients of those rows (B x ~50 C
            floats per rank, ~0.6 MB at B = 8) and scales them by 1/W, so the conditioning's
            backward on the global batch produces (1/W) sum_r dL_r/dtheta — exactly DDP's
            average — on every rank, with no all-reduce of its weights.
The trainer leaves these parameters out of the gradient buckets (``replicated_params``).

Rank safety:
  * the all-gathers run on their OWN process group (a second RCCL communicator, made by
    ``Trainer.setup_cond_gather``), so they never queue behind — or interleave with — the
    gradient buckets' all-reduces, which the graphed step issues from a side stream on the
    default group;
  * they are issued only while ``active`` is set, which the Trainer does around its own
    training step: a grad-enabled forward that runs on some ranks only (an eval()-mode prior
    used for guidance, rank-0 diagnostics) takes the local conditioning path and issues no
    collective the other ranks would have to match;
  * replicas stay identical only if the conditioning's arithmetic is bit-identical on every
    rank; ``Trainer.check_replicas`` compares a checksum of every parameter across ranks.
The collectives are plain torch.distributed calls: RCCL (captured into the graphed step) or gloo
(eager, the CPU tests).  ``log``, when a list, records (op, numel, group) of every collective
issued (the CPU tests compare the sequences of the ranks)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def replicated_params(model):
    """Names of the parameters that only the conditioning path reaches (their gradients come out
    averaged over the ranks by CondGather; no bucket all-reduce).  TPS: also the two relative-
    frame embeddings latent_to_emb_f / _r (latent_model.py:200-201)."""
    names = []
    for n, _ in model.named_parameters():
        if (n.startswith("t_embedder.") or n.startswith("aatype_to_emb.") or n.startswith("ipa_layers.")
                or ".adaLN_modulation." in n or n.startswith("emb_to_latent.adaLN_modulation.")
                or n.startswith("latent_to_emb_f.") or n.startswith("latent_to_emb_r.")):
            names.append(n)
    return names


class _LocalRows(torch.autograd.Function):
    """rows [rank*B, (rank+1)*B) of a global-batch tensor; backward: the ranks' row gradients
    all-gathered (in rank order) and scaled by 1/W."""

    @staticmethod
    def forward(ctx, xg, cg):
        ctx.cg = cg
        B = xg.shape[0] // cg.world
        return xg[cg.rank * B:(cg.rank + 1) * B].clone()

    @staticmethod
    def backward(ctx, g):
        cg = ctx.cg
        out = cg.all_gather(g.contiguous())
        return out.mul_(1.0 / cg.world), None


class CondGather:
    def __init__(self, world, rank, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.active = False  # set by the Trainer around its training step only
        self.log = None

    def all_gather(self, x):
        """[B, ...] -> [W*B, ...] in rank order (RCCL: one all_gather_into_tensor; gloo: via the
        host for device tensors)."""
        if self.log is not None:
            self.log.append(("all_gather", int(x.numel()), "cond"))
        out = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, x, group=self.group)
            return out
        xh = x.detach().cpu()
        parts = [torch.empty_like(xh) for _ in range(self.world)]
        dist.all_gather(parts, xh, group=self.group)
        out.copy_(torch.cat(parts))
        return out

    def gather_inputs(self, t, mask_b, rots, trans, aatype, tps=None):
        """The ranks' conditioning inputs as global-batch tensors (no gradient flows to them).
        tps: (end rots [B,L,3,3], end trans [B,L,3], rel7 [2,B,L,7]) of the TPS model."""
        B, L = mask_b.shape
        dev = mask_b.device
        aa = aatype.float() if aatype is not None else torch.zeros(B, L, device=dev)
        cols = [t.reshape(B, 1).float(), mask_b.float(), rots.reshape(B, 9 * L).float(),
                trans.reshape(B, 3 * L).float(), aa.reshape(B, L)]
        if tps is not None:
            erots, etrans, rel7 = tps
            cols += [erots.reshape(B, 9 * L).float(), etrans.reshape(B, 3 * L).float(),
                     rel7.float().permute(1, 0, 2, 3).reshape(B, 14 * L)]
        g = self.all_gather(torch.cat(cols, -1).detach())
        W = g.shape[0]
        t_g = g[:, 0].to(t.dtype)
        mask_g = g[:, 1:1 + L]
        rots_g = g[:, 1 + L:1 + 10 * L].reshape(W, L, 3, 3)
        trans_g = g[:, 1 + 10 * L:1 + 13 * L].reshape(W, L, 3)
        aa_g = g[:, 1 + 13 * L:1 + 14 * L].round().to(torch.int64) if aatype is not None else None
        if tps is None:
            return t_g, mask_g, rots_g, trans_g, aa_g
        o = 1 + 14 * L
        erots_g = g[:, o:o + 9 * L].reshape(W, L, 3, 3)
        etrans_g = g[:, o + 9 * L:o + 12 * L].reshape(W, L, 3)
        rel_g = g[:, o + 12 * L:o + 26 * L].reshape(W, 2, L, 7).permute(1, 0, 2, 3).contiguous()
        return t_g, mask_g, rots_g, trans_g, aa_g, (erots_g, etrans_g, rel_g)

    def local(self, xg):
        return _LocalRows.apply(xg, self)
