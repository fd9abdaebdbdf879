"""Training on the GPU: the eager autograd step runs on the device, and after optimizer steps
the HIP inference path (which packs the weights into its own layout) follows the updated
parameters — its forward equals the eager forward of the trained module (f32 tolerance)."""
import numpy as np
import pytest
import torch

from tests.conftest import build_model, load_golden, model_args
from tests.test_train import _args, _batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def test_train_steps_then_hip_inference_tracks_weights():
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4"])
    tr = Trainer(a, device=torch.device("cuda"))
    b = _batch(a, B=2)
    losses = [tr.step([b])[0].item() for _ in range(4)]
    assert np.isfinite(losses).all()
    w = tr.wrapper
    m = w.model.eval()
    m.hip_dtype = "f32"
    prep = w.prep_batch({k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()})
    x = torch.randn_like(prep["latents"])
    t = torch.full((x.shape[0],), 0.3, device="cuda")
    with torch.no_grad():
        m.backend = "hip"
        v_hip = m(x, t, **prep["model_kwargs"]).clone()
        tr.step([b])  # weights change: the engine must re-pack
        m.eval()
        v_hip2 = m(x, t, **prep["model_kwargs"])
        m.backend = "torch"
        v_ref2 = m(x, t, **prep["model_kwargs"])
    assert not torch.equal(v_hip, v_hip2)
    err = (v_hip2 - v_ref2).abs().max().item()
    assert err <= 1e-3 * max(1.0, v_ref2.abs().max().item()), err


def _loss_inputs(d, device):
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    f = lambda k: torch.from_numpy(d["in_" + k]).to(device)  # noqa: E731
    kw = dict(mask=f("mask"), start_frames=Rigid(Rotation(rot_mats=f("rots")), f("trans")), x_cond=f("x_cond"),
              x_cond_mask=f("x_cond_mask"), aatype=f("aatype"))
    return f("x"), f("x0"), f("t_loss"), f("loss_mask"), kw


def _oracle_loss_grads(d, cfg):
    """Oracle GVP loss (batch mean) and d(loss)/d(param) by autograd on the CPU restatement."""
    from oracle import mdgen_oracle as O

    _, c = model_args(cfg)
    P = O.seeded_params(c, cfg["weights_seed"])
    for v in P.values():
        v.requires_grad_(True)
    kw = O.kwargs_from_npz(d)
    f = lambda k: torch.from_numpy(d["in_" + k])  # noqa: E731
    loss, v = O.gvp_training_loss(P, c, f("x"), f("x0"), f("t_loss"), f("loss_mask"), **kw)
    loss.mean().backward()
    return loss.detach(), v.detach(), {k: p.grad for k, p in P.items()}


def _model_loss(m, d, device):
    """Transport's own GVP plan + mean_flat with the fixture's injected (t, x0)."""
    from mdgen_finetune_amd.transport import create_transport
    from mdgen_finetune_amd.transport.transport import mean_flat

    x1, x0, t, lm, kw = _loss_inputs(d, device)
    tr = create_transport(m.args, "GVP", "velocity")
    t, xt, ut = tr.path_sampler.plan(t, x0, x1)
    v = m(xt, t, **kw)
    loss = mean_flat((v - ut) ** 2, lm)
    return loss, v


# grad tolerance per train path: ||g - g_ref|| / ||g_ref|| per parameter (and for the loss)
TRAIN_TOL = {"torch": (1e-5, 1e-4), "hip-f32": (1e-5, 1e-4), "hip-bf16": (1e-3, 2e-2)}  # bf16 worst 9.1e-3


def _log_train(rec):
    import json
    import os

    path = os.environ.get("MDG_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


@pytest.mark.parametrize("path", ["torch", "hip-f32", "hip-bf16"])
def test_gvp_loss_and_grads_on_gpu_match_oracle(path):
    """Config 3's differentiated step on the GPU (the training forward + backward the Trainer
    runs) against tests/golden/small_loss.npz (loss, prediction: the reference's own outputs)
    and the oracle's autograd gradients for every parameter.
      torch     eager autograd on the device;
      hip-f32   every block's forward + backward in libmdgen_hip.so with exact-f32 operands;
      hip-bf16  the same with bf16 GEMM / attention operands (the training default).
    Tolerances (TRAIN_TOL): loss rel and per-parameter grad ||d||/||ref||."""
    d, cfg = load_golden("small_loss")
    m, _ = build_model(cfg, "cuda")
    m.train()
    if path == "torch":
        m.backend = "torch"
    else:
        m.hip_dtype = path.split("-")[1]
    loss_tol, grad_tol = TRAIN_TOL[path]
    loss, v = _model_loss(m, d, "cuda")
    lrel = float(np.abs(loss.detach().cpu().numpy() - d["out_loss"]).max() / np.abs(d["out_loss"]).max())
    prel = float(np.linalg.norm(v.detach().cpu().numpy() - d["out_pred"]) / np.linalg.norm(d["out_pred"]))
    loss.mean().backward()
    _, _, g_ref = _oracle_loss_grads(d, cfg)
    names = dict(m.named_parameters())
    worst, checked = (0.0, None), 0
    for k, gr in g_ref.items():
        if gr is None or k not in names:
            continue
        g = names[k].grad
        assert g is not None, k
        if float(gr.norm()) < 1e-8:
            continue
        rel = float((g.detach().float().cpu() - gr).norm()) / float(gr.norm())
        worst = max(worst, (rel, k))
        checked += 1
    _log_train({"test": "gvp_loss_grads", "path": path, "loss_rel": lrel, "pred_rel": prel, "worst_grad_rel": worst[0],
                "worst_param": worst[1]})
    assert lrel <= loss_tol, lrel
    assert worst[0] <= grad_tol, worst
    assert checked > 100


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("T,L,n_pad", [(8, 4, 0), (70, 4, 1), (6, 6, 2), (5, 16, 3)])
def test_hip_layer_backward_matches_eager_autograd(dtype, T, L, n_pad):
    """One LatentMDGenLayer through the HIP training Function vs eager autograd of the same
    module on the same inputs (random upstream gradient): d h_in, d mods (adaLN) and every
    parameter gradient.  Covers the L = 4 quad spatial kernels, a query tail (T = 70), padded
    residues (key-padding), the generic spatial path (L = 6) and the L >= 16 route (spatial
    attention on the temporal MFMA kernel).  f32: rel <= 1e-4; bf16: rel <= 4.5e-2 (2x the worst
    observed, 2.24e-2: profiles/r03_parity_train.jsonl)."""
    _layer_vs_eager(dtype, T, L, n_pad, 64, 4, "layer_bwd")


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("C,H,T,L,n_pad", [(256, 8, 8, 4, 0), (256, 8, 70, 4, 1), (384, 8, 9, 6, 2),
                                           (384, 8, 5, 16, 3), (256, 8, 5, 16, 3), (384, 12, 5, 16, 3),
                                           (384, 8, 300, 4, 1)])
def test_hip_layer_backward_wide_heads(dtype, C, H, T, L, n_pad):
    """The same at head_dim 32..63 (ABI 23; reference mha.py:96-102 takes any embed_dim //
    num_heads): D = 32 (--embed_dim 256 --mha_heads 8; the quad spatial forward, the generic
    spatial backward), D = 48 at L = 6 and at T = 300 (3 temporal chunks) and at L = 16
    (spatial attention on the temporal kernels).  64-column planes, the scalar attention-backward
    kernels.  Bounds as above."""
    _layer_vs_eager(dtype, T, L, n_pad, C, H, "layer_bwd_wide")


def _layer_vs_eager(dtype, T, L, n_pad, C, H, tag):
    import argparse

    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.model.latent_model import LatentMDGenLayer
    from mdgen_finetune_amd.train_hip import LayerHelper, hip_layer_forward

    torch.manual_seed(0)
    B = 2
    layer = LatentMDGenLayer(C, 4 * C, H, use_rotary_embeddings=True).cuda()
    synthetic.fill_module_(layer, 3)
    args = argparse.Namespace(embed_dim=C, mha_heads=H, no_rope=False, num_layers=1)
    owner = argparse.Namespace(args=args, latent_dim=21)
    hl = LayerHelper(owner, dtype)
    h = torch.randn(B, T, L, C, device="cuda", requires_grad=True)
    c = torch.randn(B, C, device="cuda", requires_grad=True)
    mask = torch.ones(B, T, L, device="cuda")
    if n_pad:
        mask[:, :, L - n_pad:] = 0
    gout = torch.randn(B, T, L, C, device="cuda")
    # eager reference
    out_ref = layer(h, c[:, None], mask)
    refs = torch.autograd.grad(out_ref, [h, c] + list(layer.parameters()), gout)
    # HIP Function (mods from the same adaLN module)
    out = hip_layer_forward(hl, layer, h, layer.adaLN_modulation(c), mask)
    gots = torch.autograd.grad(out, [h, c] + list(layer.parameters()), gout)
    tol = 1e-4 if dtype == "f32" else 2.6e-2
    fwd = float((out - out_ref).norm() / out_ref.norm())
    names = ["h", "c"] + [n for n, _ in layer.named_parameters()]
    worst = (fwd, "forward")
    for n, a, b in zip(names, gots, refs):
        if b is None or float(b.norm()) == 0:
            continue
        rel = float((a.float() - b).norm() / b.norm())
        worst = max(worst, (rel, n))
    _log_train({"test": tag, "dtype": dtype, "C": C, "H": H, "T": T, "L": L, "n_pad": n_pad, "fwd_rel": fwd,
                "worst_rel": worst[0], "worst": worst[1]})
    assert worst[0] <= tol, worst


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("T,n_pad", [(129, 1), (257, 0), (1000, 1)])
def test_hip_layer_backward_default_dims_multi_chunk(dtype, T, n_pad):
    """The layer backward at config 3's dims (C = 384, 16 heads, head_dim 24) and lengths whose
    temporal attention backward runs 2, 3 and 8 chunks of 128 keys / queries with tails
    (T = 129, 257, 1000), one trajectory, against eager autograd of the same module.  Also
    pads frames at the end of the trajectory for one residue (temporal key padding across the
    last chunk) besides the padded residue.  Bounds as the layer test above; the f32 path is
    measured against an fp64 eager run (eager f32's own drift from it is logged beside)."""
    import argparse

    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.model.latent_model import LatentMDGenLayer
    from mdgen_finetune_amd.train_hip import LayerHelper, hip_layer_forward

    torch.manual_seed(T)
    C, H, B, L = 384, 16, 1, 4
    layer = LatentMDGenLayer(C, 4 * C, H, use_rotary_embeddings=True).cuda()
    synthetic.fill_module_(layer, 5)
    args = argparse.Namespace(embed_dim=C, mha_heads=H, no_rope=False, num_layers=1)
    hl = LayerHelper(argparse.Namespace(args=args, latent_dim=21), dtype)
    h = torch.randn(B, T, L, C, device="cuda", requires_grad=True)
    c = torch.randn(B, C, device="cuda", requires_grad=True)
    mask = torch.ones(B, T, L, device="cuda")
    if n_pad:
        mask[:, :, L - n_pad:] = 0
    mask[:, T - 7:, 0] = 0  # residue 0 missing in the last 7 frames: padded keys in the tail chunk
    gout = torch.randn(B, T, L, C, device="cuda")
    out_ref = layer(h, c[:, None], mask)
    refs = torch.autograd.grad(out_ref, [h, c] + list(layer.parameters()), gout)
    out = hip_layer_forward(hl, layer, h, layer.adaLN_modulation(c), mask)
    gots = torch.autograd.grad(out, [h, c] + list(layer.parameters()), gout)
    tol = 1e-4 if dtype == "f32" else 2.6e-2
    names = ["h", "c"] + [n for n, _ in layer.named_parameters()]
    refs32 = refs
    if dtype == "f32":
        # The f32 path is judged against an fp64 eager run of the same layer: bias_k's gradient is
        # a sum over all T*L queries of dS rows that sum to ~0, so eager f32 itself drifts ~1e-5
        # from the exact value at T = 1000 and would eat most of a 1e-4 bound.
        import copy

        l64 = copy.deepcopy(layer).double()
        h64 = h.detach().double().requires_grad_(True)
        c64 = c.detach().double().requires_grad_(True)
        out_ref = l64(h64, c64[:, None], mask.double())
        refs = torch.autograd.grad(out_ref, [h64, c64] + list(l64.parameters()), gout.double())
    fwd = float((out.double() - out_ref.double()).norm() / out_ref.double().norm())
    worst, errs, eager = (fwd, "forward"), {}, {}
    for n, a, b, b32 in zip(names, gots, refs, refs32):
        if b is None or float(b.norm()) == 0:
            continue
        assert torch.isfinite(a).all(), n
        b = b.double()
        rel = float((a.double() - b).norm() / b.norm())
        errs[n] = rel
        eager[n] = float((b32.double() - b).norm() / b.norm())
        worst = max(worst, (rel, n))
    rec = {"test": "layer_bwd_default_dims", "dtype": dtype, "T": T, "L": L, "n_pad": n_pad, "fwd_rel": fwd,
           "worst_rel": worst[0], "worst": worst[1],
           "attn_t": max(v for k, v in errs.items() if k.startswith("mha_t"))}
    if dtype == "f32":
        rec["vs"] = "eager fp64"
        rec["eager_f32_worst_rel"] = max(eager.values())
        rec["eager_f32_bias_k_rel"] = eager.get("mha_t.attn.bias_k")
        rec["hip_bias_k_rel"] = errs.get("mha_t.attn.bias_k")
    _log_train(rec)
    assert worst[0] <= tol, worst
    if dtype == "f32":  # and no worse than eager f32's own distance from fp64 (x1.12 measured at T = 1000)
        assert worst[0] <= max(2.0 * rec["eager_f32_worst_rel"], 1e-5), rec


def _default_dims_case(B=2, T=64, L=4, seed=31, flags=()):
    """Inputs of config 3's loss at the reference's training dims (parsing.py:86-97: embed_dim
    384, 16 heads -> head_dim 24, 5 layers, IPA prepend; flags override them): seeded latents,
    noise, t, mask."""
    from mdgen_finetune_amd import synthetic

    inp = synthetic.make_inputs(seed, B, T, L, 21)
    rng = np.random.default_rng(seed + 1)
    inp["x0"] = rng.standard_normal(inp["x"].shape).astype(np.float32)
    inp["t_loss"] = rng.uniform(0.05, 0.95, B).astype(np.float32)
    inp["loss_mask"] = np.broadcast_to(inp["mask"][..., None], inp["x"].shape).astype(np.float32).copy()
    cfg = dict(flags=list(flags), latent_dim=21, L=L, T=T, tps=False, weights_seed=seed + 2)
    return inp, cfg


@pytest.mark.parametrize("dtype,B,T", [("f32", 2, 64), ("bf16", 2, 64), ("f32", 1, 320), ("bf16", 1, 320),
                                        ("f32", 1, 1000), ("bf16", 1, 1000), ("bf16", 8, 1000)])
def test_default_dims_training_grads_match_oracle(dtype, B, T):
    """The HIP training path at the dims config 3 trains (C=384, H=16, D=24, 5 layers; T = 64,
    T = 320, whose temporal attention backward runs 3 chunks with a tail, and config 3 itself:
    T = 1000, 4 passes of 256 keys, at B = 1 with every gradient and at the bench's B = 8 for the
    loss (the oracle's CPU autograd at B = 8 x T = 1000 would take minutes)):
    the GVP loss and EVERY parameter gradient against the oracle under autograd (CPU fp32).
    Bounds: f32 loss rel 1e-5, grads 1e-4; bf16 loss 1e-2, grads BF16_DEFAULT_GRAD (~2x the
    worst observed, profiles/r04_parity_train.jsonl)."""
    training_grads_vs_oracle(dtype, B, T)


def training_grads_vs_oracle(dtype, B, T, flags=(), tag="default_dims_grads", bf16_grad_tol=None, ref64=False):
    """The GVP loss and every parameter gradient of the HIP training path against the oracle's
    CPU fp32 autograd (the body of the test above; flags: model flags, e.g. wider heads).
    ref64 (f32 path): the gradients are judged against an fp64 run of the oracle instead, each
    within max(1e-4, 2x the fp32 oracle's own distance from it) — the IPA q-projection gradients
    are ill-conditioned at some dims (the fp32 oracle sits 1.5e-3 from fp64 at embed_dim 256).
    ref64 (bf16 path): a gradient the fp32 oracle itself gets only to > 1e-4 of fp64 (such an
    ill-conditioned one) is held to twice the bf16 bound; every other one to the bound."""
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation
    from mdgen_finetune_amd.transport import create_transport
    from mdgen_finetune_amd.transport.transport import mean_flat
    from oracle import mdgen_oracle as O

    inp, cfg = _default_dims_case(B=B, T=T, flags=flags)
    f = lambda k: torch.from_numpy(np.ascontiguousarray(inp[k]))  # noqa: E731
    c = O.Cfg.from_flags(list(flags), 21, 4, False)
    P = O.seeded_params(c, cfg["weights_seed"])
    for v in P.values():
        v.requires_grad_(True)
    torch.set_num_threads(16)
    kw_cpu = dict(mask=f("mask"), rots=f("rots"), trans=f("trans"), x_cond=f("x_cond"), x_cond_mask=f("x_cond_mask"),
                  aatype=f("aatype"))
    grads = B * T <= 1000
    with torch.set_grad_enabled(grads):
        loss_ref, _ = O.gvp_training_loss(P, c, f("x"), f("x0"), f("t_loss"), f("loss_mask"), **kw_cpu)
    if grads:
        loss_ref.mean().backward()
    g64 = None
    if ref64 and grads:
        P64 = {k: v.detach().double().requires_grad_(True) for k, v in P.items()}
        d = lambda k: f(k).double() if f(k).is_floating_point() else f(k)  # noqa: E731
        kw64 = dict(mask=d("mask"), rots=d("rots"), trans=d("trans"), x_cond=d("x_cond"), x_cond_mask=d("x_cond_mask"),
                    aatype=d("aatype"))
        l64, _ = O.gvp_training_loss(P64, c, d("x"), d("x0"), d("t_loss"), d("loss_mask"), **kw64)
        l64.mean().backward()
        g64 = {k: v.grad for k, v in P64.items()}

    m, _ = build_model(cfg, "cuda", T=T)
    m.train()
    m.hip_dtype = dtype
    g = lambda k: f(k).cuda()  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    assert m._use_hip_layers(torch.zeros(1, device="cuda", requires_grad=True))
    tr = create_transport(m.args, "GVP", "velocity")
    t, xt, ut = tr.path_sampler.plan(g("t_loss"), g("x0"), g("x"))
    v = m(xt, t, **kw)
    loss = mean_flat((v - ut) ** 2, g("loss_mask"))
    loss.mean().backward()
    lrel = float((loss.detach().cpu() - loss_ref.detach()).abs().max() / loss_ref.detach().abs().max())
    names = dict(m.named_parameters())
    worst, checked = (0.0, None), 0
    if not grads:  # the bench's size: the loss, and every parameter received a finite gradient
        _log_train({"test": tag, "dtype": dtype, "B": B, "T": T, "loss_rel": lrel, "flags": list(flags)})
        assert lrel <= 1e-2, lrel
        got = [p.grad for p in m.parameters() if p.grad is not None]
        assert len(got) > 250 and all(bool(torch.isfinite(gr).all()) for gr in got)
        return
    for k, p in P.items():
        if p.grad is None or k not in names or float(p.grad.norm()) < 1e-8:
            continue
        gg = names[k].grad
        assert gg is not None, k
        if g64 is not None and dtype == "f32":  # relative to the fp32 oracle's own error, against fp64
            ref = g64[k]
            own = float((p.grad.double() - ref).norm() / ref.norm())
            rel = float((gg.detach().double().cpu() - ref).norm() / ref.norm()) / max(1.0, own * 2e4)
        else:
            rel = float((gg.detach().float().cpu() - p.grad).norm()) / float(p.grad.norm())
            if g64 is not None:  # bf16: an ill-conditioned gradient (the fp32 oracle > 1e-4 from fp64) gets 2x
                own = float((p.grad.double() - g64[k]).norm() / g64[k].norm())
                if own > 1e-4:
                    rel *= 0.5
        worst = max(worst, (rel, k))
        checked += 1
    _log_train({"test": tag, "dtype": dtype, "B": B, "T": T, "loss_rel": lrel, "worst_grad_rel": worst[0],
                "worst_param": worst[1], "checked": checked, "flags": list(flags),
                "vs": ("oracle fp64 (rel / max(1, 2e4 x fp32 oracle's rel))" if dtype == "f32" else
                       "oracle fp32 (rel / 2 where the fp32 oracle is > 1e-4 from fp64)") if g64 is not None
                else "oracle fp32"})
    loss_tol, grad_tol = (1e-5, 1e-4) if dtype == "f32" else (1e-2, bf16_grad_tol or BF16_DEFAULT_GRAD)
    assert lrel <= loss_tol, lrel
    assert worst[0] <= grad_tol, worst
    assert checked > 250


BF16_DEFAULT_GRAD = 2e-2  # ~2x the worst observed (8.3e-3 at T=320, 7.7e-3 at T=64: r04_parity_train.jsonl)


def _fixed_noise(tr, B, shape, seed=5):
    """Replace the transport's (t, x0) draw with fixed device tensors (graph-safe)."""
    gen = torch.Generator().manual_seed(seed)
    x0 = torch.randn(*shape, generator=gen).cuda()
    t = (0.05 + 0.9 * torch.rand(B, generator=gen)).cuda()
    tr.wrapper.transport.sample = lambda x1: (t, x0, x1)


def test_graphed_step_equals_eager_step():
    """Trainer.graph_mode (GraphedStep: forward + loss + backward + clip + Adam + EMA replayed
    from one hipGraph) against the eager step on the same batch and noise: the updated
    parameters, the loss and the grad norm agree; later replays keep training (the loss moves)."""
    from mdgen_finetune_amd.train import Trainer

    res = {}
    for mode in (0, 1):
        a = _args(["--lr", "1e-3", "--embed_dim", "192", "--mha_heads", "8", "--ema", "--train_graph", str(mode)])
        tr = Trainer(a, device=torch.device("cuda"))
        assert tr.graph_mode == bool(mode)
        b = _batch(a, B=2)
        _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 21))
        loss, gnorm = tr.step([b], log=False)
        res[mode] = (float(loss), float(gnorm), torch.cat([p.detach().flatten() for p in tr.wrapper.model.parameters()]),
                     torch.cat([v.flatten() for v in tr.wrapper.ema.params.values() if v.is_floating_point()]))
        if mode:
            losses = [float(tr.step([b], log=False)[0]) for _ in range(3)]
            assert len(set(losses)) > 1 and np.isfinite(losses).all()
    (l0, g0, p0, e0), (l1, g1, p1, e1) = res[0], res[1]
    assert abs(l0 - l1) <= 1e-5 * abs(l0), (l0, l1)
    assert abs(g0 - g1) <= 1e-4 * abs(g0), (g0, g1)
    assert float((p0 - p1).abs().max()) <= 1e-6, float((p0 - p1).abs().max())
    assert float((e0 - e1).abs().max()) <= 1e-6


def _share_worker(rank, world, port, graph, out):
    import faulthandler
    import os

    faulthandler.enable()

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MDG_SHARE_GPU="1")
    from mdgen_finetune_amd.train import Trainer, setup_distributed

    r, w, dev = setup_distributed()
    a = _args(["--grad_clip", "0", "--embed_dim", "192", "--mha_heads", "8", "--train_graph", str(graph),
               "--bucket_cap_mb", "0.25"])
    tr = Trainer(a, r, w, dev)
    assert tr.graph_mode == bool(graph)
    b = _batch(a, B=2, seed=100 + rank)
    _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 21), seed=7 + rank)
    m = tr.wrapper.model
    params = [p for p in m.parameters() if p.requires_grad]
    def local_grads():  # returns no autograd state: the graph (and its AccumulateGrad nodes,
        # created on this stream) must be gone before GraphedStep warms up on its side stream
        prep = tr.wrapper.prep_batch({k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()})
        loss = tr.wrapper.transport.training_losses(m, prep["latents"], mask=prep["loss_mask"],
                                                    model_kwargs=prep["model_kwargs"])["loss"].mean()
        g = torch.autograd.grad(loss, params, allow_unused=True)
        return torch.cat([(x if x is not None else torch.zeros_like(p)).flatten() for x, p in zip(g, params)])

    local = local_grads()
    ref = local.clone()
    dist.all_reduce(ref)
    ref /= w
    seen = []
    orig = tr.optimizer.step
    tr.optimizer.step = lambda *a_, **k_: (seen.append(torch.cat([p.grad.flatten().clone() for p in params])),
                                           orig())[1]
    if graph:
        tr.step([b], log=False)
        got = tr._graphed.flat.clone()
    else:
        for _ in range(2):  # DDP's bucketed path from its third iteration (static graph)
            tr.wrapper.general_step({k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()},
                                    model=tr.model).backward()
            tr.optimizer.zero_grad(set_to_none=True)
        tr.step([b], log=False)
        got = seen[-1]
    pall = torch.cat([p.detach().flatten() for p in params])
    gathered = [torch.zeros_like(pall) for _ in range(w)]
    dist.all_gather(gathered, pall)
    out[rank] = (float((got - ref).abs().max()), float(ref.abs().max()), float((gathered[0] - gathered[1]).abs().max()),
                 float((local - ref).abs().max()))
    dist.destroy_process_group()


@pytest.mark.parametrize("graph", [0, 1])
def test_world2_on_one_gpu_allreduce_matches_local_mean(graph):
    """Two ranks on cuda:0 over gloo (MDG_SHARE_GPU=1), each running the HIP training Function:
    graph=0 through DistributedDataParallel (bucketed all-reduce during backward), graph=1
    through GraphedStep (flat all-reduce between its two graphs).  The averaged gradient equals
    the mean of the ranks' local gradients and the replicas stay identical after Adam."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_share_worker, args=(2, port, graph, out), nprocs=2, join=True)
    for r in range(2):
        err, scale, drift, spread = out[r]
        assert err <= 1e-5 * max(1.0, scale), (r, err, scale)
        assert drift == 0.0
        assert spread > 0.0


def test_grad_checkpointing_on_hip_layers_same_grads():
    """--grad_checkpointing with the HIP training Function (reentrant checkpoint: the layer's
    forward re-runs in backward) gives the same gradients as the stored-activation path."""
    d, cfg = load_golden("small_loss")
    grads = []
    for ck in (False, True):
        m, _ = build_model(cfg, "cuda")
        m.train()
        m.args.grad_checkpointing = ck
        loss, _ = _model_loss(m, d, "cuda")
        loss.mean().backward()
        grads.append(torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None]))
    assert grads[0].shape == grads[1].shape
    assert torch.equal(grads[0], grads[1]), float((grads[0] - grads[1]).abs().max())


def _trainer_state(tr):
    params = torch.cat([p.detach().flatten() for p in tr.wrapper.model.parameters()])
    ema = torch.cat([v.flatten() for v in tr.wrapper.ema.params.values() if v.is_floating_point()])
    moments = torch.cat([st[k].detach().flatten().float() for st in tr.optimizer.state.values()
                         for k in ("exp_avg", "exp_avg_sq", "step") if k in st])
    return params, ema, moments


def test_graphed_resume_keeps_optimizer_state_and_ema(tmp_path):
    """--ckpt resume into the graphed step (train_graph 1, the ROCm default): GraphedStep's warm-up
    must hand the capture the LOADED Adam moments / step count and EMA, not zeros.
    Train 2 graphed steps, save; resume twice (graphed and eager) and take one step on the same
    batch and noise: parameters, Adam state and EMA agree."""
    import os

    from mdgen_finetune_amd.checkpoint import load_checkpoint
    from mdgen_finetune_amd.train import Trainer

    base = ["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4", "--ema", "--ema_decay", "0.9"]
    a = _args(base + ["--train_graph", "1", "--max_steps", "2", "--epochs", "1"], tmp_path)
    tr = Trainer(a, device=torch.device("cuda"))
    tr.fit()
    ck_path = os.path.join(tmp_path, sorted(os.listdir(tmp_path))[-1])
    ck = load_checkpoint(ck_path)
    saved_steps = [float(s["step"]) for s in ck["optimizer_states"][0]["state"].values()]
    assert saved_steps and all(s == 2.0 for s in saved_steps)
    res = {}
    for mode in (1, 0):
        a2 = _args(base + ["--train_graph", str(mode), "--ckpt", ck_path], tmp_path)
        tr2 = Trainer(a2, device=torch.device("cuda"))
        b = _batch(a2, B=2, seed=3)
        _fixed_noise(tr2, 2, (2, a2.num_frames, a2.crop, 21))
        tr2.step([b], log=False)
        res[mode] = _trainer_state(tr2)
        steps = {float(st["step"]) for st in tr2.optimizer.state.values()}
        assert steps == {3.0}, (mode, steps)
    for i, what in enumerate(("params", "ema", "adam")):
        d = float((res[0][i] - res[1][i]).abs().max())
        assert d <= 1e-6 * max(1.0, float(res[0][i].abs().max())), (what, d)


def test_tps_graphed_step_equals_eager_step():
    """TPS fine-tuning (--tps_condition) in the graphed step: the relative frames (a host eigh)
    are staged outside the capture (GraphedStep._stage_rel7); the replayed step equals the eager
    step (the capture used to fail on the .cpu() inside relative_tensor7)."""
    from mdgen_finetune_amd.train import Trainer

    res = {}
    for mode in (0, 1):
        a = _args(["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4", "--tps_condition", "--train_graph",
                   str(mode)])
        a.sim_condition = False
        tr = Trainer(a, device=torch.device("cuda"))
        assert tr.graph_mode == bool(mode) and tr.wrapper.model.tps
        b = _batch(a, B=2)
        _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 28))
        loss = float(tr.step([b], log=False)[0])  # (the graphed step's loss is a static buffer)
        if mode:  # a second batch re-stages its own frames
            tr.step([_batch(a, B=2, seed=9)], log=False)
            tr2 = Trainer(a, device=torch.device("cuda"))
            tr2.graph_mode = False
            _fixed_noise(tr2, 2, (2, a.num_frames, a.crop, 28))
            tr2.step([b], log=False)
            tr2.step([_batch(a, B=2, seed=9)], log=False)
            p2 = torch.cat([p.detach().flatten() for p in tr2.wrapper.model.parameters()])
        res[mode] = (loss, torch.cat([p.detach().flatten() for p in tr.wrapper.model.parameters()]))
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[0][0])
    p1 = res[1][1]
    # two optimizer steps: the graphed step updates with the library's clip + Adam
    # (optim_hip.FusedClipAdam), the eager one with torch's; their clip norms differ in the last
    # bits, so the second step's gradients differ slightly, and Adam's eps regime (|g| ~ 1e-9,
    # v ~ 1e-20: update ~ g / (sqrt(v) + eps)) turns that into up to ~1 % of lr on those elements
    # (tools/diag_tps_graph.py: 8.6e-6 at lr 1e-3, 0 with MDG_TRAIN_FUSED_OPT=0).  A mis-staged
    # second batch moves O(lr) on most parameters.
    assert float((p1 - p2).abs().max()) <= 2e-2 * 1e-3, float((p1 - p2).abs().max())


@pytest.mark.parametrize("L", [16, 20, 48])
def test_tps_ipa_long_crop_grads_match_eager(L):
    """TPS with the IPA prepend at crops L >= 16: run_ipa calls every IPA layer twice per step
    (x_r, x_f; latent_model.py:240-243) on the HIP layer Function, whose L >= 16 spatial planes are
    saved activations; the two calls must not share them.  L = 48: the IPA core on
    the long kernels (33..256 residues).  Every parameter gradient of the HIP f32 path against
    eager autograd on the same device, rel <= 1e-4."""
    from mdgen_finetune_amd.transport.transport import mean_flat
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    a = _args(["--embed_dim", "64", "--mha_heads", "4", "--tps_condition", "--crop", str(L), "--num_frames", "4"])
    a.sim_condition = False
    torch.manual_seed(0)
    w = NewMDGenWrapper(a).cuda()
    m = w.model
    from mdgen_finetune_amd import synthetic

    synthetic.fill_module_(m, 11)  # non-zero IPA linear_out / adaLN so every path carries gradient
    m.train()
    m.hip_dtype = "f32"
    b = {k: (v.cuda() if torch.is_tensor(v) else v) for k, v in _batch(a, B=2, seed=4).items()}
    prep = w.prep_batch(b)
    gen = torch.Generator().manual_seed(2)
    x0 = torch.randn(prep["latents"].shape, generator=gen).cuda()
    t = (0.1 + 0.8 * torch.rand(2, generator=gen)).cuda()
    grads = {}
    for backend in ("hip", "torch"):
        m.train_backend = backend
        m.zero_grad(set_to_none=True)
        tt, xt, ut = w.transport.path_sampler.plan(t, x0, prep["latents"])
        v = m(xt, tt, **prep["model_kwargs"])
        mean_flat((v - ut) ** 2, prep["loss_mask"]).mean().backward()
        grads[backend] = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    worst = (0.0, None)
    for n, gr in grads["torch"].items():
        if float(gr.norm()) < 1e-10:
            continue
        assert n in grads["hip"], n
        worst = max(worst, (float((grads["hip"][n] - gr).norm() / gr.norm()), n))
    _log_train({"test": "tps_ipa_long_crop", "L": L, "worst_grad_rel": worst[0], "worst_param": worst[1]})
    assert worst[0] <= 1e-4, worst
    assert any(n.startswith("ipa_layers.") and "mha_l" in n for n in grads["hip"])


def _rccl_world1_worker(rank, port, out):
    """The body of test_graphed_step_rccl_bucket_allreduce_in_capture_world1 in a child process,
    ending with the production teardown of train.main: the graphs holding captured collectives
    released, the device drained, destroy_process_group, a normal return (no os._exit)."""
    import gc

    import torch.distributed as dist

    from mdgen_finetune_amd.train import Trainer

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    res = {}
    info = {}
    from mdgen_finetune_amd import synthetic

    for mode in ("plain", "rccl", "rccl_cg", "plain_tps", "rccl_cg_tps"):
        tps = mode.endswith("_tps")
        a = _args(["--lr", "1e-3", "--embed_dim", "192", "--mha_heads", "8", "--ema", "--train_graph", "1",
                   "--bucket_cap_mb", "0.5"] + (["--tps_condition"] if tps else []))
        a.sim_condition = not tps
        tr = Trainer(a, device=torch.device("cuda"))
        synthetic.fill_module_(tr.wrapper.model, 23)  # gradients reach every parameter
        tr.force_allreduce = not mode.startswith("plain")
        tr.dp_markers = True
        if "_cg" in mode:  # + the replicated conditioning's all-gathers (cond_dist.py) in the capture,
            # on their own communicator
            assert tr.setup_cond_gather()
            assert tr.wrapper.model._cond_gather.group is not None
        b = _batch(a, B=2)
        _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 28 if tps else 21))
        losses = [float(tr.step([b], log=False)[0]) for _ in range(2)]
        g = tr._graphed
        if not mode.startswith("plain"):
            red = g.reducer
            info[mode] = {"overlap": bool(g.overlap), "has_g2": hasattr(g, "g2"), "buckets": len(red.buckets),
                          "log": list(red.launch_log), "grads": sum(len(bk) for bk in red.buckets),
                          "replicated": len(tr.replicated), "dp_ms": g.dp_times_ms(),
                          "views": all(p.grad is None or p.grad.data_ptr() == red.views[i].data_ptr()
                                       for i, p in enumerate(g.params) if i in red.views)}
        st = _trainer_state(tr)
        res[mode] = (losses, [t.cpu() for t in st])
        torch.cuda.synchronize()
        g = red = None
        tr._graphed = None  # train.main's order: the graph before the communicator
        tr = None
    out["res"], out["info"] = res, info
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    out["teardown"] = "ok"


def test_graphed_step_rccl_bucket_allreduce_in_capture_world1():
    """The graphed step's gradient all-reduce captured INSIDE the graph (grad_buckets.py): a world-1
    RCCL group (a one-GPU box cannot hold two RCCL ranks) with the reduction forced on.  The step
    is one graph whose bucket all-reduces are side-stream branches issued from backward's hooks;
    its parameters / EMA after two steps equal the plain graphed step's (world 1: the average is
    the identity), the buckets follow backward's completion order and the first launches before
    the last gradient lands.  (Timeline of the captured collectives: tools/rccl_overlap_trace.py.)"""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_world1_worker, args=(port, out), nprocs=1, join=True)
    assert out.get("teardown") == "ok"
    for mode in ("rccl", "rccl_cg", "rccl_cg_tps"):
        info = out["info"][mode]
        assert info["overlap"] and not info["has_g2"], info
        assert info["buckets"] >= 3, info
        assert [bi for bi, _ in info["log"]] == list(range(info["buckets"])), info
        assert info["log"][0][1] < info["grads"], info
        assert info["views"]
        fb, exposed = info["dp_ms"]  # the in-graph DP markers (bench.py's train_dp line) read back
        assert 0.0 < fb < 1e4 and 0.0 <= exposed < fb, info["dp_ms"]
    # the replicated conditioning's parameters leave the buckets (TPS too: VERDICT r05 missing 3)
    assert out["info"]["rccl_cg"]["replicated"] > 20 and out["info"]["rccl_cg_tps"]["replicated"] > 20
    assert out["info"]["rccl_cg"]["grads"] + out["info"]["rccl_cg"]["replicated"] == out["info"]["rccl"]["grads"]
    for plain, modes in (("plain", ("rccl", "rccl_cg")), ("plain_tps", ("rccl_cg_tps",))):
      (l0, s0) = out["res"][plain]
      for mode in modes:
        l1, s1 = out["res"][mode]
        assert l0 == l1, (mode, l0, l1)
        for i, what in enumerate(("params", "ema", "adam")):
            d = float((s0[i] - s1[i]).abs().max())
            assert d <= 1e-6 * max(1.0, float(s0[i].abs().max())), (mode, what, d)


@pytest.mark.parametrize("tps", [False, True])
def test_training_backward_bitwise_repeatable(tps):
    """The replicated conditioning (cond_dist.py) keeps the ranks' replicas identical only if
    the same inputs give bit-identical gradients on every rank: the whole HIP training forward +
    backward (conditioning included: t-MLP, adaLN, IPA core, embedding) run twice on the same
    batch and noise gives bitwise-equal gradients for every parameter."""
    from mdgen_finetune_amd.train import Trainer

    from mdgen_finetune_amd import synthetic

    a = _args(["--embed_dim", "64", "--mha_heads", "4"] + (["--tps_condition"] if tps else []))
    a.sim_condition = not tps
    tr = Trainer(a, device=torch.device("cuda"))
    m = tr.wrapper.model
    synthetic.fill_module_(m, 29)
    b = {k: (v.cuda() if torch.is_tensor(v) else v) for k, v in _batch(a, B=2, seed=4).items()}
    _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 28 if tps else 21))
    grads = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        tr.wrapper.general_step(b, model=m).backward()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})
    assert len(grads[0]) > 50 and grads[0].keys() == grads[1].keys()
    bad = [n for n in grads[0] if not torch.equal(grads[0][n], grads[1][n])]
    assert not bad, bad[:8]
