"""mdg_ln_gate_bwd (train.hip) against torch autograd: the backward of a no-affine LayerNorm +
adaLN modulate (latent_model.py:467/475/489) fused with the gated-residual backward of the
sublayer below it (latent_model.py:472/486/491), for the C = 384 vector kernel and the generic
one (C = 64), in every operand combination the training Function uses."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _ref(h_prev, y, mods, G0, G1, C, with_dxn, with_y, shift_off, scale_off, gate_off, TL):
    """h = h_prev + gate * y (when with_y); xn = LN(h) (1 + scale) + shift; L = <xn, G1> + <h, G0>."""
    h_prev = h_prev.clone().requires_grad_(True)
    y = y.clone().requires_grad_(True)
    mods = mods.clone().requires_grad_(True)
    rows_b = torch.arange(h_prev.shape[0], device=h_prev.device) // TL
    m = mods[rows_b]
    h = h_prev + m[:, gate_off:gate_off + C] * y if with_y else h_prev
    loss = (h * G0).sum()
    if with_dxn:
        mu = h.mean(-1, keepdim=True)
        var = ((h - mu) ** 2).mean(-1, keepdim=True)
        xn = (h - mu) / torch.sqrt(var + 1e-6) * (1 + m[:, scale_off:scale_off + C]) + m[:, shift_off:shift_off + C]
        loss = loss + (xn * G1).sum()
    dh_prev, dy, dmods = torch.autograd.grad(loss, (h_prev, y, mods), allow_unused=True)
    return h, dh_prev, dy, dmods


@pytest.mark.parametrize("C", [384, 64])
@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("with_dxn,with_y", [(True, True), (True, False), (False, True)])
def test_ln_gate_bwd_matches_autograd(C, dtype, with_dxn, with_y):
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    torch.manual_seed(0)
    B, TL = 3, 100  # 100 rows per trajectory: ragged last row block (64 + 36)
    N = B * TL
    dev = "cuda"
    ct = torch.bfloat16 if dtype == "bf16" else torch.float32
    h_prev = torch.randn(N, C, device=dev)
    y = torch.randn(N, C, device=dev).to(ct).float()
    mods = 0.3 * torch.randn(B, 9 * C, device=dev)
    G0 = torch.randn(N, C, device=dev)
    G1 = torch.randn(N, C, device=dev).to(ct).float()
    shift_off, scale_off, gate_off = 3 * C, 4 * C, 2 * C
    h, dh_ref, dy_ref, dmods_ref = _ref(h_prev, y, mods, G0, G1, C, with_dxn, with_y, shift_off, scale_off, gate_off,
                                        TL)
    h = h.detach()
    mu = h.mean(-1)
    rstd = 1.0 / torch.sqrt(((h - mu[:, None]) ** 2).mean(-1) + 1e-6)
    stats = torch.stack([mu, rstd], -1).contiguous()
    dxn = G1.to(ct).contiguous() if with_dxn else None
    yk = y.to(ct).contiguous() if with_y else None
    dh_out = torch.empty(N, C, device=dev)
    dy = torch.empty(N, C, device=dev, dtype=ct) if with_y else None
    nb = lib.mdg_ln_gate_bwd_blocks(TL)
    part = torch.empty(B, nb, 4, C, device=dev)
    mdt = _lib.MDG_BF16 if dtype == "bf16" else _lib.MDG_F32
    _lib.check(lib.mdg_ln_gate_bwd(mdt, N, C, TL, _lib.ptr(dxn), _lib.ptr(h if with_dxn else None),
                                   _lib.ptr(stats if with_dxn else None), mods.data_ptr(), 9 * C, shift_off, scale_off,
                                   G0.data_ptr(), dh_out.data_ptr(), _lib.ptr(yk), gate_off, _lib.ptr(dy),
                                   part.data_ptr(), _lib.stream_handle()),
               "mdg_ln_gate_bwd")
    torch.cuda.synchronize()

    def close(a, b, tol):
        err = float((a - b).abs().max())
        assert err <= tol * max(1.0, float(b.abs().max())), err

    close(dh_out, dh_ref, 2e-5)
    p = part.sum(1)  # [B, 4, C]
    if with_dxn:
        close(p[:, 0], dmods_ref[:, shift_off:shift_off + C], 2e-5)
        close(p[:, 1], dmods_ref[:, scale_off:scale_off + C], 2e-5)
    if with_y:
        close(dy.float(), dy_ref, 1e-2 if dtype == "bf16" else 2e-5)
        close(p[:, 2], dmods_ref[:, gate_off:gate_off + C], 2e-5)
        close(p[:, 3], (dh_ref * mods[torch.arange(N, device=dev) // TL, gate_off:gate_off + C]).reshape(B, TL, C).sum(1),
              2e-5)
