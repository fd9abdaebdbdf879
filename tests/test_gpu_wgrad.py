"""mdg_wgrad (csrc/wgrad.hip): the training weight / bias gradients dW = dY^T X, db = colsum(dY)
of every linear layer in the block (the nn.Linear backward of latent_model.py:456-493 under
loss.backward()), against a plain torch fp32 reference of the same op on the same (bf16-rounded)
operands.  Tolerance: ||d|| / ||ref|| <= 1e-5 (fp32 accumulation in a different order), and the
result must be bit-identical across repeated calls (fixed split order, no atomics).  The bf16
shapes with a side divisible by 256 (fc1 / fc2: 1536 x 384, 384 x 1536) take the wide tiles
(256 x 128 / 128 x 256, wgrad_bf16_wide_kernel)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("N,M,K", [(32000, 1152, 384), (32000, 384, 1536), (544, 192, 64), (96, 200, 72),
                                   (64, 8, 8), (4000, 1536, 384), (32000, 1536, 384), (96, 256, 128),
                                   (288, 128, 512)])
def test_wgrad_matches_torch(dtype, N, M, K):
    from mdgen_finetune_amd import _lib
    from mdgen_finetune_amd.train_hip import wgrad

    lib = _lib.load()
    torch.manual_seed(N + M + K)
    ct = torch.bfloat16 if dtype == "bf16" else torch.float32
    mdt = _lib.MDG_BF16 if dtype == "bf16" else _lib.MDG_F32
    dy = torch.randn(N, M, device="cuda").to(ct)
    x = torch.randn(N, K, device="cuda").to(ct)
    dw, db = wgrad(lib, mdt, dy, x, need_b=True)
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    assert _rel(dw.double(), ref_w) <= 1e-5, _rel(dw.double(), ref_w)
    assert _rel(db.double(), ref_b) <= 1e-5, _rel(db.double(), ref_b)
    dw2, db2 = wgrad(lib, mdt, dy, x, need_b=True)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


def test_wgrad_strided_operands_and_bias_only():
    """Operands as column slices of wider rows (ld > M / K), and the bias-only form."""
    from mdgen_finetune_amd import _lib
    from mdgen_finetune_amd.train_hip import wgrad

    lib = _lib.load()
    torch.manual_seed(1)
    big = torch.randn(1024, 3 * 384, device="cuda").to(torch.bfloat16)
    dy = big[:, 384:768]
    x = torch.randn(1024, 512, device="cuda").to(torch.bfloat16)[:, :384]
    dw, db = wgrad(lib, _lib.MDG_BF16, dy, x, need_b=True)
    assert _rel(dw.double(), dy.double().t() @ x.double()) <= 1e-5
    _, db2 = wgrad(lib, _lib.MDG_BF16, dy, None, need_b=True)
    # db rides in the dW blocks when both are asked for, else the column-sum pass: two orders
    assert _rel(db.double(), db2.double()) <= 1e-6
    assert _rel(db2.double(), dy.double().sum(0)) <= 1e-5


def test_wgrad_rejects_unpadded_bf16_rows():
    from mdgen_finetune_amd import _lib
    from mdgen_finetune_amd.train_hip import wgrad

    lib = _lib.load()
    dy = torch.randn(100, 64, device="cuda").to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        wgrad(lib, _lib.MDG_BF16, dy, dy, need_b=False)
