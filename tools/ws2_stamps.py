"""Per-phase timeline of the wave-specialised MLP (mlp_ws2_kernel) from a DIAG 5 build
(-DMDG_DIAG_WS2=32 (| 64, | 128): shader-clock stamps of block 0's waves 0 (P) and 4 (Q) into f1.out).
usage: MDG_MLP_WS=2 MDG_LIB_PATH=ablib/diag32.so python tools/ws2_stamps.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402

lib = _lib.load()
M, C, F, rpm = 32000, 384, 1536, 4000
A = (torch.randn(M, C, device="cuda") * 0.5).to(torch.bfloat16)
W1 = (torch.randn(F, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
W2 = (torch.randn(C, F, device="cuda") / F ** 0.5).to(torch.bfloat16)
b1, b2 = torch.randn(F, device="cuda"), torch.randn(C, device="cuda")
hid = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
resid, xn = torch.zeros(M, C, device="cuda"), torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
mods = torch.randn(M // rpm + 1, 9 * C, device="cuda") * 0.1
f1, f2 = _lib.MdgGemmDesc(), _lib.MdgGemmDesc()
f1.dtype, f1.a_mode, f1.epi, f1.act, f1.M, f1.N, f1.K = 1, 0, 0, 1, M, F, C
f1.A, f1.lda, f1.W, f1.ldw, f1.bias, f1.out, f1.ldo = A.data_ptr(), C, W1.data_ptr(), C, b1.data_ptr(), hid.data_ptr(), F
f2.dtype, f2.a_mode, f2.epi, f2.M, f2.N, f2.K = 1, 0, 1, M, C, F
f2.A, f2.lda, f2.W, f2.ldw, f2.bias = hid.data_ptr(), F, W2.data_ptr(), F, b2.data_ptr()
f2.resid, f2.ldr, f2.gate, f2.gate_off, f2.mod_stride, f2.rows_per_mod = resid.data_ptr(), C, mods.data_ptr(), 0, 9 * C, rpm
f2.xn_out, f2.xn_mods, f2.xn_mod_stride, f2.xn_shift_off, f2.xn_scale_off, f2.ln_eps = (xn.data_ptr(), mods.data_ptr(),
                                                                                       9 * C, 0, C, 1e-6)
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    _lib.check(lib.mdg_mlp_fused(ctypes.byref(f1), ctypes.byref(f2), s), "mlp")
torch.cuda.synchronize()
st = hid.view(-1).view(torch.int64)[:8 * 512].view(8, 512).cpu()
P, Q = st[0].tolist(), st[4].tolist()
n = F // 128
t0 = P[0]
print(f"P start {0}  first barrier {P[1] - t0}   Q start {Q[0] - t0}  Q enters chunk loop {Q[1] - t0}")
labels = ["gelu B", "fc1 4c", "wait", "bar", "fc1 4c+1", "wait", "bar", "gelu A", "fc1 4c+2", "wait", "bar", "fc1 4c+3",
          "wait", "bar"]
tot = [0] * len(labels)
k = 2
prev = P[1]
for c in range(n):
    row = []
    for j, lab in enumerate(labels):
        d = P[k] - prev
        prev = P[k]
        k += 1
        tot[j] += d
        row.append(d)
    if c in (0, 5): print(f"P chunk {c:2d}: " + " ".join(f"{x:5d}" for x in row))
print("P totals: " + ", ".join(f"{lab} {t}" for lab, t in zip(labels, tot)))
print(f"P after loop: gelu B + tail barriers {P[k] - prev}, epilogue {P[k + 1] - P[k]}, end {P[k + 1] - t0}")
qt = [0, 0, 0]
k = 2
prev = Q[1]
for c in range(n):
    row = []
    for kb in range(4):
        for j in range(3):
            d = Q[k] - prev
            prev = Q[k]
            k += 1
            qt[j] += d
            row.append(d)
    if c in (0, 5): print(f"Q chunk {c:2d}: " + " ".join(f"{x:5d}" for x in row))
print(f"Q totals: W2 wait {qt[0]}, MFMA {qt[1]}, barrier {qt[2]};  epilogue {Q[k + 1] - Q[k]}, end {Q[k + 1] - t0}")
