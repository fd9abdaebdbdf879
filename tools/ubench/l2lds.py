"""Run tools/ubench/l2lds.hip (build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/ubench/libl2lds.so
tools/ubench/l2lds.hip): L2 -> LDS fill rate per CU vs bytes in flight per block, all CUs streaming."""
import ctypes
import json
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libl2lds.so"))
lib.l2lds_run.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                          ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
lib.l2vgpr_run.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
buf = torch.ones(256 << 20, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")
CUS, CLK = 256, 2.4e9
for window in (2 << 20, 256 << 20):
    for depth, pieces in ((2, 2), (2, 4), (4, 2), (4, 4), (8, 2), (8, 4)):
        steps = 2000
        ms = ctypes.c_float()
        rc = lib.l2lds_run(buf.data_ptr(), window, steps, depth, pieces, CUS, sink.data_ptr(), ctypes.byref(ms))
        if rc:
            print(json.dumps({"window": window, "depth": depth, "pieces": pieces, "rc": rc}))
            continue
        by = CUS * steps * 512 * 16 * pieces
        print(json.dumps({"window_mb": window >> 20, "depth": depth, "inflight_kb": (depth - 1) * 8 * pieces,
                          "ms": round(ms.value, 3), "TB_s": round(by / ms.value / 1e9, 2),
                          "B_per_clk_cu": round(by / (ms.value * 1e-3) / CLK / CUS, 1)}), flush=True)
for window in (2 << 20,):
    for tolds in (0, 1):
        steps = 2000
        ms = ctypes.c_float()
        rc = lib.l2vgpr_run(buf.data_ptr(), window, steps, tolds, CUS, sink.data_ptr(), ctypes.byref(ms))
        by = CUS * steps * 512 * 16 * 4
        print(json.dumps({"vgpr_loads": True, "to_lds": tolds, "rc": rc, "ms": round(ms.value, 3),
                          "TB_s": round(by / ms.value / 1e9, 2),
                          "B_per_clk_cu": round(by / (ms.value * 1e-3) / CLK / CUS, 1)}), flush=True)
for blocks in (8, 32, 64, 128, 256):
    steps = 2000
    ms = ctypes.c_float()
    rc = lib.l2lds_run(buf.data_ptr(), 2 << 20, steps, 4, 4, blocks, sink.data_ptr(), ctypes.byref(ms))
    by = blocks * steps * 512 * 16 * 4
    ms2 = ctypes.c_float()
    rc2 = lib.l2vgpr_run(buf.data_ptr(), 2 << 20, steps, 0, blocks, sink.data_ptr(), ctypes.byref(ms2))
    print(json.dumps({"blocks": blocks, "lds_dma_B_per_clk_cu": round(by / (ms.value * 1e-3) / CLK / blocks, 1),
                      "vgpr_B_per_clk_cu": round(by / (ms2.value * 1e-3) / CLK / blocks, 1), "rc": [rc, rc2]}), flush=True)
# co-resident blocks per CU: 256 / 512 / 1024 blocks of 512 threads, 32 KiB of LDS each (depth 2 x 2 pieces)
for blocks in (256, 512, 1024):
    steps = 2000
    ms = ctypes.c_float()
    rc = lib.l2lds_run(buf.data_ptr(), 2 << 20, steps, 2, 2, blocks, sink.data_ptr(), ctypes.byref(ms))
    by = blocks * steps * 512 * 16 * 2
    print(json.dumps({"blocks_total": blocks, "per_cu": blocks // CUS, "rc": rc,
                      "lds_dma_B_per_clk_cu": round(by / (ms.value * 1e-3) / CLK / CUS, 1)}), flush=True)
