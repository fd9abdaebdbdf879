"""Run one mdg_gemm shape repeatedly (for rocprofv3 counter passes).
Usage: python tools/gemm_one.py M N K EPI ACT [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench  # noqa: E402

M, N, K, epi, act = (int(a) for a in sys.argv[1:6])
it = int(sys.argv[6]) if len(sys.argv) > 6 else 20
gemm_bench.run(M, N, K, 0, epi, act=act)
