"""Static checks of the built gfx950 code (CPU; needs the in-tree objects that build() makes).

No kernel may reach an s_barrier with LDS operations still in flight (tools/lds_barrier_scan.py):
a ring slot refilled by LDS DMA after the barrier would race them (gemm.hip kRingWaitNote)."""
import glob
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_lds_reads_in_flight_at_barriers():
    import sys

    objs = sorted(glob.glob(os.path.join(REPO, "mdgen_finetune_amd", "csrc", "*.o")))
    if not objs or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("build the library first (make -C mdgen_finetune_amd/csrc)")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import lds_barrier_scan as S

    bad = []
    for o in objs:
        bad += [(os.path.basename(o),) + f for f in S.scan(S.disassemble(o))]
    assert not bad, bad[:5]
