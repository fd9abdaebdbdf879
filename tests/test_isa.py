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


def test_no_three_dword_global_accesses():
    """No kernel issues a 12-byte global / buffer access (global_load_dwordx3 and kin): the
    compiler forms them by merging dword loads of 3-float records (rots / trans rows, 7- and
    21-float latents) at 4-B alignment, the misaligned-vector class of DESIGN.md §4.  Those
    kernels read such records through ld1 / st1 (common.h), which the vectoriser never merges."""
    import re
    import sys

    objs = sorted(glob.glob(os.path.join(REPO, "mdgen_finetune_amd", "csrc", "*.o")))
    if not objs or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("build the library first (make -C mdgen_finetune_amd/csrc)")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import lds_barrier_scan as S

    pat = re.compile(r"\b(global|buffer|flat)_(load|store)_dwordx3\b")
    hits = []
    for o in objs:
        kern = None
        for ln in S.disassemble(o).split("\n"):
            m = S.KERNEL.match(ln.strip())
            if m:
                kern = m.group(1)
            if pat.search(ln):
                hits.append((os.path.basename(o), kern, ln.strip()))
    assert not hits, hits[:5]
