"""Static check of the gfx950 code objects: LDS operations still in flight at an s_barrier.

A kernel that refills an LDS ring slot by LDS DMA (global_load_lds) right after a raw
s_barrier relies on every wave having RETIRED its reads of that slot before the barrier.  The
compiler may move the last MFMAs of a K-step (and the s_waitcnt lgkmcnt guarding their
operands) below the barrier, leaving ds_reads in flight across it; a DMA write issued by
another wave after the barrier then races them (a rare, load-dependent wrong tile).  Round 3
found two kernels doing this (gemm.hip kRingWaitNote).

This scans straight-line code backwards from every s_barrier to the previous s_waitcnt that
carries an lgkmcnt: DS operations issued after that wait, or a wait of lgkmcnt(N > 0), are
reported.  A branch (s_branch / s_cbranch / a label) ends the scan without a verdict.

usage: python tools/lds_barrier_scan.py FILE.s|FILE.o ...   (exit 1 if anything is flagged)
       .o files (hipcc objects) are unbundled and disassembled with the ROCm LLVM tools.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj):
    """gfx950 disassembly of a hipcc object (its .hip_fatbin offload bundle)."""
    heads = subprocess.check_output([f"{LLVM}/llvm-objdump", "-h", obj], text=True)
    if ".hip_fatbin" not in heads:
        return ""  # host-only object (capi.o)
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.devnull])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", co], text=True)


KERNEL = re.compile(r"^(?:[0-9a-f]+ <)?(_Z\w+)>?:")
DS = re.compile(r"^ds_(read|load|write|store|bpermute|swizzle|add|max|min)")
WAIT = re.compile(r"^s_waitcnt\b.*lgkmcnt\((\d+)\)")
STOP = re.compile(r"^(s_branch|s_cbranch\w*|s_setpc|s_endpgm)\b|^\.LBB\w*:")


def scan(text):
    lines = [ln.split("//")[0].split(";")[0].strip() for ln in text.split("\n")]
    kern, out = None, []
    for i, s in enumerate(lines):
        m = KERNEL.match(s)
        if m:
            kern = m.group(1)
            continue
        if not s.startswith("s_barrier"):
            continue
        n = 0
        for j in range(i - 1, max(0, i - 3000), -1):
            t = lines[j]
            w = WAIT.match(t)
            if w:
                if n or int(w.group(1)):
                    out.append((kern, i + 1, f"{n} DS op(s) after s_waitcnt lgkmcnt({w.group(1)})"))
                break
            if STOP.match(t) or KERNEL.match(t):
                break
            if DS.match(t):
                n += 1
    return out


def main(paths):
    bad = []
    for p in paths:
        text = disassemble(p) if p.endswith(".o") else open(p).read()
        for kern, line, why in scan(text):
            bad.append(f"{os.path.basename(p)}: {kern} (line {line}): {why}")
    for b in bad:
        print(b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
