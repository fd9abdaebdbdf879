"""Summarise the rocprofv3 kernel trace of the graphed training step (tools/gpu_train_prof.sh)
into profiles/rRR_train_kernels.md: one replayed step (between two prep_latents dispatches),
its kernel count and busy time by origin, and the top kernels.
Usage: python tools/train_profile_md.py RR [trace.csv]"""
import collections
import csv
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rr = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "prof_train", "run_kernel_trace.csv")
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "prep_latents" in r["Kernel_Name"]]
seg = rows[marks[-2]:marks[-1]]  # the last complete replay


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def origin(n):
    return "libmdgen_hip" if "mdg" in n else ("hipBLASLt" if n.startswith("Cijk") else "PyTorch / runtime")


span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
busy = sum(map(dur, seg)) / 1e6
by = collections.defaultdict(lambda: [0, 0])
per = collections.defaultdict(lambda: [0, 0])
for r in seg:
    o = by[origin(r["Kernel_Name"])]
    o[0] += 1
    o[1] += dur(r)
    k = re.sub(r"\s+", " ", r["Kernel_Name"])[:100]
    per[k][0] += 1
    per[k][1] += dur(r)
out = [f"# r{rr}: one replay of the graphed training step (bench.py --train --batch 8, B=8 T=1000 L=4)",
       "", f"rocprofv3 --kernel-trace of tools/gpu_train_prof.sh; the last complete replay: {len(seg)} kernels, "
       f"span {span:.2f} ms, busy {busy:.2f} ms (the profiler adds ~10 % to the bench's wall time).", "",
       "| origin | kernels | ms |", "|---|---|---|"]
for k, (n, t) in sorted(by.items(), key=lambda kv: -kv[1][1]):
    out.append(f"| {k} | {n} | {t / 1e6:.2f} |")
out += ["", "| kernel | calls | ms | avg us |", "|---|---|---|---|"]
for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:30]:
    out.append(f"| `{k}` | {n} | {t / 1e6:.3f} | {t / n / 1e3:.1f} |")
out += ["", "Every kernel not from libmdgen_hip (names to 160 characters):", "",
        "| kernel | calls | ms | avg us |", "|---|---|---|---|"]
lib = collections.defaultdict(lambda: [0, 0])
for r in seg:
    if origin(r["Kernel_Name"]) != "libmdgen_hip":
        k = re.sub(r"\s+", " ", r["Kernel_Name"])[:160]
        lib[k][0] += 1
        lib[k][1] += dur(r)
for k, (n, t) in sorted(lib.items(), key=lambda kv: -kv[1][1]):
    out.append(f"| `{k}` | {n} | {t / 1e6:.3f} | {t / n / 1e3:.1f} |")
dst = os.path.join(REPO, "profiles", f"r{rr}_train_kernels.md")
open(dst, "w").write("\n".join(out) + "\n")
print(dst)
