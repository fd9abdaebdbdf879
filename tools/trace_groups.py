"""Group the kernels of one replayed training step (rocprofv3 kernel trace, tools/gpu_train_prof.sh)
by (kernel, grid, block, VGPRs, LDS) with total / average durations: which launch shape costs what.
Usage: python tools/trace_groups.py [trace.csv] [regex]"""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_train/run_kernel_trace.csv"
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "prep_latents" in r["Kernel_Name"]]
seg = rows[marks[-2]:marks[-1]] if len(marks) >= 2 else rows
g = collections.defaultdict(list)
for r in seg:
    n = r["Kernel_Name"]
    if not rx.search(n):
        continue
    short = re.sub(r"\(anonymous namespace\)::", "", n)
    short = re.sub(r"\(.*", "", short).replace("void ", "")[:60]
    grid = tuple(int(r[f"Grid_Size_{a}"]) // max(1, int(r[f"Workgroup_Size_{a}"])) for a in "XYZ")
    k = (short, grid, int(r["Workgroup_Size_X"]), r["VGPR_Count"], r["LDS_Block_Size"])
    g[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in g.values())
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):8.1f}us n={len(v):3d} avg={sum(v) / len(v):7.1f}  {k[0]} grid={k[1]} wg={k[2]} vgpr={k[3]} lds={k[4]}")
print(f"total {tot:.1f} us")
