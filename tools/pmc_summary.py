"""Per launch shape (kernel, grid) averages of rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ
counters), with HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024; the gfx950 FETCH correction
of MI355X_MICROARCH.md §HBM) and the SQ split of wave cycles (parked / issue-stalled / issuing),
VALU per MFMA and the MFMA pipe's busy fraction.
Usage: python tools/pmc_summary.py DIR [kernel regex]  (DIR holds *_counter_collection.csv)"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if not rx.search(r["Kernel_Name"]):
            continue
        short = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        short = re.sub(r"\(.*", "", short).replace("void ", "")[:56]
        key = (short, int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])))
        per[(key, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for (key, _), cs in per.items():
        for c, v in cs.items():
            acc[key][c].append(v)


def avg(cs, c):
    v = cs.get(c)
    return sum(v) / len(v) if v else None


print("| kernel | grid | launches | HBM MB (2F+W) | WAIT_ANY % | WAIT_INST % | issuing % | VALU/MFMA | MFMA busy % | clock GHz |")
print("|---|---|---|---|---|---|---|---|---|---|")
for key, cs in sorted(acc.items(), key=lambda kv: -(avg(kv[1], "SQ_WAVE_CYCLES") or 0)):
    f, w = avg(cs, "FETCH_SIZE"), avg(cs, "WRITE_SIZE")
    hbm = f"{(2 * f + w) * 1024 / 1e6:.1f}" if f is not None and w is not None else "-"
    wc, wa, wi, ai = (avg(cs, c) for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
    split = [f"{100 * x / wc:.0f}" if (wc and x is not None) else "-" for x in (wa, wi, ai)]
    va, mf = avg(cs, "SQ_INSTS_VALU"), avg(cs, "SQ_INSTS_MFMA")
    ratio = f"{va / mf:.1f}" if va and mf else "-"
    busy, gui = avg(cs, "SQ_VALU_MFMA_BUSY_CYCLES"), avg(cs, "GRBM_GUI_ACTIVE")
    sqb = avg(cs, "SQ_BUSY_CYCLES")
    mb = f"{100 * busy / (gui / 8 * 256 * 4) :.0f}" if busy and gui else "-"
    n = max(len(v) for v in cs.values())
    print(f"| `{key[0]}` | {key[1]} | {n} | {hbm} | {' | '.join(split)} | {ratio} | {mb} | - |")
