"""Summarise a rocprofv3 kernel trace of `bench.py --train --train-rccl1` (the graphed training
step with its per-bucket RCCL all-reduces captured in the graph): for every collective kernel of
the last replayed steps, when it started within the step, how long it ran, which library kernels
ran concurrently with it (overlap with backward) and how many kernels of the step started after
it.  Usage: python tools/rccl_overlap_trace.py <kernel_trace.csv> <buckets per step> [out.md]
[bucket bytes, comma-separated: a world-1 trace with MDG_BUCKET_MARK=1 markers]"""
import csv
import re
import sys


def main():
    path, nb = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    is_coll = [("nccl" in n.lower() or "rccl" in n.lower()) for _, _, n in rows]
    coll = [i for i, c in enumerate(is_coll) if c]
    if len(sys.argv) > 4:  # bucket sizes (bytes, comma-separated): the marked world-1 trace
        return world1_marked(path, rows, nb, out, [int(x) for x in sys.argv[4].split(",")])
    if len(coll) < nb:
        # world 1: RCCL elides a one-rank all-reduce (no collective kernel); the bucket's packing
        # `cat`, issued by the same hook on the same branch right before the collective, marks when
        # each bucket left backward
        return world1(path, rows, nb, out)
    nsteps = len(coll) // nb
    lines = [f"# In-graph RCCL bucket all-reduces ({path.split('/')[-1]})", "",
             f"{len(rows)} kernels, {len(coll)} collective kernels, {nb} buckets per step, {nsteps} steps traced.", ""]
    for s in range(max(0, nsteps - 2), nsteps):
        idx = coll[s * nb:(s + 1) * nb]
        # the step's window: from the kernel after the previous step's last collective (or the
        # trace start) to the step's last collective's end plus the optimizer tail
        lo = coll[s * nb - 1] + 1 if s > 0 else 0
        hi = coll[(s + 1) * nb] if s + 1 < nsteps else len(rows)
        t0 = rows[lo][0]
        lines += [f"## step {s} ({hi - lo} kernels, {(rows[hi - 1][1] - t0) / 1e3:.1f} us)", "",
                  "| bucket | start (us into step) | duration (us) | concurrent kernels | step kernels started after it | concurrent examples |",
                  "|---|---|---|---|---|---|"]
        for b, i in enumerate(idx):
            st, en, name = rows[i]
            conc = [rows[j][2] for j in range(lo, hi) if not is_coll[j] and rows[j][0] < en and rows[j][1] > st]
            after = sum(1 for j in range(i + 1, hi) if not is_coll[j])
            ex = sorted(set(n.split("(")[0][:40] for n in conc))[:3]
            lines.append(f"| {b} | {(st - t0) / 1e3:.1f} | {(en - st) / 1e3:.1f} | {len(conc)} | {after} | "
                         f"{', '.join(ex)} |")
        lines.append("")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


def world1_marked(path, rows, nb, out, sizes):
    """MDG_BUCKET_MARK=1 trace: one spin marker kernel per bucket, issued on the side branch right
    before the bucket's all-reduce; with the bucket sizes (bench JSON) this gives the bytes that
    leave backward in its last 0.5 ms (the part of the exchange nothing overlaps)."""
    marks = [i for i, (_, _, n) in enumerate(rows) if "prep_latents" in n]
    lo, hi = marks[-2], marks[-1]
    t0 = rows[lo][0]
    spins = [i for i in range(lo, hi) if "spin" in rows[i][2].lower()]
    bwd_end = max((rows[i][1] for i in range(lo, hi) if ("bwd" in rows[i][2] or "wgrad" in rows[i][2]
                                                         or "unpack" in rows[i][2])), default=rows[hi - 1][1])
    lines = [f"# In-graph bucket all-reduces, world-1 rehearsal with bucket markers ({path.split('/')[-1]})", "",
             f"Last complete step {(rows[hi - 1][1] - t0) / 1e3:.1f} us; backward's last kernel ends "
             f"{(bwd_end - t0) / 1e3:.1f} us into it; {len(spins)} bucket markers ({nb} buckets).", "",
             "| bucket | MB | leaves backward at (us into step) | backward left after it (us) |", "|---|---|---|---|"]
    tail = 0.0
    for b, i in enumerate(spins):
        st = rows[i][0]
        left = (bwd_end - st) / 1e3
        mb = sizes[b] / 1e6 if b < len(sizes) else float("nan")
        if left <= 500.0:
            tail += mb
        lines.append(f"| {b} | {mb:.2f} | {(st - t0) / 1e3:.1f} | {left:.1f} |")
    lines += ["", f"**{tail:.2f} MB leave backward in its last 0.5 ms** (of {sum(sizes) / 1e6:.1f} MB bucketed)."]
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


def world1(path, rows, nb, out):
    marks = [i for i, (_, _, n) in enumerate(rows) if "prep_latents" in n]
    lo, hi = marks[-2], marks[-1]  # the last complete replayed step
    t0, t1 = rows[lo][0], rows[hi - 1][1]
    bwd0 = min((i for i in range(lo, hi) if "wgrad" in rows[i][2]), default=lo)  # backward's first dW
    pack = lambda n: "CatArrayBatchedCopy" in n or "TensorListMetadata<2>" in n  # noqa: E731  (cat / foreach copy)
    cats = [i for i in range(bwd0, hi) if pack(rows[i][2])]
    bwd_end = max((rows[i][1] for i in range(lo, hi) if "adam" not in rows[i][2]
                   and ("bwd" in rows[i][2] or "wgrad" in rows[i][2])), default=t1)
    lines = [f"# In-graph bucket all-reduces, world-1 rehearsal ({path.split('/')[-1]})", "",
             "A one-rank RCCL all-reduce launches no collective kernel, so this trace cannot show the "
             "collectives themselves; each bucket's packing copy (a foreach copy into the bucket's slice: one or "
             "more multi-tensor launches, issued by the same post-accumulate hook right before the bucket's "
             "all-reduce) marks when the bucket left backward.",
             f"Last complete step: {hi - lo} kernels, {(t1 - t0) / 1e3:.1f} us; backward's last kernel "
             f"ends {(bwd_end - t0) / 1e3:.1f} us into the step; {nb} buckets expected.", "",
             "| packing kernel | start (us into step) | duration (us) | step kernels started after it |",
             "|---|---|---|---|"]
    for i in cats:
        st, en, name = rows[i]
        short = re.search(r"CatArrayBatchedCopy\w*|multi_tensor_apply_kernel", name).group(0)
        lines.append(f"| `{short}` | {(st - t0) / 1e3:.1f} | {(en - st) / 1e3:.1f} | {hi - i - 1} |")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
