"""Copy the judged rocprof summaries from gpurun_out/ into profiles/ (tracked) for round RR:
  profiles/rRR_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `bench.py --steps 3`
  profiles/rRR_summary.md         per-kernel table (calls, avg us, share)
  profiles/traffic_rRR.json       HBM bytes per launch of the bench roofline kernels from the
                                  FETCH_SIZE / WRITE_SIZE passes (tools/roof_pmc.sh): KiB
                                  counters x 1024, FETCH_SIZE doubled (gfx950: FETCH_SIZE
                                  reports half the bytes of 16-B/lane streaming reads,
                                  MI355X_MICROARCH.md §HBM); mean of the last 50 dispatches
                                  (the roofline timing loop).
Usage: python tools/make_profiles.py RR [B T L]
With a non-default B T L only the traffic of that shape (gpurun_out/pmc_roof_B_T_L, from
ROOF_ARGS="B T L" bash tools/roof_pmc.sh) is merged into traffic_rRR.json."""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rr = sys.argv[1]
B, T, L = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (8, 1000, 4)
out = os.path.join(REPO, "profiles")
os.makedirs(out, exist_ok=True)

default_shape = (B, T, L) == (8, 1000, 4)
pmc_dir = os.path.join(REPO, "gpurun_out", "pmc_roof" if default_shape else f"pmc_roof_{B}_{T}_{L}")
stats = os.path.join(REPO, "gpurun_out", "prof", "run_kernel_stats.csv")
if os.path.exists(stats) and default_shape:
    shutil.copy(stats, os.path.join(out, f"r{rr}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    lines = [f"# r{rr}: rocprofv3 --kernel-trace --stats, `python bench.py --steps 3 --warmup 1 --no-cpu-baseline`",
             "", "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in rows[:20]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['Percentage']):.2f} |")
    trace = os.path.join(REPO, "gpurun_out", "prof", "run_kernel_trace.csv")
    if os.path.exists(trace):
        # bench.roofline times each roofline kernel in a loop of 50 launches after the timed
        # windows (plus one warm-up launch): those are the last 50 dispatches of its name; the
        # rest ran inside the hipGraph windows.
        pats = (("mlp_rowln_kernel", "mlp_fused"), ("mlp_ws2_kernel", "mlp_fused"), ("rowln_qkv_kernel", "rowln_qkv"), ("gemm_rowln_kernel", "gemm_out_proj_rowln"),
                ("gemm_bf16_b4_kernel<2", "gemm_qkv_temporal"), ("attn_temporal_bf16", "attn_temporal"))
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(trace)):
            for pat, name in pats:
                if pat in r["Kernel_Name"]:
                    per[name].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        bench_live, work = {}, {}
        bl = os.path.join(REPO, "gpurun_out", "prof", "bench_prof.log")
        if os.path.exists(bl):
            try:
                d = json.loads([x for x in open(bl).read().splitlines() if x.startswith("{")][-1])
                for rf in [d["roofline"]] + d.get("roofline_more", []):
                    bench_live[rf["kernel"]] = rf["avg_launch_us"]
                    work[rf["kernel"]] = (rf.get("flops_per_launch"), rf.get("bytes_per_launch"))
            except Exception:
                pass
        lines += ["", "## Bench roofline kernels: rocprof vs the bench's live HIP-event timing",
                  "", "| roofline kernel | rocprof avg of the 50 timed dispatches (us) | bench live avg (us) | in-graph avg, every "
                  "launch of this kernel name (us) | in-graph estimate for this launch (us) | in-graph fraction of the "
                  "MFMA roof (2.5 PF) / of HBM (8 TB/s), algorithmic work |",
                  "|---|---|---|---|---|---|"]
        for name in dict.fromkeys(n for _, n in pats):
            v = sorted(per.get(name, []))
            if len(v) < 60:
                continue
            loop = [x[1] for x in v[-50:]]
            graph = [x[1] for x in v[:-51]]
            # (with the fused MLP the row-LN kernel serves only out_proj, x2 per layer)
            g = sum(graph) / len(graph)
            fl, by = work.get(name, (None, None))
            fr = (f"{fl / (g * 1e-6) / 2.5e15:.3f} / {by / (g * 1e-6) / 8e12:.3f}" if fl and by else "n/a")
            lines.append(f"| {name} | {sum(loop) / len(loop):.1f} | {bench_live.get(name, 'n/a')} | "
                         f"{g:.1f} | {g:.1f} | {fr} |")
    open(os.path.join(out, f"r{rr}_summary.md"), "w").write("\n".join(lines) + "\n")

# each roofline kernel's last 50 dispatches are its bench.roofline timing loop (the row-LN
# family's: the out_proj one; the fc2 one when the MLP is not fused)
KMAP = {"gemm_bf16_b4_kernel<2": "gemm_qkv_temporal", "attn_temporal_bf16": "attn_temporal",
        "gemm_rowln_kernel": "gemm_out_proj_rowln", "mlp_rowln_kernel": "mlp_fused", "mlp_ws2_kernel": "mlp_fused",
        "rowln_qkv_kernel": "rowln_qkv"}
res = collections.defaultdict(dict)
for cname, scale in (("FETCH_SIZE", 2 * 1024), ("WRITE_SIZE", 1024)):
    p = os.path.join(pmc_dir, f"{cname}_counter_collection.csv")
    if not os.path.exists(p):
        continue
    shutil.copy(p, os.path.join(out, f"r{rr}_pmc_{cname}{'' if default_shape else f'_B{B}_T{T}_L{L}'}.csv"))
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        for pat, name in KMAP.items():
            if pat in r["Kernel_Name"]:
                by[name].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for name, v in by.items():
        v.sort()
        last = [x[1] for x in v[-50:]]
        res[name][cname] = sum(last) / len(last) * scale
tpath = os.path.join(out, f"traffic_r{rr}.json")
traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}  # (other shapes' entries kept)
for name, d in res.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        e = traffic.setdefault(name, {})
        e[f"B{B}_T{T}_L{L}_bf16"] = round(d["FETCH_SIZE"] + d["WRITE_SIZE"])
        sfx = "" if default_shape else f"_B{B}_T{T}_L{L}"
        e["read_bytes" + sfx], e["write_bytes" + sfx] = round(d["FETCH_SIZE"]), round(d["WRITE_SIZE"])
if traffic:
    json.dump(traffic, open(tpath, "w"), indent=1)
print(json.dumps(traffic, indent=1))
