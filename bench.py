#!/usr/bin/env python
"""Benchmark: denoised frames/sec of MDGen's forward-sim denoising on MI355X.

Workload (BASELINE.json configs[1]): tetrapeptide forward simulation, num_frames T=1000,
crop L=4, default model (5 layers, C=384, 16 heads, IPA prepend), bf16 GEMM/attention
operands, synthetic seed-derived weights and inputs (no checkpoint/dataset offline).

One bench "step" = one sim_inference rollout window: Sampler.sample_ode('euler', 50) over
B trajectories of T frames = 49 Euler denoising steps (each a full forward + Euler update)
plus the window's conditioning precompute, through the drop-in engine call
(HipEngine.sample_euler: input staging + one hipGraph replay + output copy).  Default
B=16 trajectories per GPU, run as 2 concurrent 8-trajectory chains ("lanes": parallel
branches of the one hipGraph, engine._run_lanes).
value = frames denoised per second = ranks * B * T * 49 * steps / max-over-ranks time.

Multi-GPU (--gpus N > 1): inference does not shard (temporal attention couples all T frames of
a trajectory), so N ranks run N independent replicas of the window ("replicas only", scaling
"weak"); no collective on the data path.  The path that does shard is config 3's training
(DDP, /root/reference/src/train.py:46-60), so an N-GPU line also carries a "train_dp" object:
the graphed GVP training step at B=8 per GPU x T=1000, gradients averaged over RCCL (bucket
all-reduces captured in the step's graph, replicated conditioning on its own communicator).
Launch: with no launcher environment this process is an orchestrator that never touches the
GPU: it spawns one worker process per GPU per leg (inference, then train_dp), each on
cuda:LOCAL_RANK with its own RCCL group, waits for them (bounded), and prints ONE line.  Under
torch.distributed.run (WORLD_SIZE set; must equal --gpus) each launched process orchestrates
its own rank's workers the same way.  A train_dp leg that fails or times out is reported as
such in the line; the inference line stands.

Extra fields: "roofline" for the dominant kernel (the fused MLP, mlp_ws2_kernel: fc1 +
GELU + fc2 + gated residual + next LN in one launch, the largest share of the step per
profiles/; live HIP-event timing on the stream the kernel runs on; with MDG_FUSED_MLP=0 the
fc2 row-LN GEMM instead), "roofline_more" for the next ones (the out_proj row-LN GEMM, the
temporal q|k|v GEMM, the temporal attention), "cpu_baseline" (the oracle restatement timed on
this host's cores).  Each roofline entry is priced against its BINDING roof: algorithmic
FLOPs / 2.5 PF vs algorithmic bytes / 8 TB/s, whichever is longer ("bound"); both fractions
are reported ("mfma_frac", "hbm_frac") with the kernel's arithmetic intensity.
"""
import argparse
import ctypes
import json
import math
import os
import signal
import subprocess
import sys
import tempfile
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
ROUND = "06"  # the round whose profiles/ files (summary, PMC traffic) this bench line cites
sys.path.insert(0, REPO)

PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}   # MI355X dense MFMA (MI355X_MICROARCH.md:42-43)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed rollout windows")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="trajectories per GPU")
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--crop", type=int, default=4)
    ap.add_argument("--num-steps", type=int, default=50, help="ODE grid points (49 Euler steps)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--lanes", type=int, default=2, help="concurrent sub-batch chains per window (streams)")
    ap.add_argument("--sweep-batches", default="1,8,32",
                    help="extra per-GPU batch sizes timed beside the headline (comma list, '' = none)")
    ap.add_argument("--no-f32-line", action="store_true", help="skip the fp32-operand (parity path) line")
    ap.add_argument("--sweep-steps", type=int, default=2, help="timed windows per sweep / f32 line")
    ap.add_argument("--sampler", default="euler", choices=["euler", "dopri5"],
                    help="dopri5: an evidence line for the reference's DEFAULT sampler (parsing.py:102): one "
                         "window = Sampler.sample_ode() (adaptive dopri5, atol 1e-6 / rtol 1e-3, 50 saved points) "
                         "with every adaptive step one hipGraph replay; reports NFE and accepted / rejected steps")
    ap.add_argument("--model-args", default="",
                    help="--train only: extra model flags, e.g. '--embed_dim 256 --mha_heads 8' (head_dim 32); "
                         "the line then carries no step roofline (its FLOP model is the default model's)")
    ap.add_argument("--train", action="store_true",
                    help="BASELINE config 3 evidence line: the GVP training step (forward + loss + backward + "
                         "clip + Adam + EMA, the HIP block stack, graphed) at B trajectories x T frames per GPU "
                         "(use --batch 8); ranks average gradients over RCCL")
    ap.add_argument("--no-cond-gather", action="store_true",
                    help="--train-rccl1: bucket every gradient (no replicated conditioning, cond_dist.py)")
    ap.add_argument("--train-rccl1", action="store_true",
                    help="with --train at one GPU: a world-1 RCCL group with the gradient reduction forced on, "
                         "so the step's graph carries its per-bucket all-reduces (rehearsal of the N-GPU step)")
    ap.add_argument("--train-batch", type=int, default=8, help="trajectories per GPU of the N-GPU line's train_dp leg")
    ap.add_argument("--no-train-dp", action="store_true", help="N > 1: skip the train_dp leg")
    ap.add_argument("--leg-timeout", type=float, default=900.0, help="s: bound on the primary leg's workers")
    ap.add_argument("--train-dp-timeout", type=float, default=360.0, help="s: bound on the train_dp leg's workers")
    ap.add_argument("--tps", action="store_true",
                    help="TPS / interpolation model (BASELINE config 4: --tps_condition, latent 28, start + end "
                         "frames conditioned; use with --frames 100); an evidence line, not the headline")
    return ap.parse_args()


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def make_model(T, L, seed=0, tps=False):
    import argparse as ap_

    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.model.latent_model import LatentMDGenModel

    args = ap_.Namespace(embed_dim=384, mha_heads=16, num_layers=5, ipa_heads=4, ipa_head_dim=32, ipa_qk=8,
                         ipa_v=8, dropout=0.0, no_rope=False, prepend_ipa=True, abs_pos_emb=True, crop=L,
                         num_frames=T, time_multiplier=100.0, sim_condition=not tps, tps_condition=tps)
    m = LatentMDGenModel(args, 28 if tps else 21).eval()
    synthetic.fill_module_(m, seed)
    return m


def inputs(B, T, L, seed, device, tps=False):
    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    inp = synthetic.make_inputs(seed, B, T, L, 28 if tps else 21, tps=tps)
    g = lambda k: torch.from_numpy(inp[k]).to(device)  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    if tps:
        kw["end_frames"] = Rigid(Rotation(rot_mats=g("end_rots")), g("end_trans"))
    return g("x"), kw, inp


def time_kernel(fn, iters=20):
    """Average device time of fn() (launches on the current stream) via HIP events."""
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def _traffic(kernel, B, T, L, dtype):
    """HBM bytes per launch from the committed PMC passes (profiles/traffic_r{ROUND}.json, this
    round's tools/roof_pmc.sh; shapes or kernels it lacks from the earlier rounds' files of the same
    kernels): FETCH_SIZE x2 + WRITE_SIZE per the gfx950 correction of MI355X_MICROARCH.md §HBM, or None."""
    for rr in (ROUND, "05", "04", "03"):
        try:
            v = json.load(open(os.path.join(REPO, "profiles", f"traffic_r{rr}.json")))[kernel].get(f"B{B}_T{T}_L{L}_{dtype}")
        except Exception:
            v = None
        if v is not None:
            return v
    return None


def roofline(eng, st, dtype, B, T, L):
    """Rooflines of the launches that dominate the step, at the shape they run with in the
    timed region (B = one lane's trajectories), launched exactly as in the step (same
    workspace buffers, layer-0 weights) and timed with HIP events on their stream:
      * attn_temporal — the largest launch type per step (profiles/r01_summary.md):
        4*B*L*H*T*(T+1)*D FLOPs (QK^T and PV over T+1 keys incl. the bias row, unpadded D);
      * gemm_qkv_temporal — 2*M*N*K with M = B*T*L, N = 3C, K = C (+ RoPE/scatter epilogue);
      * gemm_fc2_rowln — fc2 with the gated residual + LayerNorm epilogue, 2*M*C*4C (the
        MLP's second GEMM when the MLP is not fused);
      * mlp_fused — fc1 + GELU + fc2 + gated residual + LN in one kernel, 4*M*C*4C;
      * gemm_out_proj_rowln — out_proj + gated residual + LN, 2*M*C*C;
      * rowln_qkv — the spatial out_proj + gated residual + LN_t and the temporal q|k|v in one
        kernel (LN_t(h) on chip), 2*M*C*C + 2*M*3C*C."""
    from mdgen_finetune_amd import _lib

    lib, P = eng.lib, eng._packed
    ws = st.ws.data_ptr()
    off = _lib.workspace_offsets(st.dims)
    H, D, C = eng.H, eng.D, eng.C
    N = B * T * L
    s = _lib.stream_handle()
    kvb = st.kvb[0][1]

    # the planes as the step stores them (packed: row stride D, bf16 with D % 8 == 0)
    packed = eng.describe_plan(B, T, L).get("planes", "").startswith("packed")
    attn_fn = lib.mdg_attn_temporal_packed if packed else lib.mdg_attn_temporal

    def attn():
        _lib.check(attn_fn(eng.mdg_dtype, B, T, L, H, D, ws + off["qkv_t"], ws + off["kbias"], kvb.data_ptr(),
                           ws + off["o"], s), "attn_temporal")

    g = _lib.MdgGemmDesc()
    g.dtype, g.a_mode, g.epi, g.M, g.N, g.K = eng.mdg_dtype, _lib.MDG_A_PLAIN, _lib.MDG_EPI_QKV, N, 3 * C, C
    g.A, g.lda = ws + off["xn"], C
    g.W, g.ldw, g.bias = P["layers"][0]["wqkv1"].data_ptr(), C, P["layers"][0]["bqkv1"].data_ptr()
    g.qkv_layout = _lib.MDG_QKV_TEMPORAL_PACKED if packed else _lib.MDG_QKV_TEMPORAL
    g.qkv_out, g.H, g.D, g.T, g.L = ws + off["qkv_t"], H, D, T, L
    g.qscale = D ** -0.5 * math.log2(math.e)
    g.rope, g.rope_rows = _lib.ptr(st.rope_t), T + 1

    def gemm():
        _lib.check(lib.mdg_gemm(ctypes.byref(g), s), "qkv gemm")

    # fc2 + gated residual + LN of the next consumer (its own scratch residual / mods)
    mods = torch.zeros(B, 9 * C, device=st.h.device)
    h_scratch = torch.zeros_like(st.h)
    f = _lib.MdgGemmDesc()
    f.dtype, f.a_mode, f.epi, f.M, f.N, f.K = eng.mdg_dtype, _lib.MDG_A_PLAIN, _lib.MDG_EPI_GATE_RES, N, C, 4 * C
    f.A, f.lda = ws + off["hid"], 4 * C
    f.W, f.ldw, f.bias = P["layers"][0]["w2"].data_ptr(), 4 * C, P["layers"][0]["b2"].data_ptr()
    f.resid, f.ldr, f.gate, f.gate_off = h_scratch.data_ptr(), C, mods.data_ptr(), 8 * C
    f.mod_stride, f.rows_per_mod = 9 * C, T * L
    f.xn_out, f.xn_mods, f.xn_mod_stride, f.xn_shift_off, f.xn_scale_off = ws + off["xn"], mods.data_ptr(), 9 * C, 0, C
    f.ln_eps = 1e-6

    def fc2():
        _lib.check(lib.mdg_gemm(ctypes.byref(f), s), "fc2 rowln gemm")

    # the fused MLP with the same fc2 descriptor and the fc1 one the step builds
    f1 = _lib.MdgGemmDesc()
    f1.dtype, f1.a_mode, f1.epi, f1.act, f1.M, f1.N, f1.K = eng.mdg_dtype, _lib.MDG_A_PLAIN, _lib.MDG_EPI_STORE, 1, N, 4 * C, C
    f1.A, f1.lda = ws + off["xn"], C
    f1.W, f1.ldw, f1.bias = P["layers"][0]["w1"].data_ptr(), C, P["layers"][0]["b1"].data_ptr()
    f1.out, f1.ldo = ws + off["hid"], 4 * C

    def mlp():
        _lib.check(lib.mdg_mlp_fused(ctypes.byref(f1), ctypes.byref(f), s), "mlp fused")

    # out_proj + gated residual + LN (K = C), the same row-LN kernel as fc2
    o = _lib.MdgGemmDesc()
    ctypes.memmove(ctypes.byref(o), ctypes.byref(f), ctypes.sizeof(f))
    o.K, o.A, o.lda = C, ws + off["o"], C
    o.W, o.ldw, o.bias = P["layers"][0]["wo1"].data_ptr(), C, P["layers"][0]["bo1"].data_ptr()

    def out_proj():
        _lib.check(lib.mdg_gemm(ctypes.byref(o), s), "out_proj rowln gemm")

    def rowln_qkv():
        _lib.check(lib.mdg_rowln_qkv(ctypes.byref(o), ctypes.byref(g), s), "rowln_qkv")

    # algorithmic bytes per launch: every operand read once + every output written once, in the
    # path's storage types (bf16 activations / weights, fp32 residual stream), head dim UNPADDED
    # (D = 24; the kernels' 32-wide pad is not counted), adaLN rows / biases / RoPE tables omitted
    cb = 2 if dtype == "bf16" else 4
    HD = H * D
    bytes_fc2 = N * 4 * C * cb + 2 * N * C * 4 + N * C * cb + 4 * C * C * cb   # hid, h r+w, xn, W2
    bytes_qkv = N * C * cb + 3 * N * HD * cb + 3 * C * C * cb                     # xn, q|k|v, Wqkv
    bytes_attn = 3 * N * HD * cb + N * HD * cb                                    # q|k|v, o
    bytes_mlp = N * C * cb + 2 * N * C * 4 + N * C * cb + 8 * C * C * cb          # xn, h r+w, xn out, W1+W2
    bytes_op = N * C * cb + 2 * N * C * 4 + N * C * cb + C * C * cb               # o, h r+w, xn out, Wo
    bytes_rq = N * C * cb + 2 * N * C * 4 + 3 * N * HD * cb + 4 * C * C * cb      # o, h r+w, q|k|v, Wo+Wqkv
    # (the bf16 step stores the planes packed: these are also the bytes it moves; the f32 path
    # pads D to 32 columns)
    out = {}
    fused, fused_qkv = _fusions(eng.describe_plan(B, T, L))
    kernels = [("mlp_fused", mlp, 4.0 * N * C * 4 * C, bytes_mlp)] if fused else \
        [("gemm_fc2_rowln", fc2, 2.0 * N * C * 4 * C, bytes_fc2)]
    if fused_qkv:  # (the temporal out_proj stays a row-LN GEMM)
        kernels += [("rowln_qkv", rowln_qkv, 8.0 * N * C * C, bytes_rq)]
    kernels += [("gemm_out_proj_rowln", out_proj, 2.0 * N * C * C, bytes_op)]
    if not fused_qkv:
        kernels += [("gemm_qkv_temporal", gemm, 2.0 * N * 3 * C * C, bytes_qkv)]
    kernels += [("attn_temporal", attn, 4.0 * B * L * H * T * (T + 1) * D, bytes_attn)]
    for name, fn, flops, nbytes in kernels:
        sec = time_kernel(fn, 50)
        # the binding roof: whichever of the MFMA time and the HBM time of the algorithmic work
        # is longer (arithmetic intensity below / above the ridge 2.5 PF / 8 TB/s = 312 FLOP/B)
        t_mfma, t_hbm = flops / (PEAK_TFLOPS[dtype] * 1e12), nbytes / (PEAK_HBM_GBS * 1e9)
        mfma_ach, hbm_ach = flops / sec / 1e12, nbytes / sec / 1e9
        if t_hbm > t_mfma:
            roof = {"bound": "hbm", "achieved": round(hbm_ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(hbm_ach / PEAK_HBM_GBS, 4)}
        else:
            roof = {"bound": "mfma", "achieved": round(mfma_ach, 2), "peak": PEAK_TFLOPS[dtype], "unit": "TFLOP/s",
                    "frac": round(mfma_ach / PEAK_TFLOPS[dtype], 4)}
        out[name] = {"kernel": name, **roof, "traffic": _traffic(name, B, T, L, dtype),
                     "avg_launch_us": round(sec * 1e6, 2), "flops_per_launch": flops, "bytes_per_launch": nbytes,
                     "intensity_flop_per_byte": round(flops / nbytes, 1),
                     "mfma_frac": round(mfma_ach / PEAK_TFLOPS[dtype], 4),
                     "hbm_frac": round(hbm_ach / PEAK_HBM_GBS, 4), "shape": f"B={B} T={T} L={L}",
                     "timing": "standalone: 50 back-to-back launches outside the graph, one lane's shape, the "
                               "step's workspace activations and layer-0 weights, zero adaLN rows; in the graph two "
                               f"lanes share the chip and each launch takes longer (in-graph averages: profiles/r{ROUND}_summary.md)"}
    return out


def max_over_ranks(el, world, device):
    """The job's time: the slowest rank's timed region (all_reduce MAX; identity at world 1)."""
    if world > 1:
        tt = torch.tensor([el], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = tt.item()
    return el


def job_value(world, B, T, n_euler, steps, el):
    """Whole-job frames/s: every rank denoises B*T frames per Euler step (replicas, weak
    scaling), over the max-over-ranks time."""
    return world * B * T * n_euler * steps / el


def step_model(B, T, L, C=384, H=16, nl=5, lat=21, dtype="bf16", fused_mlp=False, fused_qkv=False):
    """Algorithmic work of ONE denoise step (forward + Euler update) of B trajectories, from the
    model dims (counted 2*M*N*K per GEMM, 4*S*(S+1)*D per attention head-sequence):
      flops        — GEMMs 32*C^2 per token per layer + temporal attention 4*(T+1)*C per token
                     per layer + spatial 4*(L+1)*C + embedding / FinalLayer 4*lat*C per token
                     (the per-window IPA / adaLN precompute is excluded: x-independent, amortised
                     over 49 steps);
      design_bytes — the HBM bytes the kernel sequence of this build moves per step when every
                     kernel reads its operands once and writes its outputs once (DESIGN.md §3
                     per-kernel min bytes x launches): the data-flow floor of the unfused-layer
                     design, not of the model;
      floor_bytes  — model floor: bf16/f32 weights once + x in, x out (fp32)."""
    N = B * T * L
    D = C // H
    cb = 2 if dtype == "bf16" else 4
    flops = N * nl * (32.0 * C * C + 4.0 * (T + 1) * C + 4.0 * (L + 1) * C) + N * 4.0 * lat * C
    emb = N * (lat * 4 + C * 4 + C * 4 + C * cb)
    spatial = N * C * cb * 2
    rowln = N * (C * cb + 8 * C + C * cb)
    qkv = N * (C * cb + 3 * C * cb)
    attn = N * 4 * C * cb
    fc1 = N * (C * cb + 4 * C * cb)
    fc2 = N * (4 * C * cb + 8 * C + C * cb)
    if fused_mlp:  # the hidden activation never reaches HBM: xn in, h r+w, xn out
        fc1, fc2 = 0, N * (C * cb + 8 * C + C * cb)
    if fused_qkv:  # spatial out_proj + LN_t + temporal q|k|v in one kernel: LN_t(h) stays on chip
        qkv -= N * C * cb  # (and the out_proj's xn write, below)
    final = N * (C * cb + 3 * lat * 4)
    design = emb + nl * (spatial + 2 * rowln - (N * C * cb if fused_qkv else 0) + qkv + attn + fc1 + fc2) + final
    params = nl * 16 * C * C + 2 * lat * C
    floor = params * cb + N * lat * 4 * 2
    return {"flops": flops, "design_bytes": design, "floor_bytes": floor, "D": D}


def _fusions(plan):
    """(fused MLP, fused out_proj + q|k|v) of a kernel plan (mdg_describe_plan)."""
    return plan.get("mlp", "").startswith("mlp_fused"), plan.get("temporal", "").startswith("rowln_qkv")


def step_roofline(B, T, L, dtype, sec_per_denoise, fused_mlp=False, fused_qkv=False):
    """Whole-step position against both roofs (not one kernel): achieved TFLOP/s of the step's
    algorithmic FLOPs vs the dense MFMA peak, and achieved GB/s of the design's data flow vs HBM."""
    sm = step_model(B, T, L, dtype=dtype, fused_mlp=fused_mlp, fused_qkv=fused_qkv)
    tf = sm["flops"] / sec_per_denoise / 1e12
    gbs = sm["design_bytes"] / sec_per_denoise / 1e9
    t_mfma = sm["flops"] / (PEAK_TFLOPS[dtype] * 1e12)
    t_hbm = sm["design_bytes"] / (PEAK_HBM_GBS * 1e9)
    return {"flops_per_frame": round(sm["flops"] / (B * T), 1), "flops_per_denoise_step": sm["flops"],
            "achieved_tflops": round(tf, 1), "peak_tflops": PEAK_TFLOPS[dtype],
            "mfma_frac": round(tf / PEAK_TFLOPS[dtype], 4),
            "design_bytes_per_denoise_step": sm["design_bytes"], "achieved_gbs": round(gbs, 1),
            "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
            "design_floor_frac": round(max(t_mfma, t_hbm) / sec_per_denoise, 4),
            "binding": "hbm (design data flow)" if t_hbm > t_mfma else "mfma",
            "roof_frames_per_s_mfma": round(B * T / t_mfma, 1),
            "roof_frames_per_s_design_hbm": round(B * T / t_hbm, 1),
            "model_floor_bytes": sm["floor_bytes"]}


def time_windows(eng, zs, kw, num_steps, steps, warmup, use_graph=True):
    """Wall time of `steps` rollout windows (after `warmup`), inputs resident on the device."""
    for _ in range(max(1, warmup)):
        ys = eng.sample_euler(zs, num_steps=num_steps, use_graph=use_graph, **kw)
    torch.cuda.synchronize()
    assert torch.isfinite(ys[-1]).all(), "non-finite samples"
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.sample_euler(zs, num_steps=num_steps, use_graph=use_graph, **kw)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def sweep_line(dev, T, L, B, dtype, lanes, num_steps, steps, seed):
    """One extra (batch, dtype) point: frames/s and the step-level roofline."""
    from mdgen_finetune_amd.engine import get_engine

    m = make_model(T, L).to(dev)
    m.hip_dtype = dtype
    eng = get_engine(m)
    eng.lanes = lanes if (lanes > 1 and B % lanes == 0 and B >= 8) else 1
    zs, kw, _ = inputs(B, T, L, seed=seed, device=dev)
    with torch.no_grad():
        sec = time_windows(eng, zs, kw, num_steps, steps, 1)
    n_euler = num_steps - 1
    out = {"batch": B, "dtype": dtype, "lanes": eng.lanes, "value": round(B * T * n_euler / sec, 1),
           "unit": "frames/s", "ms_per_window": round(sec * 1e3, 3),
           "us_per_denoise_step": round(sec / n_euler * 1e6, 2),
           "step_roofline": step_roofline(B, T, L, dtype, sec / n_euler, *_fusions(eng.describe_plan(B // eng.lanes, T, L)))}
    del eng, m
    torch.cuda.empty_cache()
    return out


def cpu_baseline(T, L, seconds, tps=False):
    """The oracle (oracle/mdgen_oracle.py, fp32 PyTorch-CPU restatement pinned to the
    reference) timed on this host: forward + Euler update at B=1, T frames, L=4 (the TPS model
    with start + end frames for tps), repeated until `seconds` of CPU work."""
    from mdgen_finetune_amd import synthetic
    from oracle import mdgen_oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    lat = 28 if tps else 21
    c = O.Cfg(crop=L, latent_dim=lat, tps=tps)
    P = O.seeded_params(c, 0)
    inp = synthetic.make_inputs(1, 1, T, L, lat, tps=tps)
    f = lambda k: torch.from_numpy(inp[k])  # noqa: E731
    kw = dict(mask=f("mask"), rots=f("rots"), trans=f("trans"), x_cond=f("x_cond"), x_cond_mask=f("x_cond_mask"),
              aatype=f("aatype"))
    if tps:
        kw.update(end_rots=f("end_rots"), end_trans=f("end_trans"))
    x = f("x")
    dt = float(torch.linspace(0, 1, 50)[1])
    with torch.no_grad():
        O.forward(P, c, x, torch.zeros(1), **kw)  # warm
        n, t0 = 0, time.perf_counter()
        while True:
            v = O.forward(P, c, x, torch.zeros(1), **kw)
            x = x + dt * v
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= 50:
                break
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(T * n / el, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} denoising steps (oracle forward + Euler update{', TPS model' if tps else ''}), B=1 "
                      f"T={T} L={L}, fp32, {el:.1f} s on {threads} threads of {cpu}"}


def step_kernel_roofline(eng, B, T, L, dtype, lanes, zs, kw):
    """Small-M shapes (TPS T=100, B=1 windows) have no single dominant launch type (every
    launch is a few tiles; the MLP runs split over blocks with a reduction pass): the roofline
    unit is one whole denoise step (all its launches) of one lane, timed with HIP events on its
    stream, replayed standalone from the engine's state, priced at the step's algorithmic FLOPs."""
    from mdgen_finetune_amd import _lib

    Bl = B // lanes
    st = eng._state(Bl, T, L, lane=1 if lanes > 1 else 0)
    gs = next(iter(eng._graphs.values()))
    mods, mods_f, ipa = gs.cond
    lane_mods = mods[0] if lanes > 1 else mods
    io = eng._step_io(st, gs.states[0].data_ptr(), gs.states[1].data_ptr(), None,
                      None if ipa is None else ipa[0].data_ptr(), lane_mods[0].data_ptr(), mods_f[0].data_ptr(),
                      gs.dts[0], base=eng._states[(B, T, L, 0)].base.data_ptr())
    s = _lib.stream_handle()

    def step():
        _lib.check(eng.lib.mdg_denoise_step(ctypes.byref(st.model_struct), ctypes.byref(io), gs.mask.data_ptr(),
                                            st.ws.data_ptr(), s), "mdg_denoise_step")

    sec = time_kernel(step, 50)
    sm = step_model(Bl, T, L, dtype=dtype, lat=eng.lat)
    tf = sm["flops"] / sec / 1e12
    return {"kernel": "denoise_step (every launch of one step of one lane)", "bound": "mfma", "achieved": round(tf, 2),
            "peak": PEAK_TFLOPS[dtype], "unit": "TFLOP/s", "frac": round(tf / PEAK_TFLOPS[dtype], 4), "traffic": None,
            "avg_launch_us": round(sec * 1e6, 2), "flops_per_launch": sm["flops"], "shape": f"B={Bl} T={T} L={L}",
            "timing": "standalone: 50 back-to-back steps of one lane from the window's state (HIP events)"}


def cpu_train_baseline(T, L, seconds):
    """The eager CPU training step (the reference's arithmetic: the build's torch backend on the
    CPU, fp32, autograd + Adam) at B=1, T frames, timed until `seconds` of CPU work."""
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.train import Trainer

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames",
                             str(T), "--crop", str(L), "--batch_size", "1", "--synthetic_size", "1"])
    tr = Trainer(args)
    b = next(iter(tr.loader))
    tr.step([b], log=False)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        tr.step([b], log=False)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 20:
            break
    return {"value": round(T * n / el, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} eager training steps (torch CPU autograd + Adam, the reference's fp32 arithmetic), "
                      f"B=1 T={T} L={L}, {el:.1f} s on {threads} threads"}


def train_main(a, world, rank, dev, share, dp=False):
    """Config 3 (BASELINE.json configs[2]): training frames/s = world * B * T * steps / time of
    `steps` optimizer steps (GraphedStep replays; the batch is on the device).  dp: the N-GPU
    line's train_dp leg (B = --train-batch, in-graph DP markers; returns its object on rank 0)."""
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.train import Trainer

    B, T, L = (a.train_batch if dp else a.batch), a.frames, a.crop
    args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames",
                             str(T), "--crop", str(L), "--batch_size", str(B), "--synthetic_size", str(B * world),
                             "--hip_dtype", a.dtype, "--seed", "137"] + a.model_args.split())
    torch.set_float32_matmul_precision("medium")  # train.py:13
    rehearse = a.train_rccl1 and world == 1
    if rehearse:  # a world-1 RCCL group with the reduction forced on: the in-graph bucket all-reduces run
        torch.distributed.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                                             world_size=1, device_id=dev)
    if world > 1 and a.no_cond_gather:
        args.cond_allgather = 0
    tr = Trainer(args, rank, world, dev)
    tr.force_allreduce = rehearse
    tr.dp_markers = True  # in-graph events around backward's end and the last bucket all-reduce
    if rehearse and not a.no_cond_gather:  # the replicated conditioning's all-gathers at world 1 too
        tr.setup_cond_gather()
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in next(iter(tr.loader)).items()}
    for _ in range(max(1, a.warmup)):
        loss, _ = tr.step([batch], log=False)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all(), "non-finite loss"
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = tr.step([batch], log=False)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = max_over_ranks(time.perf_counter() - t0, world, torch.device("cpu") if share else dev)
    # the DP markers of a few more replays (untimed): forward + backward, and the all-reduce time
    # left after backward's end (the bucket all-reduces backward did not hide)
    dpt = []
    if tr._graphed is not None and tr._graphed.markers is not None:
        for _ in range(5):
            tr.step([batch], log=False)
            dpt.append(tr._graphed.dp_times_ms())
    n_diff = tr.check_replicas(resync=False) if world > 1 else 0
    seen = ranks_seen(world, dev, share)
    if rank != 0:
        _release(tr)
        return None
    sec = el / a.steps
    sm = step_model(B, T, L, dtype=a.dtype)
    flops = 3.0 * sm["flops"]  # forward + backward (2x) of the block stack per optimizer step
    tf = flops / sec / 1e12
    cpu = None if (a.no_cpu_baseline or world > 1 or dp) else cpu_train_baseline(T, L, a.cpu_seconds)
    out = {"metric": "training frames/sec (GVP flow-matching optimizer step), 1000-frame x crop4 forward-sim, "
                     "1/2/4/8 MI355X",
           "value": round(world * B * T * a.steps / el, 1), "unit": "frames/s", "n_gpus": 1 if share else world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(sec * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
           "data": "synthetic (seeded weights and tetrapeptide trajectories; no dataset offline)",
           "config": {"workload": f"training step: prep_batch + GVP loss + backward + grad clip + Adam + EMA, "
                                  f"B={B} trajectories x T={T} frames x L={L} per GPU",
                      "model": ("LatentMDGenModel default (5 layers, C=384, 16 heads, IPA prepend, abs pos emb)"
                                if not a.model_args else f"LatentMDGenModel {a.model_args} (IPA prepend, abs pos emb)"),
                      "global_batch": B * world, "seq_len": T, "crop": L,
                      "parallelism": f"dp{world}" + (
                          (" (per-bucket RCCL all-reduces captured in the step's graph, overlapped with backward)"
                           if tr._graphed is not None and tr._graphed.overlap else
                           " (flat all-reduce between two graphs)") if (world > 1 or rehearse) else ""),
                      "allreduce_rehearsal_world1": bool(rehearse),
                      "hipgraph": bool(tr.graph_mode)},
           "step_roofline": {"flops_per_step": flops, "flops_basis": "3 x forward FLOPs of the block stack + "
                                                                     "embedding / FinalLayer (step_model), B per GPU",
                             "achieved_tflops": round(tf, 1), "peak_tflops": PEAK_TFLOPS[a.dtype],
                             "mfma_frac": round(tf / PEAK_TFLOPS[a.dtype], 4)},
           "loss": float(loss), "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2),
           "cpu_baseline": cpu, "ranks_seen": seen}
    if dpt:
        out["dp_markers"] = {"fwd_bwd_ms": round(sum(x[0] for x in dpt) / len(dpt), 3),
                             "exposed_allreduce_ms": round(sum(x[1] for x in dpt) / len(dpt), 3),
                             "replays": len(dpt),
                             "what": "in-graph timing events: step start -> backward's end (main stream), and "
                                     "backward's end -> the last bucket all-reduce done (side stream; 0 = hidden)"}
    if world > 1:
        out["replicas_identical"] = n_diff == 0
        out["replicated_conditioning"] = bool(tr.replicated)
        out["allreduce"] = ("per-bucket RCCL all-reduces in the step's graph (side stream), conditioning "
                            "all-gathers on a second communicator" if (tr._graphed is not None and tr._graphed.overlap)
                            else "flat all-reduce between two graphs")
    if a.model_args:  # (step_model prices the default model only)
        out["step_roofline"] = None
    if share:
        out["shared_gpu"] = True
        out["ranks_sharing_gpu"] = world
    if (rehearse or world > 1) and tr._graphed is not None and tr._graphed.reducer is not None:
        red = tr._graphed.reducer
        out["replicated_conditioning_params"] = sum(p.numel() for p in tr.wrapper.model.parameters()
                                                    if id(p) in tr.replicated)
        out["allreduce_buckets"] = {"n": len(red.buckets), "bytes": [int(sl.numel() * 4) for sl in red.slices],
                                    "launched_after_grads": [n for _, n in red.launch_log],
                                    "grads_total": sum(len(b) for b in red.buckets)}
    _release(tr)
    if dp:
        return out
    emit(out)
    if rehearse:
        torch.distributed.destroy_process_group()


def _release(tr):
    """The graph holding captured collectives goes before the communicator."""
    import gc

    tr._graphed = None
    gc.collect()
    torch.cuda.synchronize()


def dopri5_main(a, world, rank, dev, share):
    """The reference's default sampler: frames/s = world * B * T * windows / time, where a
    window is Sampler(transport).sample_ode() (dopri5) from x0 ~ N(0, I) to t = 1 through the
    drop-in call (wrapper.py:472-478), every adaptive step one hipGraph replay
    (integrators.odeint_dopri5_graphed) and one host read."""
    import functools

    from mdgen_finetune_amd.transport import Dopri5Stats, Sampler, create_transport

    B, T, L = a.batch, a.frames, a.crop
    m = make_model(T, L).to(dev)
    m.hip_dtype = a.dtype
    zs, kw, _ = inputs(B, T, L, seed=100 + rank, device=dev)
    sampler = Sampler(create_transport(m.args, "GVP", "velocity"))
    fn = sampler.sample_ode()  # dopri5 (parsing.py:102)
    model = functools.partial(m.forward_inference, **kw)
    from mdgen_finetune_amd.engine import get_engine

    fn.lanes = get_engine(m)._nlanes(B)
    with torch.no_grad():
        for _ in range(max(1, a.warmup)):
            ys = fn(zs, model)
        torch.cuda.synchronize()
        assert torch.isfinite(ys[-1]).all(), "non-finite samples"
        if world > 1:
            torch.distributed.barrier()
        stats = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sampler.dopri5_stats = Dopri5Stats()
            fn(zs, model)
            stats.append(sampler.dopri5_stats)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = max_over_ranks(time.perf_counter() - t0, world, torch.device("cpu") if share else dev)
    if rank != 0:
        return
    nfe = sum(s.nfe for s in stats) / len(stats)
    sec = el / a.steps
    out = {"metric": "denoised frames/sec, 1000-frame x crop4 forward-sim window, dopri5 (the reference's default "
                     "sampler), 1/2/4/8 MI355X",
           "value": round(world * B * T * a.steps / el, 1), "unit": "frames/s", "n_gpus": 1 if share else world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(sec * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
           "data": "synthetic (seed-derived weights and tetrapeptide latents/frames; no checkpoint offline)",
           "config": {"workload": f"sim_inference rollout window: adaptive dopri5 (atol 1e-6, rtol 1e-3, 50 saved "
                                  f"points) x B={B} trajectories x T={T} frames x L={L}, per GPU",
                      "global_batch": B * world, "seq_len": T, "crop": L, "parallelism": f"replicas{world}"},
           "nfe_per_window": nfe, "accepted_steps": [s.accepted for s in stats],
           "rejected_steps": [s.rejected for s in stats],
           "ms_per_evaluation": round(sec / nfe * 1e3, 3),
           "forward_frames_per_s": round(world * B * T * nfe * a.steps / el, 1),  # comparable to the Euler line
           "lanes": getattr(fn, "lanes", None)}
    # the whole window against the MFMA roof: nfe forwards of B trajectories (the conditioning and
    # the solver's vector arithmetic included in the time, excluded from the FLOPs)
    sm = step_model(B, T, L, dtype=a.dtype)
    tf = sm["flops"] * nfe / sec / 1e12
    out["step_roofline"] = {"unit_of_work": "one dopri5 evaluation = one forward of B trajectories",
                            "flops_per_evaluation": sm["flops"], "achieved_tflops": round(tf, 1),
                            "peak_tflops": PEAK_TFLOPS[a.dtype], "mfma_frac": round(tf / PEAK_TFLOPS[a.dtype], 4)}
    if not a.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(T, L, a.cpu_seconds)
        # the oracle's forward rate on the host, priced at this window's measured evaluation count
        per_eval = T / cpu["value"]  # seconds per B=1 forward (+ Euler update) on the host
        cpu = dict(cpu, value=round(T / (per_eval * nfe), 2),
                   sample=cpu["sample"] + f"; dopri5 window = {nfe:.0f} such forwards (this run's NFE)")
        out["cpu_baseline"] = cpu
    emit(out)


def emit(obj):
    """The leg's result: printed (in-process run) or written for the orchestrator (MDG_BENCH_OUT)."""
    path = os.environ.get("MDG_BENCH_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(obj, f)
    else:
        print(json.dumps(obj), flush=True)


def ranks_seen(world, dev, share):
    """Distinct devices the ranks ran on: every rank's PCI (domain, bus, device) all-gathered."""
    if world <= 1:
        return 1
    pr = torch.cuda.get_device_properties(dev)
    code = torch.tensor([pr.pci_domain_id * 2 ** 16 + pr.pci_bus_id * 2 ** 8 + pr.pci_device_id], dtype=torch.int64,
                        device=torch.device("cpu") if share else dev)
    allc = [torch.empty_like(code) for _ in range(world)]
    torch.distributed.all_gather(allc, code)
    return len({int(c.item()) for c in allc})


def _primary_leg(a):
    return "train" if a.train else ("dopri5" if a.sampler == "dopri5" else "infer")


def dry_leg(a, leg, world, rank):
    """MDG_BENCH_DRYRUN=1 (the CPU tests of the launch path): the leg's rendezvous, barrier and
    max-over-ranks over gloo with a fixed CPU sleep as the "step"; no GPU, no model."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
        if os.environ.get("MDG_BENCH_DRYRUN_FAIL") == leg and rank == world - 1:
            sys.exit(3)  # (the tests' failing-rank case: the other ranks block in the barrier)
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        time.sleep(0.01 * (1 + rank))
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, world, torch.device("cpu"))
    seen = world
    if world > 1:
        allp = [None] * world
        dist.all_gather_object(allp, os.getpid())
        seen = len(set(allp))
        dist.destroy_process_group()
    if rank == 0:
        B = a.train_batch if leg == "train_dp" else a.batch
        emit({"metric": "dry run", "leg": leg, "value": round(world * B * a.frames * a.steps / el, 1),
              "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
              "ranks_seen": seen, "dryrun": True})


def run_leg(a, leg):
    """One rank of one leg: rank / world from the environment, cuda:LOCAL_RANK (cuda:0 for every
    rank with MDG_BENCH_SHARE_GPU=1: the N-rank rehearsal on a one-GPU box, gloo for the barrier /
    max-over-ranks, RCCL refusing two ranks per GPU), RCCL group for world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MDG_BENCH_DRYRUN") == "1":
        return dry_leg(a, leg, world, rank)
    share = os.environ.get("MDG_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    try:
        if leg == "train_dp":
            out = train_main(a, world, rank, dev, share, dp=True)
            if rank == 0:
                emit(out)
        elif leg == "train":
            train_main(a, world, rank, dev, share)
        elif leg == "dopri5":
            dopri5_main(a, world, rank, dev, share)
        else:
            infer_main(a, world, rank, dev, share)
    finally:
        if world > 1 and torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


def _wait_all(procs, timeout):
    """Wait for every worker; past `timeout` s kill the stragglers' process groups.  Returns one
    exit status per worker ('timeout' for a killed one)."""
    t_end = time.monotonic() + timeout
    rcs = [None] * len(procs)
    while any(r is None for r in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None and p.poll() is not None:
                rcs[i] = p.returncode
        if any(r not in (None, 0) for r in rcs):  # one rank failed: the others would wait forever
            t_end = min(t_end, time.monotonic() + min(30.0, timeout))
        if time.monotonic() > t_end:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
                    rcs[i] = "timeout"
            break
        time.sleep(0.2)
    return rcs


def orchestrate(a, argv):
    """--gpus N > 1: launch the legs' worker processes (never touching the GPU here) and print one
    line.  Without a launcher this process starts all N ranks; under torch.distributed.run
    (WORLD_SIZE = N) each launched process starts its own rank's worker, the launched processes
    agreeing on a fresh rendezvous port per leg over a gloo group of their own."""
    import datetime

    import torch.distributed as dist

    N = a.gpus
    share = os.environ.get("MDG_BENCH_SHARE_GPU") == "1"
    dry = os.environ.get("MDG_BENCH_DRYRUN") == "1"
    launched = "WORLD_SIZE" in os.environ
    store = None
    if launched:  # the launcher's key-value store (no process group: nothing here touches a device)
        base, orank, _ = next(dist.rendezvous("env://"))
        store = dist.PrefixStore("mdg_bench", base)
        store.set_timeout(datetime.timedelta(seconds=a.leg_timeout + a.train_dp_timeout + 600))
        ranks = [(orank, int(os.environ.get("LOCAL_RANK", "0")))]
    else:
        orank = 0
        ranks = [(r, r) for r in range(N)]

    def bcast(key, val):
        if store is None:
            return val
        if orank == 0:
            store.set(key, json.dumps(val))
        return json.loads(store.get(key))

    def gather(key, val):
        if store is None:
            return [val]
        store.set(f"{key}/{orank}", json.dumps(val))
        return [json.loads(store.get(f"{key}/{r}")) for r in range(N)]
    if not (share or dry):
        ndev = torch.cuda.device_count()  # (counts devices without initialising HIP)
        need = 1 + max(lr for _, lr in ranks)
        if ndev < need:
            print(f"bench.py: --gpus {N} needs {need} visible GPUs on this node, found {ndev}", file=sys.stderr)
            return 2
    primary = _primary_leg(a)
    legs = [primary] + (["train_dp"] if (primary == "infer" and not a.tps and not a.no_train_dp) else [])
    results = {}
    for leg in legs:
        port = [bcast(f"port/{leg}", _free_port() if orank == 0 else None)]
        fd, outp = tempfile.mkstemp(prefix=f"mdg_bench_{leg}_", suffix=".json")
        os.close(fd)
        env0 = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
        env0.update(MDG_BENCH_LEG=leg, WORLD_SIZE=str(N), LOCAL_WORLD_SIZE=str(N if not launched else
                                                                             os.environ.get("LOCAL_WORLD_SIZE", N)),
                    MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port[0]), MDG_BENCH_OUT=outp)
        procs = []
        for r, lr in ranks:
            env = dict(env0, RANK=str(r), LOCAL_RANK=str(lr))
            if r != 0:
                env.pop("MDG_BENCH_OUT")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                          stdout=sys.stderr, start_new_session=True))
        rcs = _wait_all(procs, a.leg_timeout if leg == primary else a.train_dp_timeout)
        if launched:  # every launched process learns every rank's status
            rcs = [x for r_ in gather(f"rc/{leg}", rcs) for x in r_]
        res = None
        if orank == 0:
            try:
                with open(outp) as f:
                    res = json.load(f)
            except (OSError, ValueError):
                res = None
        os.unlink(outp)
        results[leg] = (rcs, res)
        if leg == primary and any(rc != 0 for rc in rcs):
            break
    rc = 0
    if orank == 0:
        rcs, line = results[primary]
        if any(r_ != 0 for r_ in rcs) or line is None:
            print(f"bench.py: the {primary} leg failed: worker exit statuses {rcs}", file=sys.stderr)
            rc = 1
        else:
            if "train_dp" in results:
                trcs, tline = results["train_dp"]
                if any(r_ != 0 for r_ in trcs) or tline is None:
                    tline = {"status": "failed", "worker_exit": trcs,
                             "note": "the N-GPU training leg did not complete (its workers' stderr is in the log)"}
                line["train_dp"] = tline
            line["launch"] = ("torch.distributed.run (one worker per launched rank)" if launched else
                              f"self-launched: {N} worker processes" + (" sharing cuda:0 (rehearsal)" if share
                                                                        else ", one per GPU"))
            print(json.dumps(line), flush=True)
    gather("done", rc)
    return rc


def main():
    a = parse()
    leg = os.environ.get("MDG_BENCH_LEG")
    if leg:  # a worker of orchestrate()
        return run_leg(a, leg)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != a.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {a.gpus}: refusing to report a different GPU count",
              file=sys.stderr)
        sys.exit(2)
    if a.gpus == 1:  # the headline: in this process
        return run_leg(a, _primary_leg(a))
    sys.exit(orchestrate(a, sys.argv[1:]))


def infer_main(a, world, rank, dev, share):
    from mdgen_finetune_amd.engine import get_engine

    B, T, L = a.batch, a.frames, a.crop
    m = make_model(T, L, tps=a.tps).to(dev)
    m.hip_dtype = a.dtype
    eng = get_engine(m)
    eng.lanes = a.lanes
    zs, kw, _ = inputs(B, T, L, seed=100 + rank, device=dev, tps=a.tps)

    def window():
        return eng.sample_euler(zs, num_steps=a.num_steps, use_graph=not a.no_graph, **kw)

    with torch.no_grad():
        for _ in range(max(1, a.warmup)):
            ys = window()
        torch.cuda.synchronize()
        assert torch.isfinite(ys[-1]).all(), "non-finite samples"

        def barrier():
            if world > 1:
                torch.distributed.barrier()

        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ys = window()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        el = max_over_ranks(el, world, torch.device("cpu") if share else dev)
        n_euler = a.num_steps - 1
        value = job_value(world, B, T, n_euler, a.steps, el)
        # roofline launches at the shape the timed region runs them with (one lane's batch)
        nl = a.lanes if (a.lanes > 1 and B % a.lanes == 0) else 1
        Bl = B // nl
        st = eng._state(Bl, T, L, lane=1 if nl > 1 else 0)
        roofs = roofline(eng, st, a.dtype, Bl, T, L) if rank == 0 and not a.tps else None
        if rank == 0 and a.tps:
            roofs = {"step": step_kernel_roofline(eng, B, T, L, a.dtype, nl, zs, kw)}
        plan = eng.describe_plan(Bl, T, L)
        seen = ranks_seen(world, dev, share)

    # extra lines (rank 0, single process): the B sweep SURVEY §8(d) asks for and the fp32
    # parity-path throughput, each with its own step-level roofline
    sweep = []
    if rank == 0 and world == 1 and not a.tps:
        for Bs in [int(b) for b in a.sweep_batches.split(",") if b.strip()]:
            if Bs != B:
                sweep.append(sweep_line(dev, T, L, Bs, a.dtype, a.lanes, a.num_steps, a.sweep_steps, 300 + Bs))
        if not a.no_f32_line and a.dtype != "f32":
            sweep.append(sweep_line(dev, T, L, B, "f32", a.lanes, a.num_steps, a.sweep_steps, 100))

    out = None
    if rank == 0:
        cpu = None if (a.no_cpu_baseline or world > 1) else cpu_baseline(T, L, a.cpu_seconds, tps=a.tps)
        out = {
            "metric": "denoised frames/sec, 1000-frame x crop4 forward-sim step, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": 1 if share else world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (seed-derived weights and tetrapeptide latents/frames; no checkpoint offline)",
            "config": {"workload": f"sim_inference rollout window: Euler ODE {n_euler} denoising steps x "
                                   f"B={B} trajectories x T={T} frames x L={L} residues (+ per-window "
                                   "conditioning), per GPU",
                       "model": "LatentMDGenModel default (5 layers, C=384, 16 heads, IPA prepend, abs pos emb)",
                       "global_batch": B * world, "seq_len": T, "crop": L, "denoise_steps_per_step": n_euler,
                       "parallelism": f"replicas{world}", "hipgraph": not a.no_graph,
                       "lanes": a.lanes},
            "us_per_denoise_step": round(el / a.steps / n_euler * 1e6, 2),
            "step_roofline": step_roofline(B, T, L, a.dtype, el / a.steps / n_euler / world, *_fusions(plan)),
            "kernel_plan": plan,
            "batch_sweep": sweep,
            "roofline": list(roofs.values())[0] if roofs else None,
            "roofline_more": list(roofs.values())[1:] if roofs else None,
            "cpu_baseline": cpu,
            "ranks_seen": seen,
        }
        if a.tps:  # BASELINE config 4 evidence line (tps_inference.py path), not the headline metric
            out["config"]["workload"] = (f"tps_inference window: Euler ODE {n_euler} denoising steps x B={B} "
                                         f"interpolations x T={T} frames x L={L} residues, start + end frames "
                                         "conditioned (+ per-window dual-IPA conditioning), per GPU")
            out["config"]["model"] = "LatentMDGenModel --tps_condition (latent 28, 5 layers, C=384, 16 heads, IPA prepend)"
        if share:  # rehearsal: every rank on cuda:0 — not a multi-GPU measurement
            out["shared_gpu"] = True
            out["ranks_sharing_gpu"] = world
        emit(out)


if __name__ == "__main__":
    main()
