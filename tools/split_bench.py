"""The reference's own sim_inference call shape over a split of tetrapeptides, timed two ways on
one GPU (VERDICT r05 "next" 5): serial (one peptide per window, --batch 1: the reference's loop,
/root/reference/src/sim_inference.py:100-136) against --peptides_per_window K (K peptides' rows
side by side in one window).  Default model (5 layers, C=384, 16 heads, IPA prepend), synthetic
weights and start frames, T=1000, Euler 50, bf16; each window = sample + atom14 reconstruction +
restart geometry (sim_inference.rollout_group).  Prints one JSON object.
usage: python tools/split_bench.py [--peptides 16] [--rollouts 2] [--k 1,4,8,16]"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peptides", type=int, default=16)
    ap.add_argument("--rollouts", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--k", default="1,4,8,16")
    a = ap.parse_args()
    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.data import SyntheticMDDataset
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.sim_inference import RESTYPES, peptide_generator, rollout_group, seq_to_aatype
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames",
                             str(a.frames), "--crop", "4", "--sampling_method", "euler"])
    w = NewMDGenWrapper(args)
    synthetic.fill_module_(w.model, 0)
    w = w.eval().cuda()
    w.model.hip_dtype = "bf16"
    g = torch.Generator().manual_seed(3)
    jobs = []
    for k in range(a.peptides):
        seq = "".join(RESTYPES[int(i)] for i in torch.randint(0, 20, (4,), generator=g))
        it = SyntheticMDDataset(1, 4, size=1, seed=k)[0]
        b = {"torsions": it["torsions"][None], "torsion_mask": it["torsion_mask"][None], "trans": it["trans"][None],
             "rots": it["rots"][None], "seqres": seq_to_aatype(seq)[None], "mask": torch.ones(1, 4)}
        jobs.append((f"{seq}_{k}", {key: v.cuda() for key, v in b.items()}))
    out = {"metric": "sim_inference rollout frames/s over a split (rollout = sample + atom14 + restart)",
           "peptides": a.peptides, "windows_per_peptide": a.rollouts, "frames": a.frames, "crop": 4,
           "trajectories_per_peptide": 1, "model": "LatentMDGenModel default, bf16, Euler 50", "runs": []}
    dev = torch.device("cuda")
    for K in [int(x) for x in a.k.split(",")]:
        def go():
            gens = [(n, b, peptide_generator(0, i, dev)) for i, (n, b) in enumerate(jobs)]
            with torch.no_grad():
                for g0 in range(0, len(gens), K):
                    rollout_group(w, gens[g0:g0 + K], a.frames, a.rollouts, 1, 21)
            torch.cuda.synchronize()

        # warm: one group of this K (graph capture for its row count)
        gens = [(n, b, peptide_generator(0, i, dev)) for i, (n, b) in enumerate(jobs[:K])]
        with torch.no_grad():
            rollout_group(w, gens, a.frames, 1, 1, 21)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        go()
        el = time.perf_counter() - t0
        frames = a.peptides * a.rollouts * a.frames
        out["runs"].append({"peptides_per_window": K, "rows_per_window": K, "seconds": round(el, 3),
                            "frames_per_s": round(frames / el, 1),
                            "denoised_frames_per_s": round(frames * 49 / el, 1)})
        print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    base = out["runs"][0]["frames_per_s"]
    for r in out["runs"]:
        r["speedup_vs_serial"] = round(r["frames_per_s"] / base, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
