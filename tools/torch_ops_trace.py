"""Which PyTorch operators launch device work in the training step: one eager step of the
bench.py --train configuration (B=8, T=1000, L=4) under torch.profiler, grouped by operator and
the top Python frames that called it.  Writes gpurun_out/torch_ops.txt.
Usage (GPU box): python tools/torch_ops_trace.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.train import Trainer

    B, T, L = 8, 1000, 4
    args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames", str(T),
                             "--crop", str(L), "--batch_size", str(B), "--synthetic_size", str(B), "--seed", "137",
                             "--train_graph", "0"])
    dev = torch.device("cuda", 0)
    tr = Trainer(args, 0, 1, dev)
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in next(iter(tr.loader)).items()}
    for _ in range(2):
        tr.step([batch], log=False)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=False) as prof:
        tr.step([batch], log=False)
        torch.cuda.synchronize()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "torch_ops.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=60))
        f.write("\n\n")
        f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_device_time_total", row_limit=60,
                                                             max_name_column_width=60, max_src_column_width=200))
    print("wrote gpurun_out/torch_ops.txt")


if __name__ == "__main__":
    main()
