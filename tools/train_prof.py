"""torch.profiler summary of the training step (where the GVP step's time goes)."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd.parsing import parse_train_args  # noqa: E402
from mdgen_finetune_amd.train import Trainer  # noqa: E402

B = int(os.environ.get("B", "8"))
args = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames", "1000",
                         "--crop", "4", "--batch_size", str(B), "--synthetic_size", str(B)]
                        + sys.argv[1:])
tr = Trainer(args, device=torch.device("cuda"))
batch = next(iter(tr.loader))
for _ in range(2):
    tr.step([batch])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(2):
        tr.step([batch])
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=60, max_name_column_width=70))
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25, max_name_column_width=60))
