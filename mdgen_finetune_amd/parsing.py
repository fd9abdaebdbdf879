"""Command-line flags of the reference's ``train.py`` (src/mdgen/parsing.py:5-131), so a
reference launch line (and the ``args`` Namespace stored in a reference checkpoint) drives
this build unchanged.  Flags whose feature is outside this build (design / MPNN / hyena /
inpainting / no_frames ...) are still accepted; the model constructor refuses the ones that
would change the network (latent_model.UNSUPPORTED_FLAGS)."""
from __future__ import annotations

import argparse
import os

_S, _I, _F, _B = str, int, float, "flag"

# (group, flag, type, default)  — defaults as in the reference
_FLAGS = [
    (None, "ckpt", _S, None), (None, "validate", _B, False), (None, "num_workers", _I, 4),
    ("epoch", "epochs", _I, 100), ("epoch", "overfit", _B, False), ("epoch", "overfit_peptide", _S, None),
    ("epoch", "overfit_frame", _B, False), ("epoch", "train_batches", _I, None), ("epoch", "val_batches", _I, None),
    ("epoch", "val_repeat", _I, 1), ("epoch", "inference_batches", _I, 0), ("epoch", "batch_size", _I, 8),
    ("epoch", "val_freq", _I, None), ("epoch", "val_epoch_freq", _I, 1), ("epoch", "no_validate", _B, False),
    ("epoch", "designability_freq", _I, 1),
    ("log", "print_freq", _I, 100), ("log", "ckpt_freq", _I, 1), ("log", "wandb", _B, False),
    ("log", "run_name", _S, "default"),
    ("optim", "accumulate_grad", _I, 1), ("optim", "grad_clip", _F, 1.0), ("optim", "check_grad", _B, False),
    ("optim", "grad_checkpointing", _B, False), ("optim", "adamW", _B, False), ("optim", "ema", _B, False),
    ("optim", "ema_decay", _F, 0.999), ("optim", "lr", _F, 1e-4), ("optim", "precision", _S, "32-true"),
    ("data", "train_split", _S, None), ("data", "val_split", _S, None), ("data", "data_dir", _S, None),
    ("data", "num_frames", _I, 50), ("data", "crop", _I, 256), ("data", "suffix", _S, ""),
    ("data", "atlas", _B, False), ("data", "copy_frames", _B, False), ("data", "no_pad", _B, False),
    ("data", "short_md", _B, False),
    ("mask", "design_key_frames", _B, False), ("mask", "no_aa_emb", _B, False), ("mask", "no_torsion", _B, False),
    ("mask", "no_design_torsion", _B, False), ("mask", "supervise_no_torsions", _B, False),
    ("mask", "supervise_all_torsions", _B, False),
    ("ablation", "no_offsets", _B, False), ("ablation", "no_frames", _B, False),
    ("model", "hyena", _B, False), ("model", "no_rope", _B, False), ("model", "dropout", _F, 0.0),
    ("model", "scale_factor", _F, 1.0), ("model", "interleave_ipa", _B, False), ("model", "prepend_ipa", _B, False),
    ("model", "oracle", _B, False), ("model", "num_layers", _I, 5), ("model", "embed_dim", _I, 384),
    ("model", "mha_heads", _I, 16), ("model", "ipa_heads", _I, 4), ("model", "ipa_head_dim", _I, 32),
    ("model", "ipa_qk", _I, 8), ("model", "ipa_v", _I, 8), ("model", "time_multiplier", _F, 100.0),
    ("model", "abs_pos_emb", _B, False), ("model", "abs_time_emb", _B, False),
    ("transport", "alpha_max", _F, 8.0), ("transport", "discrete_loss_weight", _F, 0.5),
    ("transport", "dirichlet_flow_temp", _F, 1.0), ("transport", "allow_nan_cfactor", _B, False),
    ("video", "tps_condition", _B, False), ("video", "design", _B, False), ("video", "design_from_traj", _B, False),
    ("video", "sim_condition", _B, False), ("video", "inpainting", _B, False), ("video", "dynamic_mpnn", _B, False),
    ("video", "mpnn", _B, False), ("video", "frame_interval", _I, None), ("video", "cond_interval", _I, None),
]
# flags with choices (the reference spells path-type with a dash; argparse stores path_type)
_CHOICES = [
    ("--path-type", "GVP", ["Linear", "GVP", "VP"]),
    ("--prediction", "velocity", ["velocity", "score", "noise"]),
    ("--sampling_method", "dopri5", ["dopri5", "euler"]),
]
# This build's own additions (not in the reference): data source and the distributed knobs.
_EXTRA = [
    ("synthetic", _B, False, "train on synthetic trajectories (no dataset offline)"),
    ("synthetic_size", _I, 64, "number of synthetic trajectories"),
    ("max_steps", _I, None, "stop after this many optimizer steps"),
    ("seed", _I, 137, "base RNG seed (rank r uses seed + r for its noise draws)"),
    ("bucket_cap_mb", _F, 32.0, "gradient bucket size of the all-reduce overlapped with backward (DDP and the graphed step)"),
    ("model_dir", _S, None, "checkpoint directory (default workdir/<run_name>, the reference's MODEL_DIR)"),
    ("train_backend", _S, "hip", "'hip': on a ROCm device every block's forward + backward runs in "
                                 "libmdgen_hip.so (train_hip.py); 'torch': eager autograd"),
    ("hip_dtype", _S, "bf16", "operand type of the HIP GEMM / attention kernels: 'bf16' (fp32 accumulate, "
                              "the reference's matmul precision 'medium') or 'f32' (exact fp32)"),
    ("train_graph", _I, 1, "1: on a ROCm device the optimizer step replays hipGraphs (forward + loss + "
                           "backward [+ RCCL gradient all-reduce between two graphs] + clip + Adam + EMA); "
                           "0: eager step (also used for grad accumulation > 1 and 16-mixed)"),
    ("cond_allgather", _I, 1, "data-parallel training (world > 1): 1 = the conditioning (t-MLP, adaLN, IPA "
                              "prepend) runs on the all-gathered batch of every rank and its parameters' "
                              "gradients come out rank-averaged, so they leave the gradient all-reduce "
                              "(cond_dist.py); 0 = every gradient all-reduced"),
    ("check_replicas", _I, 1, "world > 1: every print_freq steps compare a checksum of every parameter / EMA "
                              "tensor across ranks and re-broadcast rank 0's state if any differ"),
    ("allreduce_overlap", _I, 1, "graphed step with world > 1 over RCCL: 1 = per-bucket all-reduces captured "
                                 "in the graph on a side stream, each issued as backward completes its bucket "
                                 "(--bucket_cap_mb); 0 = one flat all-reduce between two graphs"),
]

_REQUIRED = ("train_split", "val_split", "data_dir")


def build_parser(require_data=True):
    p = argparse.ArgumentParser(description="MDGen trainer (MI355X build)")
    groups = {}
    for grp, name, typ, default in _FLAGS:
        g = p if grp is None else groups.setdefault(grp, p.add_argument_group(grp))
        if typ is _B:
            g.add_argument(f"--{name}", action="store_true", default=default)
        else:
            g.add_argument(f"--{name}", type=typ, default=default,
                           required=require_data and name in _REQUIRED)
    for flag, default, choices in _CHOICES:
        p.add_argument(flag, type=str, default=default, choices=choices)
    ex = p.add_argument_group("mi355x build")
    for name, typ, default, help_ in _EXTRA:
        if typ is _B:
            ex.add_argument(f"--{name}", action="store_true", default=default, help=help_)
        else:
            ex.add_argument(f"--{name}", type=typ, default=default, help=help_)
    return p


def parse_train_args(argv=None):
    """parsing.py:5-131: returns the Namespace and sets MODEL_DIR=workdir/<run_name>."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--synthetic", action="store_true")
    known, _ = pre.parse_known_args(argv)
    args = build_parser(require_data=not known.synthetic).parse_args(argv)
    args.model_dir = args.model_dir or os.path.join("workdir", args.run_name)
    os.environ["MODEL_DIR"] = args.model_dir
    return args


def default_args(**overrides):
    """A Namespace with every default (no data flags required), updated by ``overrides``."""
    args = build_parser(require_data=False).parse_args([])
    for k, v in overrides.items():
        setattr(args, k, v)
    return args
