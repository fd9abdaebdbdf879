import argparse
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libmdgen_hip.so")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return d, json.loads(str(d["config"]))


def model_args(cfg, T=None):
    """argparse.Namespace with the reference's flag names for a golden config."""
    from oracle.mdgen_oracle import Cfg

    c = Cfg.from_flags(cfg.get("flags", []), cfg["latent_dim"], cfg.get("L", 4), cfg.get("tps", False))
    return argparse.Namespace(
        embed_dim=c.embed_dim, mha_heads=c.mha_heads, num_layers=c.num_layers, ipa_heads=c.ipa_heads,
        ipa_head_dim=c.ipa_head_dim, ipa_qk=c.ipa_qk, ipa_v=c.ipa_v, dropout=0.0, no_rope=False,
        prepend_ipa=True, abs_pos_emb=True, crop=cfg.get("L", 4), num_frames=T or cfg.get("T", 1),
        time_multiplier=100.0, sim_condition=not c.tps, tps_condition=c.tps, path_type="GVP",
        prediction="velocity", sampling_method="euler"), c


def build_model(cfg, device="cpu", T=None):
    import torch  # noqa: F401

    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.model.latent_model import LatentMDGenModel

    args, c = model_args(cfg, T)
    m = LatentMDGenModel(args, cfg["latent_dim"]).eval()
    synthetic.fill_module_(m, cfg["weights_seed"])
    return m.to(device), c


@pytest.fixture
def golden():
    return load_golden
