"""The CPU oracle (oracle/mdgen_oracle.py) against golden vectors produced by the reference
itself (oracle/gen_golden.py): pins the restatement before it is used to judge the HIP path."""
import numpy as np
import pytest
import torch

from oracle import mdgen_oracle as O
from tests.conftest import load_golden

FORWARD_CASES = ["small_sim_T1", "small_sim_T8", "small_sim_pad", "small_tps_T8", "full_sim_T1",
                 "full_sim_T64", "full_tps_T100"]


def _setup(name):
    d, cfg = load_golden(name)
    c = O.Cfg.from_flags(cfg["flags"], cfg["latent_dim"], cfg["L"], cfg["tps"])
    return d, cfg, c, O.seeded_params(c, cfg["weights_seed"]), O.kwargs_from_npz(d)


@pytest.mark.parametrize("name", FORWARD_CASES)
def test_oracle_forward_matches_reference(name):
    d, cfg, c, P, kw = _setup(name)
    cap = {}
    with torch.no_grad():
        v = O.forward(P, c, torch.from_numpy(d["in_x"]), torch.from_numpy(d["in_t"]), capture=cap, **kw)
    np.testing.assert_allclose(v.numpy(), d["out_v"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(cap["ipa"].numpy(), d["out_ipa"], rtol=0, atol=2e-5)
    for i in range(c.num_layers):
        if f"out_layer{i}" in d.files:
            np.testing.assert_allclose(cap[f"layer{i}"].numpy(), d[f"out_layer{i}"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("name", ["small_sim_T8", "full_sim_T64"])
def test_oracle_euler_matches_reference(name):
    d, cfg, c, P, kw = _setup(name)
    with torch.no_grad():
        ys = O.euler_sample(P, c, torch.from_numpy(d["in_zs"]), **kw)
    assert ys.shape[0] == int(d["out_euler_n"])
    np.testing.assert_allclose(ys[1].numpy(), d["out_euler_step1"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(ys[-1].numpy(), d["out_euler_final"], rtol=0, atol=5e-5)


def test_oracle_gvp_loss_matches_reference():
    d, cfg, c, P, kw = _setup("small_loss")
    with torch.no_grad():
        loss, v = O.gvp_training_loss(P, c, torch.from_numpy(d["in_x"]), torch.from_numpy(d["in_x0"]),
                                      torch.from_numpy(d["in_t_loss"]), torch.from_numpy(d["in_loss_mask"]), **kw)
    np.testing.assert_allclose(loss.numpy(), d["out_loss"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(v.numpy(), d["out_pred"], rtol=0, atol=2e-5)


def test_oracle_mha_unit_rope_biaskv_and_full_padding():
    """RoPE position of the appended bias_k row (S), key padding, and a sequence whose every
    real key is padded (only the bias row survives)."""
    d, cfg = load_golden("mha_rope_biaskv")
    from mdgen_finetune_amd.synthetic import param_value

    C = cfg["C"]
    P = {}
    for n in ("k_proj", "v_proj", "q_proj", "out_proj"):
        P[f"m.attn.{n}.weight"] = torch.from_numpy(param_value(cfg["seed"], f"{n}.weight", (C, C)))
        P[f"m.attn.{n}.bias"] = torch.from_numpy(param_value(cfg["seed"], f"{n}.bias", (C,)))
    for n in ("bias_k", "bias_v"):
        P[f"m.attn.{n}"] = torch.from_numpy(param_value(cfg["seed"], n, (1, 1, C)))
    x = torch.from_numpy(d["in_x"]).transpose(0, 1)          # [N, S, C]
    valid = 1 - torch.from_numpy(d["in_key_padding_mask"])
    with torch.no_grad():
        o = O.mha(P, "m", x, valid, cfg["H"]).transpose(0, 1)
    np.testing.assert_allclose(o.numpy(), d["out_o"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("name,tps", [("state_dict_sim", False), ("state_dict_tps", True)])
def test_param_shapes_match_reference_state_dict(name, tps):
    d, cfg = load_golden(name)
    ref = {k: tuple(__import__("json").loads(s)) for k, s in zip(d["out_keys"], d["out_shapes"])}
    c = O.Cfg(latent_dim=cfg["latent_dim"], tps=tps)
    mine = dict(O.param_shapes(c))
    buffers = {k for k in ref if k.endswith("inv_freq") or k == "pos_embed"}
    assert set(mine) == set(ref) - buffers
    for k, s in mine.items():
        assert ref[k] == tuple(s), k
