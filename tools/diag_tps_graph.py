"""Diagnostic (GPU box): test_tps_graphed_step_equals_eager_step with the graphed step's optimizer
on the library kernels (MDG_TRAIN_FUSED_OPT=1) and on torch's (=0): per parameter, the largest
difference to the eager trainer after two steps and the Adam moments at that element.
Usage: python tools/diag_tps_graph.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from mdgen_finetune_amd.train import Trainer
    from tests.test_gpu_train import _fixed_noise
    from tests.test_train import _args, _batch

    a = _args(["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4", "--tps_condition", "--train_graph", "1"])
    a.sim_condition = False
    b, b2 = _batch(a, B=2), _batch(a, B=2, seed=9)
    for fused in ("1", "0"):
        os.environ["MDG_TRAIN_FUSED_OPT"] = fused
        tr = Trainer(a, device=torch.device("cuda"))
        _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 28))
        tr.step([b], log=False)
        tr.step([b2], log=False)
        tr2 = Trainer(a, device=torch.device("cuda"))
        tr2.graph_mode = False
        _fixed_noise(tr2, 2, (2, a.num_frames, a.crop, 28))
        tr2.step([b], log=False)
        tr2.step([b2], log=False)
        rows = []
        for (name, p1), p2 in zip(tr.wrapper.model.named_parameters(), tr2.wrapper.model.parameters()):
            d = (p1.detach() - p2.detach()).abs().flatten()
            i = int(d.argmax())
            s1, s2 = tr.optimizer.state.get(p1, {}), tr2.optimizer.state.get(p2, {})
            mom = lambda s, k: (float(s[k].flatten()[min(i, s[k].numel() - 1)]) if k in s  # noqa: E731
                                else float("nan"))
            rows.append((float(d[i]), name, mom(s1, "exp_avg"), mom(s2, "exp_avg"), mom(s1, "exp_avg_sq"),
                         mom(s2, "exp_avg_sq"), mom(s1, "step"), mom(s2, "step")))
        rows.sort(reverse=True)
        print(f"MDG_TRAIN_FUSED_OPT={fused}: worst parameters (max |diff|, name, m graph/eager, v graph/eager, "
              f"step graph/eager)")
        for r in rows[:8]:
            print("  %.3e %-45s m %.3e %.3e v %.3e %.3e step %s %s" % r)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
