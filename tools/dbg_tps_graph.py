"""Debug: TPS graphed step vs eager step loss (one GPU)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_gpu_train import _fixed_noise  # noqa: E402
from tests.test_train import _args, _batch  # noqa: E402
from mdgen_finetune_amd.train import Trainer  # noqa: E402
from mdgen_finetune_amd.model.latent_model import relative_tensor7  # noqa: E402
from mdgen_finetune_amd.rigid_utils import frames_to_tensors  # noqa: E402

for mode in (0, 1, 0):
    a = _args(["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4", "--tps_condition", "--train_graph", str(mode)])
    a.sim_condition = False
    tr = Trainer(a, device=torch.device("cuda"))
    b = _batch(a, B=2)
    _fixed_noise(tr, 2, (2, a.num_frames, a.crop, 28))
    if mode == 0:
        bd = {k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()}
        prep = tr.wrapper.prep_batch(bd)
        r, t = frames_to_tensors(prep["model_kwargs"]["start_frames"])
        er, et = frames_to_tensors(prep["model_kwargs"]["end_frames"])
        rel = relative_tensor7(r, t, er, et)
        print("rel eager", rel.flatten()[:8].tolist())
        with torch.enable_grad():
            l1 = tr.wrapper.general_step(bd, log=False)[0]
            l2 = tr.wrapper.general_step(bd, log=False)[0]
        print("eager general_step twice", float(l1), float(l2))
    loss, _ = tr.step([b], log=False)
    print("mode", mode, "loss", float(loss))
    if mode == 1:
        print("rel feed", tr._graphed.rel7.flatten()[:8].tolist())
        loss2, _ = tr.step([b], log=False)
        print("mode 1 second loss", float(loss2))
