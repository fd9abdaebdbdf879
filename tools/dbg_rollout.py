"""Debug: stage-by-stage HIP vs CPU comparison of the TPS rollout test (dumps npz)."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from pathlib import Path
from mdgen_finetune_amd.checkpoint import load_from_checkpoint
from mdgen_finetune_amd.tps_inference import _synthetic_traj, collate_samples, get_sample
from tests.test_geometry import _small_ckpt
tmp = Path("gpurun_out/dbg"); tmp.mkdir(parents=True, exist_ok=True)
ck = _small_ckpt(tmp, T=8, tps=True)
g = torch.Generator().manual_seed(11)
zs = torch.randn(2, 8, 4, 28, generator=g)
res = {}
for dev in ("cuda", "cpu"):
    w = load_from_checkpoint(ck).eval().to(dev)
    if dev == "cpu":
        w.model.backend = "torch"
    else:
        w.model.hip_dtype = "f32"
    arr, aat = _synthetic_traj("AKDW", 32, 4)
    rng = np.random.RandomState(0)
    batch = collate_samples([get_sample(arr, aat, [0, 3], [20, 30], num_frames=8, rng=rng, device=dev) for _ in range(2)])
    with torch.no_grad():
        prep = w.prep_batch(batch)
        samples, _ = w.sample_latents(batch, zs0=zs.to(dev))
        a14, _ = w.inference(batch, zs0=zs.to(dev))
        # eager model on this device for the velocity at t=0
        kw = prep["model_kwargs"]
        w.model.backend = "torch"
        v_t = w.model(zs.to(dev), torch.zeros(2, device=dev), **kw)
        if dev == "cuda":
            w.model.backend = "hip"
        v_h = w.model(zs.to(dev), torch.zeros(2, device=dev), **kw)
    res[dev] = dict(latents=prep["latents"].cpu().numpy(), x_cond=kw["x_cond"].cpu().numpy(),
                    cond=kw["x_cond_mask"].cpu().numpy(), samples=samples.cpu().numpy(), a14=a14.cpu().numpy(),
                    v_torch=v_t.cpu().numpy(), v_model=v_h.cpu().numpy(), trans=batch["trans"].cpu().numpy())
for k in res["cpu"]:
    a, b = res["cuda"][k], res["cpu"][k]
    print(k, a.shape, float(np.abs(a.astype(np.float64) - b).max()))
np.savez("gpurun_out/dbg/rollout.npz", **{f"{d}_{k}": v for d in res for k, v in res[d].items()})
