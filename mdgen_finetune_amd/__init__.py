"""mdgen_finetune_amd — MI355X-native (gfx950) MDGen flow-matching denoising hot path.

Drop-in for the reference's LatentMDGenModel.forward / Sampler.sample_ode / sim_inference /
train entry points, with every token-wise op of the denoising step in libmdgen_hip.so.
"""
__version__ = "0.1.0"
