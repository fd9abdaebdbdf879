from .latent_model import LatentMDGenModel  # noqa: F401
