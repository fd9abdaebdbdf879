from .transport import Sampler, Transport, create_transport, mean_flat  # noqa: F401
