from .integrators import Dopri5Stats, odeint_dopri5  # noqa: F401
from .transport import Sampler, Transport, create_transport, mean_flat  # noqa: F401
