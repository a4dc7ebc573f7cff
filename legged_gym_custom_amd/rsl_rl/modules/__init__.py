from .actor_critic import ActorCritic  # noqa: F401
from .support_networks import AdaptationEncoder, MlpEstimator, PrivilegedEncoder, ScanEncoder  # noqa: F401
