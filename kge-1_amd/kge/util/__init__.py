from .loss import KgeLoss  # noqa: F401
from .optimizer import KgeOptimizer, KgeLRScheduler  # noqa: F401
