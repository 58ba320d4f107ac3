from .fromage import Fromage  # noqa: F401
from .madam import Madam  # noqa: F401
from .fused_adam import FusedAdam  # noqa: F401
