from . import horus, las, simple  # noqa: F401  (register policies)
from .base import Policy, make_policy, policies

__all__ = ["Policy", "make_policy", "policies"]
