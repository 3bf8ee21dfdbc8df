"""Import-only stand-in for `torch_complex` (golden capture only)."""
from . import functional, tensor  # noqa: F401
