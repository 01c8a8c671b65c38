"""Optimizers and LR schedule of the DCUE trainer."""
from .adam import NativeAdam  # noqa: F401
