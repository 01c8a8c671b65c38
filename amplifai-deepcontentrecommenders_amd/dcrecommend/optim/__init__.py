"""Optimizers and LR schedule of the DCUE trainer."""
from .adam import NativeAdam  # noqa: F401
from .native import NativeRanger, NativeSGD  # noqa: F401
