"""MI355X (gfx950) HIP engine for the MRA-GAN CycleGAN training step."""
from ._lib import LIB_PATH, MraganError, exported_symbols, lib  # noqa: F401
