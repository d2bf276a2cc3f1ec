"""mog_air — MI355X-native (gfx950 HIP) implementation of the AIR per-object-step
hot path of taufikxu/MOG-ASR (air/air_model.py, air/transformer.py, air/vae.py,
air/concrete.py).  Host side in Python over the C ABI of libmog_air.so."""
from . import _lib  # noqa: F401

__all__ = ["air_model", "ops", "params"]
