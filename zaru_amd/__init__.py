"""zaru_amd -- MI355X (gfx950) backend for Zaru's detection/landmark hot path.

``zaru_amd.nn`` mirrors ``zaru::nn`` (NeuralNetwork, Loader, Cnn, ColorMapper) over the C ABI
of ``include/zaru_hip.h``; every network and the image->tensor preprocessing run as
hand-written HIP kernels.  There is no CPU fallback: without the built extension or a GPU the
calls raise ``zaru_amd._lib.ZaruError``.
"""
from ._lib import ZaruError, device_count, lib  # noqa: F401

__all__ = ["ZaruError", "device_count", "lib"]
