"""Python mirror of ``zaru::nn`` (crates/zaru/src/nn/mod.rs) over the HIP C ABI.

``NeuralNetwork`` / ``Loader`` / ``Cnn`` / ``ColorMapper`` keep the reference's names and
argument meaning; inference always runs through ``libzaru_hip.so`` on the GPU.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import Frame, View, check, lib

MODELS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models")


class Loader:
    """NeuralNetwork loader (nn/mod.rs:205-362)."""

    def __init__(self, data: bytes):
        self._data = data
        self._outputs: Optional[List[int]] = None
        self._device = 0

    def with_output_selection(self, outputs: Sequence[int]) -> "Loader":
        self._outputs = list(outputs)
        return self

    def with_gpu_support(self) -> "Loader":  # always on: the HIP backend is the GPU backend
        return self

    def on_device(self, device: int) -> "Loader":
        self._device = device
        return self

    def load(self) -> "NeuralNetwork":
        return NeuralNetwork._create(self._data, self._outputs, self._device)


class NeuralNetwork:
    """A loaded network (nn/mod.rs:365-539); ``estimate`` is batched over dim 0."""

    def __init__(self):
        raise TypeError("use NeuralNetwork.from_onnx(...).load() or from_path(...).load()")

    @staticmethod
    def from_onnx(data: bytes) -> Loader:
        return Loader(bytes(data))

    @staticmethod
    def from_path(path: str) -> Loader:
        if not str(path).endswith(".onnx"):
            raise ValueError("neural network file must have `.onnx` extension")
        with open(path, "rb") as f:
            return Loader(f.read())

    @classmethod
    def _create(cls, data: bytes, outputs, device):
        self = object.__new__(cls)
        self._buf = data
        sel = (C.c_uint32 * len(outputs))(*outputs) if outputs else None
        h = C.c_void_p()
        check(lib().zr_session_create(data, len(data), sel, len(outputs or []), device,
                                      C.byref(h)))
        self._h = h
        self.device = device
        self._inputs = [self._io(0, 0)]
        n = C.c_size_t()
        check(lib().zr_session_num_io(self._h, 1, C.byref(n)))
        self._outputs = [self._io(1, i) for i in range(n.value)]
        return self

    def _io(self, is_out, idx):
        name = C.c_char_p()
        shape = (C.c_int64 * 8)()
        rank = C.c_size_t()
        check(lib().zr_session_io(self._h, is_out, idx, C.byref(name), shape, C.byref(rank)))
        return name.value.decode(), tuple(shape[i] for i in range(rank.value))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._LIB is not None:
            _lib._LIB.zr_session_destroy(h)
            self._h = None

    def num_inputs(self) -> int:
        return len(self._inputs)

    def num_outputs(self) -> int:
        return len(self._outputs)

    def inputs(self):
        return list(self._inputs)

    def outputs(self):
        return list(self._outputs)

    def output_shapes(self, batch: int):
        return [(batch,) + s[1:] for _, s in self._outputs]

    def estimate(self, x: np.ndarray) -> List[np.ndarray]:
        """NeuralNetwork::estimate (nn/mod.rs:450): x is [B, C, H, W] f32 (host)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        want = self._inputs[0][1][1:]
        if x.ndim != 4 or tuple(x.shape[1:]) != tuple(want):
            raise ValueError(f"input shape {x.shape} does not match [B, {want}]")
        b = x.shape[0]
        outs = [np.empty(s, np.float32) for s in self.output_shapes(b)]
        ins = (C.c_void_p * 1)(x.ctypes.data)
        ptrs = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        check(lib().zr_session_run(self._h, b, ins, 1, ptrs, len(outs)))
        return outs

    def estimate_device(self, batch: int, d_input: int, d_outputs: Sequence[int], stream=None):
        """Enqueue inference on device-resident tensors (pointers as ints)."""
        ptrs = (C.c_void_p * len(d_outputs))(*d_outputs)
        check(lib().zr_session_run_async(self._h, batch, d_input, ptrs, len(d_outputs), stream))

    def stats(self):
        b, f, n = C.c_double(), C.c_double(), C.c_size_t()
        check(lib().zr_session_stats(self._h, C.byref(b), C.byref(f), C.byref(n)))
        return {"bytes_per_image": b.value, "flops_per_image": f.value, "launches": n.value}


class ColorMapper:
    """ColorMapper::linear (nn/mod.rs:134-168)."""

    def __init__(self, lo: float, hi: float):
        if not hi > lo:
            raise ValueError("ColorMapper range must satisfy end > start")
        self.lo, self.hi = float(lo), float(hi)

    @staticmethod
    def linear(lo: float, hi: float) -> "ColorMapper":
        return ColorMapper(lo, hi)


def views_array(views) -> "C.Array":
    arr = (View * len(views))()
    for i, v in enumerate(views):
        arr[i] = View(*v) if not isinstance(v, View) else v
    return arr


class Cnn:
    """Cnn (nn/mod.rs:30-127): a NeuralNetwork plus the image->tensor map.

    ``estimate_views`` samples every view (RotatedRect in root-image coordinates, as a
    (cx, cy, w, h, rad) tuple) of one RGBA8 image on the GPU and runs the network on all of
    them as one batch.
    """

    def __init__(self, nn: NeuralNetwork, color_mapper: ColorMapper):
        if nn.num_inputs() != 1:
            raise ValueError(f"CNN network has to take exactly 1 input, this one takes "
                             f"{nn.num_inputs()}")
        shape = nn.inputs()[0][1]
        if len(shape) != 4 or shape[1] != 3:
            raise ValueError(f"invalid model input shape for NCHW CNN: {shape}")
        self.nn = nn
        self.color_mapper = color_mapper
        self.input_resolution = (int(shape[3]), int(shape[2]))

    def estimate_views(self, image: np.ndarray, views) -> List[np.ndarray]:
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 4:
            raise ValueError("image must be HxWx4 RGBA8")
        h, w = img.shape[:2]
        va = views_array(views)
        outs = [np.empty(s, np.float32) for s in self.nn.output_shapes(len(views))]
        ptrs = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        check(lib().zr_cnn_estimate_views(self.nn._h, img.ctypes.data, w, h, w * 4, va,
                                          len(views), self.color_mapper.lo,
                                          self.color_mapper.hi, ptrs))
        return outs

    def estimate_views_device(self, frames: Sequence[Frame], views, view_frame,
                              d_outputs: Sequence[int], stream=None):
        fa = (Frame * len(frames))(*frames)
        va = views_array(views)
        vf = (C.c_uint32 * len(views))(*view_frame)
        ptrs = (C.c_void_p * len(d_outputs))(*d_outputs)
        check(lib().zr_cnn_estimate_views_async(self.nn._h, fa, len(frames), va, vf, len(views),
                                                self.color_mapper.lo, self.color_mapper.hi,
                                                ptrs, stream))


def preprocess_views_device(frames: Sequence[Frame], views, view_frame, ow: int, oh: int,
                            lo: float, hi: float, d_out: int, stream=None):
    fa = (Frame * len(frames))(*frames)
    va = views_array(views)
    vf = (C.c_uint32 * len(views))(*view_frame)
    check(lib().zr_preprocess_views_async(fa, len(frames), va, vf, len(views), ow, oh, lo, hi,
                                          d_out, stream))


def model_bytes(name: str) -> bytes:
    with open(os.path.join(MODELS_DIR, name + ".onnx"), "rb") as f:
        return f.read()
