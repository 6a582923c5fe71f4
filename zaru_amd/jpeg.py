"""JPEG frame source over the C ABI: baseline JPEG bytes -> RGBA8 frames in
HBM, byte-identical to the reference's libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:
164-182; `decode_jpeg` returns RGBA with alpha 255).  Entropy decoding runs on the calling
thread, the pixel stages on the GPU (kernels/jpeg.hip)."""
from __future__ import annotations

import ctypes as C

from ._lib import DeviceBuffer, check, lib


def info(data: bytes):
    """(width, height) of a JPEG stream (SOF parse, no decoding)."""
    w, h = C.c_uint32(), C.c_uint32()
    check(lib().zr_jpeg_info(data, len(data), C.byref(w), C.byref(h)))
    return w.value, h.value


class JpegDecoder:
    """A reusable decoder (zr_jpeg_decoder): coefficient staging and planes grow on demand."""

    def __init__(self, device: int = 0):
        p = C.c_void_p()
        check(lib().zr_jpeg_decoder_create(device, C.byref(p)))
        self._h = p.value

    def close(self):
        if self._h:
            lib().zr_jpeg_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode_into(self, data: bytes, d_rgba: int, row_stride: int, stream=None):
        """Enqueue the decode of `data` into the device buffer at `d_rgba` (RGBA8 rows of
        `row_stride` bytes) on `stream` (default stream when None)."""
        check(lib().zr_jpeg_decode_async(self._h, data, len(data), d_rgba, row_stride, stream))

    def decode(self, data: bytes):
        """Decode to a host numpy array [H, W, 4] (test / convenience path)."""
        w, h = info(data)
        buf = DeviceBuffer(w * h * 4)
        try:
            self.decode_into(data, buf.ptr, w * 4, None)
            return buf.download((h, w, 4), "uint8")
        finally:
            buf.free()
