"""JPEG frame source over the C ABI: baseline JPEG bytes -> RGBA8 frames in
HBM, byte-identical to the reference's libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:
164-182; `decode_jpeg` returns RGBA with alpha 255).  Streams with restart intervals are
entropy-decoded on the GPU, one thread per interval (kernels/jpeg_huff.hip); others on the
calling thread.  The pixel stages always run on the GPU (kernels/jpeg.hip)."""
from __future__ import annotations

import ctypes as C

from ._lib import DeviceBuffer, check, lib


def info(data: bytes):
    """(width, height) of a JPEG stream (SOF parse, no decoding)."""
    w, h = C.c_uint32(), C.c_uint32()
    check(lib().zr_jpeg_info(data, len(data), C.byref(w), C.byref(h)))
    return w.value, h.value


class _Layout(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("ncomp", C.c_uint32),
                ("h_samp", C.c_uint32), ("v_samp", C.c_uint32), ("total_blocks", C.c_uint32),
                ("bw", C.c_uint32 * 3), ("bh", C.c_uint32 * 3), ("qsel", C.c_uint32 * 3),
                ("quant", (C.c_uint16 * 64) * 4)]


def coefficients(data: bytes):
    """Host-only entropy decoding (no GPU): (layout dict, int16 [total_blocks, 64] quantised
    coefficients in natural order, components concatenated)."""
    import numpy as np
    lay = _Layout()
    check(lib().zr_jpeg_coefficients(data, len(data), None, 0, C.byref(lay)))
    coef = np.empty((lay.total_blocks, 64), np.int16)
    check(lib().zr_jpeg_coefficients(data, len(data), coef.ctypes.data, lay.total_blocks, C.byref(lay)))
    d = {k: getattr(lay, k) for k in ("width", "height", "ncomp", "h_samp", "v_samp", "total_blocks")}
    d["bw"], d["bh"], d["qsel"] = list(lay.bw), list(lay.bh), list(lay.qsel)
    d["quant"] = np.array([list(r) for r in lay.quant], np.uint16)
    return d, coef


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

    def decode_batch_into(self, datas, d_rgba, row_strides, stream=None):
        """Enqueue the decodes of the byte strings `datas` into the device buffers `d_rgba[i]`
        (RGBA8 rows of `row_strides[i]` bytes) on `stream`: one Huffman launch for all frames
        that decode on the device (zr_jpeg_decode_batch_async)."""
        n = len(datas)
        if not (len(d_rgba) == len(row_strides) == n):
            raise ValueError("datas, d_rgba and row_strides differ in length")
        bufs = (C.c_char_p * n)(*datas)
        lens = (C.c_size_t * n)(*[len(d) for d in datas])
        outs = (C.c_void_p * n)(*d_rgba)
        strides = (C.c_size_t * n)(*row_strides)
        check(lib().zr_jpeg_decode_batch_async(self._h, n, bufs, lens, outs, strides, stream))

    def status(self):
        """(device entropy decodes, host entropy decodes since creation, corrupt flag of the last
        call)."""
        g, h, c = C.c_uint64(), C.c_uint64(), C.c_int()
        check(lib().zr_jpeg_decoder_status(self._h, C.byref(g), C.byref(h), C.byref(c)))
        return g.value, h.value, c.value

    def frame_errors(self):
        """Per frame of the last call: True where its (device-decoded) entropy data was corrupt;
        the rest of such an interval decodes as zero blocks (libjpeg-turbo's rule)."""
        import numpy as np
        n = C.c_size_t()
        check(lib().zr_jpeg_frame_errors(self._h, None, 0, C.byref(n)))
        flags = np.zeros(n.value, np.int32)
        check(lib().zr_jpeg_frame_errors(self._h, flags.ctypes.data, n.value, C.byref(n)))
        return flags.astype(bool)

    def decode(self, data: bytes):
        """Decode to a host numpy array [H, W, 4] (test / convenience path)."""
        w, h = info(data)
        buf = DeviceBuffer(w * h * 4)
        try:
            self.decode_into(data, buf.ptr, w * 4, None)
            return buf.download((h, w, 4), "uint8")
        finally:
            buf.free()
