"""ctypes binding of the C ABI in include/zaru_hip.h (zaru_amd/lib/libzaru_hip.so).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C zaru_amd/csrc``).
There is no fallback: if the shared object is missing or has no GPU to run on, every
entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libzaru_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "zaru_hip.h")

ZR_OK = 0
ERRORS = {-1: "invalid argument", -2: "model", -3: "device", -4: "shape", -5: "internal"}


class ZaruError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)} error: {msg}")
        self.code = code


class View(C.Structure):
    """zr_view: RotatedRect in root-image coordinates (centre, size, clockwise radians)."""
    _fields_ = [("cx", C.c_float), ("cy", C.c_float), ("w", C.c_float), ("h", C.c_float),
                ("rad", C.c_float)]


class Frame(C.Structure):
    _fields_ = [("rgba", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32),
                ("row_stride", C.c_uint64)]


_LIB = None

# (name, restype, argtypes) for every exported entry point of include/zaru_hip.h
_P, _SZ, _F, _U32, _I = C.c_void_p, C.c_size_t, C.c_float, C.c_uint32, C.c_int
SIGNATURES = [
    ("zr_session_create", _I, [_P, _SZ, _P, _SZ, _I, C.POINTER(_P)]),
    ("zr_session_destroy", None, [_P]),
    ("zr_session_num_io", _I, [_P, _I, C.POINTER(_SZ)]),
    ("zr_session_io", _I, [_P, _I, _SZ, C.POINTER(C.c_char_p), _P, C.POINTER(_SZ)]),
    ("zr_session_run", _I, [_P, _SZ, _P, _SZ, _P, _SZ]),
    ("zr_session_run_async", _I, [_P, _SZ, _P, _P, _SZ, _P]),
    ("zr_cnn_estimate_views", _I, [_P, _P, _U32, _U32, _SZ, _P, _SZ, _F, _F, _P]),
    ("zr_cnn_estimate_views_async", _I, [_P, _P, _SZ, _P, _P, _SZ, _F, _F, _P, _P]),
    ("zr_preprocess_views_async", _I, [_P, _SZ, _P, _P, _SZ, _U32, _U32, _F, _F, _P, _P]),
    ("zr_detection_candidates_async", _I, [_P, _P, _U32, _U32, _U32, _F, _U32, _P, _P, _P]),
    ("zr_track_seed_async", _I, [_P, _SZ, _P, _P, _P]),
    ("zr_track_update_async", _I, [_P, _SZ, _P, _P, _SZ, _P, _SZ, _P, _P, _P]),
    ("zr_view_describe", _I, [_P, _SZ, _U32, _P]),
    ("zr_detect_post_async", _I, [_P, _P, _P, _P, _SZ, _P, _P, _P, _SZ, _P, _SZ, _U32, _U32, _P, _P]),
    ("zr_detect_post_mapped_async", _I, [_P, _P, _P, _P, _SZ, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    ("zr_due_compact_async", _I, [_P, _SZ, _P, _P, _P, _P, _P, _P]),
    ("zr_track_lost_compact_async", _I, [_P, _SZ, _P, _P, _P, _P, _P, _P]),
    ("zr_track_reseed_best_async", _I, [_P, _P, _SZ, _P, _SZ, _P, _P, _P, _P, _P]),
    ("zr_cnn_estimate_device_views_count_async", _I, [_P, _P, _SZ, _P, _SZ, _P, _F, _F, _P, _P]),
    ("zr_track_seed_detections_async", _I, [_P, _P, _SZ, _P, _P, _P, _SZ, _P, _F, _I, _P, _P, _P, _P]),
    ("zr_hand_manage_async", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P, _SZ, _P, C.c_double, _I,
                                  _P, _P, _P]),
    ("zr_comm_unique_id", _I, [_P]),
    ("zr_comm_create", _I, [_P, _I, _I, _I, C.POINTER(_P)]),
    ("zr_comm_destroy", None, [_P]),
    ("zr_comm_size", _I, [_P, C.POINTER(_I)]),
    ("zr_comm_all_gather_async", _I, [_P, _P, _P, _SZ, _P]),
    ("zr_debug_glibc_math", _I, [_I, _P, _P, _P, _SZ, _P]),
    ("zr_cnn_estimate_device_views_async", _I, [_P, _P, _SZ, _P, _SZ, _F, _F, _P, _P]),
    ("zr_jpeg_decoder_create", _I, [C.c_int, _P]),
    ("zr_jpeg_decoder_destroy", None, [_P]),
    ("zr_jpeg_info", _I, [_P, _SZ, _P, _P]),
    ("zr_jpeg_decode_async", _I, [_P, _P, _SZ, _P, _SZ, _P]),
    ("zr_jpeg_decode_batch_async", _I, [_P, _SZ, _P, _P, _P, _P, _P]),
    ("zr_jpeg_coefficients", _I, [_P, _SZ, _P, _SZ, _P]),
    ("zr_jpeg_decoder_status", _I, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(_I)]),
    ("zr_jpeg_frame_errors", _I, [_P, _P, _SZ, C.POINTER(_SZ)]),
    ("zr_session_stats", _I, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(_SZ)]),
    ("zr_plan_describe", _I, [_P, _SZ, _P, _SZ, _P, _SZ, C.POINTER(_SZ)]),
    ("zr_profile_enable", _I, [_P, _I]),
    ("zr_profile_read", _I, [_P, _P, _SZ, C.POINTER(_SZ)]),
    ("zr_last_error", C.c_char_p, []),
    ("zr_device_count", _I, [C.POINTER(_I)]),
    ("zr_malloc", _I, [C.POINTER(_P), _SZ]),
    ("zr_free", _I, [_P]),
    ("zr_host_alloc", _I, [C.POINTER(_P), _SZ]),
    ("zr_host_free", _I, [_P]),
    ("zr_memcpy_async", _I, [_P, _P, _SZ, _I, _P]),
    ("zr_memcpy2d_async", _I, [_P, _SZ, _P, _SZ, _SZ, _SZ, _I, _P]),
    ("zr_stream_create", _I, [C.POINTER(_P)]),
    ("zr_stream_destroy", _I, [_P]),
    ("zr_stream_synchronize", _I, [_P]),
    ("zr_event_create", _I, [C.POINTER(_P)]),
    ("zr_event_create_timing", _I, [C.POINTER(_P)]),
    ("zr_event_elapsed", _I, [C.POINTER(_F), _P, _P]),
    ("zr_stream_wait_event", _I, [_P, _P]),
    ("zr_event_destroy", _I, [_P]),
    ("zr_event_record", _I, [_P, _P]),
    ("zr_event_synchronize", _I, [_P]),
    ("zr_event_query", _I, [_P]),
]


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ZaruError(-3, f"HIP extension not built: {LIB_PATH} missing "
                            "(run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def check(rc: int):
    if rc != ZR_OK:
        raise ZaruError(rc, lib().zr_last_error().decode(errors="replace"))


def device_count() -> int:
    n = C.c_int(0)
    check(lib().zr_device_count(C.byref(n)))
    return n.value


def plan_describe(onnx: bytes, outputs=None) -> str:
    sel = (C.c_uint32 * len(outputs))(*outputs) if outputs else None
    need = C.c_size_t(0)
    check(lib().zr_plan_describe(onnx, len(onnx), sel, len(outputs or []), None, 0,
                                 C.byref(need)))
    buf = C.create_string_buffer(need.value)
    check(lib().zr_plan_describe(onnx, len(onnx), sel, len(outputs or []), buf, need.value,
                                 C.byref(need)))
    return buf.value.decode()


class DeviceBuffer:
    """Owning device allocation (through the C ABI helpers, no HIP/torch import needed)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().zr_malloc(C.byref(p), max(4, int(nbytes))))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    @classmethod
    def from_array(cls, a, stream=None):
        import numpy as np
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a, stream)
        return b

    def upload(self, a, stream=None):
        import numpy as np
        a = np.ascontiguousarray(a)
        check(lib().zr_memcpy_async(self.ptr, a.ctypes.data, a.nbytes, 0, stream))
        check(lib().zr_stream_synchronize(stream))

    def download(self, shape, dtype, stream=None):
        import numpy as np
        out = np.empty(shape, dtype)
        check(lib().zr_memcpy_async(out.ctypes.data, self.ptr, out.nbytes, 1, stream))
        check(lib().zr_stream_synchronize(stream))
        return out

    def free(self):
        if getattr(self, "ptr", None) and _LIB is not None:
            _LIB.zr_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


def synchronize(stream=None):
    check(lib().zr_stream_synchronize(stream))


class _StdoutToStderr:
    """RCCL prints a version banner on stdout when it initialises; bench.py's one JSON line on
    stdout must stay the only thing there, so fd 1 points at stderr meanwhile."""

    def __enter__(self):
        import os
        import sys
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        import os
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Comm:
    """The node communicator of the multi-GPU path (zr_comm_*): RCCL over xGMI,
    one rank per GPU.  `unique_id()` on one rank; its 128 bytes reach the others by any side
    channel (bench.py: the gloo control group); `Comm(uid, world, rank, device)` joins."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        with _StdoutToStderr():
            check(lib().zr_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid: bytes, world: int, rank: int, device: int):
        if len(uid) != 128:
            raise ValueError("a communicator id is 128 bytes")
        p = C.c_void_p()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        with _StdoutToStderr():
            check(lib().zr_comm_create(buf, world, rank, device, C.byref(p)))
        self.ptr, self.world, self.rank = p.value, world, rank

    def size(self) -> int:
        n = C.c_int()
        check(lib().zr_comm_size(self.ptr, C.byref(n)))
        return n.value

    def all_gather_async(self, d_send: int, d_recv: int, nbytes: int, stream=None):
        check(lib().zr_comm_all_gather_async(self.ptr, d_send, d_recv, nbytes, stream))

    def close(self):
        if getattr(self, "ptr", None) and _LIB is not None:
            _LIB.zr_comm_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()
