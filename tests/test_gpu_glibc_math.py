"""glibc_math.h on the GPU (the functions kernels/track.hip evaluates) against this machine's
glibc on the host, bit for bit: 2^24 strided bit patterns per function (every binade, both
signs, NaN/Inf/denormals) and 2^22 atan2f pairs.  The host build of the same source is checked
over all 2^32 inputs by tools/libm_exhaustive.cpp (tests/test_glibc_math_cpu.py)."""
import ctypes as C
import os

import numpy as np
import pytest

from zaru_amd._lib import DeviceBuffer, check, lib

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def glibc():
    L = C.CDLL(os.path.join(REPO, "tests", "native", "libglibc_math_check.so"))
    L.gm_glibc.restype = None
    L.gm_glibc.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    return L


def device_eval(fn, a, b=None):
    da = DeviceBuffer.from_array(a)
    db = DeviceBuffer.from_array(b) if b is not None else None
    out = DeviceBuffer(a.nbytes)
    check(lib().zr_debug_glibc_math(fn, da.ptr, db.ptr if db else None, out.ptr, a.size, None))
    return out.download(a.shape, np.float32)


def assert_bitwise(want, got, inputs):
    same = (want.view(np.uint32) == got.view(np.uint32)) | (np.isnan(want) & np.isnan(got))
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, [(hex(int(inputs.view(np.uint32)[i])), want[i], got[i]) for i in bad[:8]]


@pytest.mark.parametrize("fn,name", [(0, "sinf"), (1, "cosf"), (2, "expf"), (3, "atanf")])
def test_device_matches_glibc(fn, name):
    n = 1 << 24
    u = (np.arange(n, dtype=np.uint64) * 256 + 97).astype(np.uint32)  # stride 256 over 2^32
    a = u.view(np.float32).copy()
    want = np.empty_like(a)
    glibc().gm_glibc(fn, a.ctypes.data, None, want.ctypes.data, n)
    assert_bitwise(want, device_eval(fn, a), a)


def test_device_atan2f_matches_glibc():
    rng = np.random.default_rng(5)
    n = 1 << 22
    y = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32).copy()
    x = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32).copy()
    y[: n // 2] = rng.uniform(-500, 500, n // 2).astype(np.float32)
    x[: n // 2] = rng.uniform(-500, 500, n // 2).astype(np.float32)
    x[n // 2: n // 2 + 4096] = 1.0
    y[n // 2 + 4096: n // 2 + 8192] = 0.0
    want = np.empty_like(y)
    glibc().gm_glibc(4, y.ctypes.data, x.ctypes.data, want.ctypes.data, n)
    assert_bitwise(want, device_eval(4, y, x), y)
