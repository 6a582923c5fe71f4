"""The device restatement of glibc's sinf / cosf / expf / atanf / atan2f
(zaru_amd/csrc/kernels/glibc_math.h, used by kernels/track.hip for LandmarkTracker::track_impl
on the device) compiled for the host, against this machine's glibc 2.35: strided sweeps over the
f32 bit patterns plus random atan2f pairs.  The full 2^32 sweep (every input of every function,
2^32 random atan2f pairs) is tools/libm_exhaustive.cpp; its committed result is checked here too.
Reference use: Rust f32::{sin, cos, exp, atan2} -> glibc (rect.rs:287-325,417-423,
matrix.rs:571-579, vector.rs:568-573, num.rs:6-8)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "tests", "native", "libglibc_math_check.so")
FNS = {"sinf": 0, "cosf": 1, "expf": 2, "atanf": 3}


@pytest.fixture(scope="module")
def gm():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build()")
    L = C.CDLL(LIB)
    L.gm_sweep.restype = C.c_uint64
    L.gm_sweep.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64]
    for f in (L.gm_glibc, L.gm_mine):
        f.restype = None
        f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    return L


@pytest.mark.parametrize("name", list(FNS))
def test_strided_sweep_matches_glibc(gm, name):
    # stride 251 (prime): 17.1 M inputs covering every binade and both signs
    n = (1 << 32) // 251
    assert gm.gm_sweep(FNS[name], 7, n, 251) == 0


@pytest.mark.parametrize("name", list(FNS))
def test_special_inputs_match_glibc(gm, name):
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.17549435e-38, 3.4028235e38,
                         -3.4028235e38, 0.78539816, 0.7853982, 120.0, -120.0, 119.99999, 88.0, 88.72283,
                         88.72284, -103.97208, -103.97207, -87.33655, 2.0 ** 25, -(2.0 ** 25), 0.4375,
                         1.1875, 2.4375, 0.6875, np.pi, -np.pi, np.pi / 2, 1e30, -1e30], np.float32)
    a = np.ascontiguousarray(specials)
    want, got = np.empty_like(a), np.empty_like(a)
    gm.gm_glibc(FNS[name], a.ctypes.data, None, want.ctypes.data, a.size)
    gm.gm_mine(FNS[name], a.ctypes.data, None, got.ctypes.data, a.size)
    same = (want.view(np.uint32) == got.view(np.uint32)) | (np.isnan(want) & np.isnan(got))
    assert same.all(), a[~same]


def test_atan2f_random_pairs_match_glibc(gm):
    rng = np.random.default_rng(11)
    n = 1 << 21
    y = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    # the landmark / detection angle inputs: moderate coordinates differences and dot products
    y[: n // 2] = rng.uniform(-500, 500, n // 2).astype(np.float32)
    x[: n // 2] = rng.uniform(-500, 500, n // 2).astype(np.float32)
    x[n // 2: n // 2 + 1000] = 1.0
    want, got = np.empty_like(y), np.empty_like(y)
    gm.gm_glibc(4, y.ctypes.data, x.ctypes.data, want.ctypes.data, n)
    gm.gm_mine(4, y.ctypes.data, x.ctypes.data, got.ctypes.data, n)
    same = (want.view(np.uint32) == got.view(np.uint32)) | (np.isnan(want) & np.isnan(got))
    assert same.all(), np.nonzero(~same)[0][:10]


def test_exhaustive_record_is_clean():
    """profiles/r03_libm_exhaustive.json: tools/libm_exhaustive.cpp over all 2^32 inputs."""
    rec = json.load(open(os.path.join(REPO, "profiles", "r03_libm_exhaustive.json")))
    assert rec["inputs_each"] == 1 << 32 and rec["atan2f_pairs"] == 1 << 32
    for k in ("sinf", "cosf", "expf", "atanf", "atan2f"):
        assert rec[f"{k}_mismatch"] == 0, k
