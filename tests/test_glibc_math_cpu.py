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


VARIANT_CHILD = r"""
import ctypes as C, json, sys
import numpy as np
out = {}
for tag, path in (("fma", sys.argv[1]), ("nofma", sys.argv[2])):
    L = C.CDLL(path)
    for f in (L.gm_glibc, L.gm_mine):
        f.restype = None
        f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    L.gm_sweep.restype = C.c_uint64
    L.gm_sweep.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64]
    for fn, name in enumerate(("sinf", "cosf", "expf")):
        a = np.array(json.load(open(sys.argv[3]))[name], np.uint32).view(np.float32)
        g, m = np.empty_like(a), np.empty_like(a)
        L.gm_glibc(fn, a.ctypes.data, None, g.ctypes.data, a.size)
        L.gm_mine(fn, a.ctypes.data, None, m.ctypes.data, a.size)
        out[f"{tag}/{name}"] = bool((g.view(np.uint32) == m.view(np.uint32)).all())
        out[f"{tag}/{name}/sweep"] = int(L.gm_sweep(fn, 3, (1 << 32) // 4093, 4093))
print(json.dumps(out))
"""


@pytest.mark.parametrize("tunables", ["", "glibc.cpu.hwcaps=-AVX2,-FMA"])
def test_both_glibc_builds_are_restated(tunables):
    """glibc picks sinf / cosf / expf per CPU through IFUNCs: the -mfma builds on FMA hosts (this
    image, the GPU box), the baseline builds otherwise; they round differently on 36 of the 3 x 2^32
    inputs (tests/golden/glibc_fma_variant_inputs.json, tools/libm_variants.cpp).  With the
    baseline build forced (GLIBC_TUNABLES=glibc.cpu.hwcaps=-AVX2,-FMA) glibc must agree with the
    ZR_GLIBC_FMA=0 restatement on those inputs and disagree with the FMA one, and by default the
    reverse; a strided sweep must agree everywhere else.  profiles/r04_libm_exhaustive_nofma.json
    holds the all-inputs run of the baseline build under the same tunable."""
    import subprocess
    import sys
    nofma = os.path.join(REPO, "tests", "native", "libglibc_math_check_nofma.so")
    if not os.path.exists(nofma):
        pytest.fail(f"{nofma} missing: run __graft_entry__.build()")
    env = dict(os.environ)
    if tunables:
        env["GLIBC_TUNABLES"] = tunables
    r = subprocess.run([sys.executable, "-c", VARIANT_CHILD, LIB, nofma,
                        os.path.join(REPO, "tests", "golden", "glibc_fma_variant_inputs.json")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout)
    resolved = "nofma" if tunables else "fma"
    other = "fma" if tunables else "nofma"
    for name in ("sinf", "cosf", "expf"):
        assert res[f"{resolved}/{name}"], (tunables, name)
        assert not res[f"{other}/{name}"], (tunables, name)
        assert res[f"{resolved}/{name}/sweep"] == 0, (tunables, name)


def test_exhaustive_record_is_clean():
    """profiles/r03_libm_exhaustive.json: tools/libm_exhaustive.cpp over all 2^32 inputs."""
    rec = json.load(open(os.path.join(REPO, "profiles", "r03_libm_exhaustive.json")))
    assert rec["inputs_each"] == 1 << 32 and rec["atan2f_pairs"] == 1 << 32
    for k in ("sinf", "cosf", "expf", "atanf", "atan2f"):
        assert rec[f"{k}_mismatch"] == 0, k
    # the baseline (ZR_GLIBC_FMA=0) build against glibc forced to its baseline IFUNCs
    rec = json.load(open(os.path.join(REPO, "profiles", "r04_libm_exhaustive_nofma.json")))
    assert rec["fma_build"] == 0 and rec["inputs_each"] == 1 << 32 and rec["atan2f_pairs"] >= 1 << 30
    for k in ("sinf", "cosf", "expf", "atanf", "atan2f"):
        assert rec[f"{k}_mismatch"] == 0, k
