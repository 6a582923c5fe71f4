"""Host-side mirror of Zaru's detection / landmark API (C++ in zaru_amd/csrc/host, built as
``zaru_amd/lib/_zaru_host*.so``) over the HIP C ABI.

Names follow the reference: ``Detector`` (crates/zaru/src/detection.rs), ``NonMaxSuppression``
(detection/nms.rs), ``Estimator`` / ``LandmarkTracker`` (landmark.rs), ``Rect`` /
``RotatedRect`` (zaru-image/src/rect.rs), plus the batched ``DetectTrackPipeline`` that runs a
whole batch of device-resident frames through detect -> track.
"""
from __future__ import annotations

import glob
import importlib.util
import os

from ._lib import LIB_DIR, ZaruError, lib

_MOD = None


def _load():
    global _MOD
    if _MOD is not None:
        return _MOD
    lib()  # the C ABI library must be present (and is what the host module links)
    cands = glob.glob(os.path.join(LIB_DIR, "_zaru_host*.so"))
    if not cands:
        raise ZaruError(-3, f"host extension not built in {LIB_DIR} (run __graft_entry__.build())")
    spec = importlib.util.spec_from_file_location("zaru_amd._zaru_host", cands[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.set_models_dir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "models"))
    _MOD = mod
    return mod


def __getattr__(name):
    return getattr(_load(), name)
