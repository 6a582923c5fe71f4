"""BASELINE.json configs C1 and C2 on the GPU, through the C ABI.

C1: the 640x480 plumbing frame (tests/configs.py) through Detector::detect on the HIP backend
    equals the oracle's CPU chain on the same frame (same detections, conf
    and box within the f32 noise).
C2: batch 64 of seeded 128x128 BlazeFace tensors (seed 0x5A52550000000002) through
    zr_session_run against the f64 oracle, image by image (|err| <= 2e-3, the bar of
    test_gpu_parity.py), and batch-64 results bitwise equal to single-image runs.
"""
import os

import numpy as np
import pytest

import oracle as O

from configs import c1_frame, c2_batch

pytestmark = pytest.mark.gpu

MODELS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zaru_amd", "models")
ABS_TOL = 2e-3


def test_c1_detector_matches_cpu_chain():
    import zaru_amd.host as H
    img = c1_frame()
    r = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, 640, 480), 128, 128)
    v = O.view_compose(O.view_full(640, 480), r)
    reg, cls = O.Net(os.path.join(MODELS, "face_detection_short_range.onnx"), f64=False).run(
        O.preproc(img, v, 128, 128, -1.0, 1.0)[None])
    want = O.detect_post(O.FACE, reg[0], cls[0], 640, 480, 128, 128)
    got = H.Detector("face").detect(img)
    assert len(got) == len(want) == 1
    for a, b in zip(got, want):
        assert abs(a.confidence() - b.conf) <= 1e-4
        assert abs(a.angle() - b.angle) <= 2e-4
        assert np.allclose(a.bounding_rect().tuple(), b.rect.tuple(), atol=2e-3 * 5)


def test_c2_blazeface_batch64_vs_f64():
    from zaru_amd.nn import NeuralNetwork, model_bytes
    x = c2_batch()
    nn = NeuralNetwork.from_onnx(model_bytes("face_detection_short_range")).load()
    reg, cls = nn.estimate(x)
    assert reg.shape == (64, 896, 16) and cls.shape == (64, 896, 1)
    ref = O.Net(os.path.join(MODELS, "face_detection_short_range.onnx"), f64=True)
    worst = 0.0
    for i in range(64):
        r64, c64 = ref.run(x[i:i + 1], as_f64=True)
        worst = max(worst, float(np.abs(reg[i] - r64[0]).max()), float(np.abs(cls[i] - c64[0]).max()))
    print(f"C2: max|gpu - f64| over 64 images = {worst:.3e}")
    assert worst <= ABS_TOL
    for i in (0, 31, 63):
        one = nn.estimate(x[i:i + 1])
        assert np.array_equal(one[0][0], reg[i]) and np.array_equal(one[1][0], cls[i])
