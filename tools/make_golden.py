#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (it needs /root/reference for the reference's own test images;
the GPU box never runs this).  Everything it writes is data:

* reference_kat.json   -- the reference's own known-answer unit tests, re-expressed as data
                          (nms.rs:169-218, rect.rs:451-718, image/tests.rs:15-139,
                          nn/mod.rs:724-733, face/detection.rs:164-173, mediapipe.rs:563-624).
* sad_linus_face.npz   -- BlazeFace input for crates/zaru/src/face/detection.rs:164-173
                          (sad_linus.jpg, letterboxed as detection.rs:224-228), stored as the
                          uint8 colour codes the ColorMapper maps, plus f64-oracle outputs.
* sad_linus_mesh.npz   -- FaceMesh V1 inputs for mediapipe.rs:603-624 (0 deg, +-10 deg views of
                          sad_linus_cropped.jpg), same encoding, plus f64-oracle outputs.
* models_f64.npz       -- two seeded random inputs per hot-path model (codes k in 0..255) and
                          the f64-oracle outputs (SURVEY.md §8c fixture F2).
* decode_cases.npz     -- raw detector outputs (real + crafted overlapping candidates) with the
                          oracle's decoded, NMS'd, image-mapped detections (fixture F3).
* nms_ties.npz         -- > 20 saturated (1.0f) tied candidates per frame, Average and Remove
                          mode outputs of the oracle (anchor-order ties; unpinned by Rust above
                          20 candidates).  `python tools/make_golden.py ties` remakes only this.

JPEG decoding here uses PIL/libjpeg; the reference uses zune-jpeg, so pixels may differ by
+-1.  That is why fixtures store decoded colour codes, never the JPEG.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")
MODELS = os.path.join(REPO, "zaru_amd", "models")
REF_IMG = "/root/reference/3rdparty/img"

TAU = float(np.float32(2 * math.pi))
F32_PI = np.float32(math.pi)


def deg_to_rad_f32(d: float) -> float:
    """Rust f32::to_radians: self * (PI / 180.0) in f32."""
    return float(np.float32(d) * (F32_PI / np.float32(180.0)))


# ------------------------------------------------------------------ known-answer tests
COLORS = {  # image/mod.rs Color constants (RGBA)
    "NONE": [0, 0, 0, 0],
    "BLACK": [0, 0, 0, 255],
    "WHITE": [255, 255, 255, 255],
    "RED": [255, 0, 0, 255],
    "GREEN": [0, 255, 0, 255],
    "YELLOW": [255, 255, 0, 255],
}


def reference_kat() -> dict:
    kat = {}
    # nn/mod.rs:724-733
    kat["color_mapper"] = [
        {"lo": -1.0, "hi": 1.0, "code": 0, "want": -1.0},
        {"lo": -1.0, "hi": 1.0, "code": 255, "want": 1.0},
        {"lo": 1.0, "hi": 2.0, "code": 0, "want": 1.0},
        {"lo": 1.0, "hi": 2.0, "code": 255, "want": 2.0},
    ]
    # detection/nms.rs:169-218 ; rects are from_center(x, y, w, h); scale(s) multiplies size
    kat["nms"] = [
        {"name": "nms_suppresses_non_maximum", "mode": "remove", "iou": 0.3,
         "dets": [[0.6, [0, 0, 1, 1]], [0.55, [0, 0, 1.5, 1.5]]],
         "want": [[0.6, [0, 0, 1, 1]]]},
        {"name": "nms_ignores_nonoverlapping", "mode": "remove", "iou": 0.3,
         "dets": [[1.0, [0, 0, 1, 1]], [1.0, [5, 0, 1, 1]]], "want_len": 2},
        {"name": "nma_averages_detections", "mode": "average", "iou": 0.0,
         "dets": [[1.0, [-1, 3, 1, 1]], [0.5, [-1, 3, 4, 4]]],
         "want": [[1.0, [-1, 3, 2, 2]]]},
    ]
    # rect.rs:451-718 (exact assert_eq cases; approx ones carry "tol")
    kat["iou"] = [
        {"a": [9, 9, 1, 1], "b": [9, 9, 2, 2], "want": 0.25},
        {"a": [9, 9, 2, 2], "b": [9, 9, 1, 1], "want": 0.25},
    ]
    kat["intersection"] = [  # from_ranges(x0..=x1, y0..=y1) given as top-left boxes
        {"a_tl": [0, 0, 10, 10], "b_tl": [5, 5, 0, 0], "want_tl": [5, 5, 0, 0]},
        {"a_tl": [5, 5, 0, 0], "b_tl": [0, 0, 10, 10], "want_tl": [5, 5, 0, 0]},
        {"a_tl": [5, 5, 0, 0], "b_tl": [6, 0, 4, 10], "want_area": 0.0},
    ]
    kat["fit_aspect"] = [
        {"r": [10, 10, 50, 100], "aspect": [1, 1], "want": [10, 10, 100, 100]},
        {"r": [10, 10, 100, 50], "aspect": [1, 1], "want": [10, 10, 100, 100]},
        {"r": [10, 10, 100, 98], "aspect": [1, 1], "want": [10, 10, 100, 100]},
    ]
    kat["transform"] = [  # RotatedRect(from_top_left(...), rad); dir in/out
        {"tl": [0, 0, 1, 1], "rad": 0.0, "dir": "in", "p": [0, 0], "want": [0, 0]},
        {"tl": [0, 0, 1, 1], "rad": 0.0, "dir": "out", "p": [0, 0], "want": [0, 0]},
        {"tl": [0, 0, 1, 1], "rad": 0.0, "dir": "in", "p": [1, -1], "want": [1, -1]},
        {"tl": [0, 0, 1, 1], "rad": 0.0, "dir": "out", "p": [1, -1], "want": [1, -1]},
        {"tl": [10, 20, 1, 1], "rad": 0.0, "dir": "in", "p": [0, 0], "want": [-10, -20]},
        {"tl": [10, 20, 1, 1], "rad": 0.0, "dir": "in", "p": [10, 20], "want": [0, 0]},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "in", "p": [0.5, 0.5], "want": [0.5, 0.5]},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "out", "p": [0.5, 0.5], "want": [0.5, 0.5]},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "in", "p": [0, 0], "want": [0, 1], "tol": 1},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "out", "p": [0, 0], "want": [1, 0], "tol": 1},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "in", "p": [1, 0], "want": [0, 0], "tol": 1},
        {"tl": [0, 0, 1, 1], "rad": TAU / 4, "dir": "out", "p": [0, -1], "want": [2, 0], "tol": 1},
        {"tl": [10, 20, 1, 1], "rad": TAU / 2, "dir": "in", "p": [10, 20], "want": [1, 1], "tol": 1},
        {"tl": [10, 20, 1, 1], "rad": TAU / 2, "dir": "in", "p": [11, 21], "want": [0, 0], "tol": 1},
        {"tl": [10, 20, 1, 1], "rad": TAU / 2, "dir": "out", "p": [0, 0], "want": [11, 21], "tol": 1},
    ]
    kat["rrect_bounding"] = [  # want: [tl..., rad]
        {"rad": 0.0, "pts": [[0, 0], [1, 1]], "want_tl": [0, 0, 1, 1], "exact": True},
        {"rad": 0.0, "pts": [[0, 0], [10, 0]], "want_tl": [0, 0, 10, 0], "exact": True},
        {"rad": TAU / 2, "pts": [[0, 0], [1, 1]], "want_tl": [0, 0, 1, 1], "exact": False},
        {"rad": TAU / 4, "pts": [[0, 0], [1, 1]], "want_tl": [0, 0, 1, 1], "exact": False},
        {"rad": TAU / 4, "pts": [[0, 0], [9, 9]], "want_tl": [0, 0, 9, 9], "exact": True},
    ]
    # image/tests.rs:71-139: (image rows of colour names, view chain, expected get(x, y))
    kat["views"] = [
        {"name": "rotated_views/no_rot", "image": [["YELLOW", "WHITE"], ["WHITE", "RED"]],
         "chain": [[[0, 0, 2, 2], 0.0]],
         "get": [[0, 0, "YELLOW"], [1, 0, "WHITE"], [0, 1, "WHITE"], [1, 1, "RED"]]},
        {"name": "rotated_views/flip", "image": [["YELLOW", "WHITE"], ["WHITE", "RED"]],
         "chain": [[[0, 0, 2, 2], TAU / 2]],
         "get": [[0, 0, "RED"], [1, 0, "WHITE"], [0, 1, "WHITE"], [1, 1, "YELLOW"]]},
        {"name": "rotated_views/right_angle", "image": [["YELLOW", "WHITE"], ["WHITE", "RED"]],
         "chain": [[[0, 0, 2, 2], TAU / 4]],
         "get": [[0, 0, "WHITE"], [1, 0, "RED"], [0, 1, "YELLOW"], [1, 1, "WHITE"]]},
        {"name": "rotated_views/chained_flip", "image": [["YELLOW", "WHITE"], ["WHITE", "RED"]],
         "chain": [[[0, 0, 2, 2], TAU / 4], [[0, 0, 2, 2], TAU / 4]],
         "get": [[0, 0, "RED"], [1, 0, "WHITE"], [0, 1, "WHITE"], [1, 1, "YELLOW"]]},
        {"name": "rotated_views/bot_right", "image": [["YELLOW", "WHITE"], ["WHITE", "RED"]],
         "chain": [[[0, 0, 2, 2], TAU / 4], [[-1, 1, 2, 2], 0.0]],
         "get": [[0, 0, "NONE"], [1, 0, "YELLOW"]]},
        {"name": "view/green", "image": [["RED", "GREEN"]],
         "chain": [[[1, 0, 1, 1], 0.0]], "size": [1, 1], "get": [[0, 0, "GREEN"]]},
        {"name": "view/oob", "image": [["RED", "GREEN"]],
         "chain": [[[1, 0, 99, 100], 0.0]], "size": [99, 100],
         "get": [[0, 0, "GREEN"], [0, 1, "NONE"], [1, 0, "NONE"]]},
    ]
    # image/tests.rs:15-69 view_data: chained views -> resulting root-space rect (top-left form)
    kat["view_data"] = [
        {"image": [3, 3], "chain": [[1, 1, 1, 1]], "want_tl": [1, 1, 1, 1]},
        {"image": [3, 3], "chain": [[1, 1, 1, 1], [-1, -1, 2, 2]], "want_tl": [0, 0, 2, 2]},
        {"image": [3, 3], "chain": [[1, 1, 1, 1], [0, 0, 2, 2]], "want_tl": [1, 1, 2, 2]},
        {"image": [3, 3], "chain": [[1, 1, 1, 1], [-1, -1, 3, 3]], "want_tl": [0, 0, 3, 3]},
        {"image": [3, 3], "chain": [[1, 1, 2, 2]], "want_tl": [1, 1, 2, 2]},
        {"image": [3, 3], "chain": [[1, 1, 2, 2], [1, 1, 2, 2]], "want_tl": [2, 2, 2, 2]},
    ]
    # qualitative model tests (face/detection.rs:164-173, mediapipe.rs:575-624)
    kat["models"] = {
        "detects_face": {"min_conf": 0.8, "max_abs_angle_deg": 5.0},
        "facemesh": {"min_conf": 0.9, "angle_tol_deg": 5.0,
                     "cases": [{"view_deg": 0.0, "expect_deg": 0.0},
                               {"view_deg": 10.0, "expect_deg": -10.0},
                               {"view_deg": -10.0, "expect_deg": 10.0}]},
    }
    return kat


# ------------------------------------------------------------------ image fixtures
def load_rgba(name: str) -> np.ndarray:
    from PIL import Image
    return np.array(Image.open(os.path.join(REF_IMG, name)).convert("RGBA"))


def to_codes(x: np.ndarray, lo: float, hi: float) -> np.ndarray:
    """Invert ColorMapper::map: x = k*((hi-lo)/255)+lo -> k (exact for these tensors)."""
    adj = np.float32((np.float32(hi) - np.float32(lo)) / np.float32(255.0))
    k = np.rint((x - np.float32(lo)) / adj).astype(np.int32)
    assert k.min() >= 0 and k.max() <= 255
    back = k.astype(np.float32) * adj + np.float32(lo)
    assert np.array_equal(back, x), "colour code round trip must be exact"
    return k.astype(np.uint8)


def sad_linus_face():
    img = load_rgba("sad_linus.jpg")
    h, w = img.shape[:2]
    rect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, w, h), 128, 128)
    view = O.view_compose(O.view_full(w, h), rect)
    x = O.preproc(img, view, 128, 128, -1.0, 1.0)
    net = O.Net(os.path.join(MODELS, "face_detection_short_range.onnx"), f64=True)
    reg, cls = net.run(x[None], as_f64=True)
    dets = O.detect_post(O.FACE, reg[0].astype(np.float32), cls[0].astype(np.float32), w, h,
                         128, 128)
    np.savez_compressed(
        os.path.join(GOLD, "sad_linus_face.npz"),
        codes=to_codes(x, -1.0, 1.0), image_wh=np.array([w, h]),
        regressors=reg.astype(np.float32), classificators=cls.astype(np.float32),
        det_conf=np.array([d.conf for d in dets], np.float32),
        det_angle=np.array([d.angle for d in dets], np.float32),
        det_rect=np.array([d.rect.tuple() for d in dets], np.float32))
    return dets


def sad_linus_mesh():
    img = load_rgba("sad_linus_cropped.jpg")
    h, w = img.shape[:2]
    net = O.Net(os.path.join(MODELS, "face_landmark.onnx"), f64=True)
    codes, lms, flags, degs = [], [], [], []
    for deg in (0.0, 10.0, -10.0):
        rad = deg_to_rad_f32(abs(deg)) * (1 if deg >= 0 else -1)
        v1 = O.view_compose(O.view_full(w, h), O.RRect(O.Rect.from_top_left(0, 0, w, h), rad))
        lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, v1.rect.w, v1.rect.h), 192, 192)
        v2 = O.view_compose(v1, lrect)
        x = O.preproc(img, v2, 192, 192, -1.0, 1.0)
        lm, flag = net.run(x[None], as_f64=True)
        codes.append(to_codes(x, -1.0, 1.0))
        lms.append(lm.reshape(468, 3).astype(np.float32))
        flags.append(np.float32(flag.reshape(-1)[0]))
        degs.append(deg)
    np.savez_compressed(os.path.join(GOLD, "sad_linus_mesh.npz"), codes=np.stack(codes),
                        landmarks=np.stack(lms), flag_logit=np.array(flags, np.float32),
                        view_deg=np.array(degs, np.float32), image_wh=np.array([w, h]))


MODEL_SPECS = {  # name: (file, input size, lo, hi)
    "face_detection_short_range": ("face_detection_short_range.onnx", 128, -1.0, 1.0),
    "face_landmark": ("face_landmark.onnx", 192, -1.0, 1.0),
    "palm_detection_lite": ("palm_detection_lite.onnx", 192, 0.0, 1.0),
    "hand_landmark_lite": ("hand_landmark_lite.onnx", 224, 0.0, 1.0),
}


def models_f64():
    out = {}
    for mi, (name, (fn, s, lo, hi)) in enumerate(MODEL_SPECS.items()):
        net = O.Net(os.path.join(MODELS, fn), f64=True)
        rng = np.random.default_rng(0x5A525500 + mi)
        for k in range(2):
            codes = rng.integers(0, 256, size=(3, s, s), dtype=np.uint8)
            adj = np.float32((np.float32(hi) - np.float32(lo)) / np.float32(255.0))
            x = codes.astype(np.float32) * adj + np.float32(lo)
            outs = net.run(x[None], as_f64=True)
            out[f"{name}/{k}/codes"] = codes
            for oi, o in enumerate(outs):
                out[f"{name}/{k}/out{oi}"] = o.astype(np.float32)
        print("models_f64:", name, [o.shape for o in outs])
    np.savez_compressed(os.path.join(GOLD, "models_f64.npz"), **out)


def decode_cases():
    """Raw BlazeFace / palm outputs with known decoded results (fixture F3)."""
    cases = {}
    face = np.load(os.path.join(GOLD, "sad_linus_face.npz"))
    cases["face_real/boxes"] = face["regressors"][0]
    cases["face_real/confs"] = face["classificators"][0]
    cases["face_real/img"] = np.array([1280, 720])
    rng = np.random.default_rng(0x5A52550F)
    for kind, name, na, npar in ((O.FACE, "face", 896, 16), (O.PALM, "palm", 2016, 18)):
        for case in range(4):
            boxes = rng.normal(0, 3, size=(na, npar)).astype(np.float32)
            confs = rng.normal(-6, 1, size=(na,)).astype(np.float32)
            # plant clusters of overlapping candidates around a few anchors
            for _ in range(3 + case):
                a = int(rng.integers(0, na))
                nb = rng.integers(max(0, a - 12), min(na, a + 12), size=5)
                size = float(rng.uniform(8, 60))
                for j in [a, *nb.tolist()]:
                    confs[j] = np.float32(rng.uniform(0.1, 4.0))
                    boxes[j, 0:2] = rng.normal(0, 1.5, 2)
                    boxes[j, 2:4] = size * rng.uniform(0.85, 1.15, 2)
            img = [int(rng.integers(64, 2000)), int(rng.integers(64, 2000))]
            cases[f"{name}_{case}/boxes"] = boxes
            cases[f"{name}_{case}/confs"] = confs
            cases[f"{name}_{case}/img"] = np.array(img)
    # expected outputs
    for key in sorted({k.split("/")[0] for k in cases}):
        kind = O.PALM if key.startswith("palm") else O.FACE
        s = 128 if kind == O.FACE else 192
        iw, ih = (int(v) for v in cases[f"{key}/img"])
        dets = O.detect_post(kind, cases[f"{key}/boxes"], cases[f"{key}/confs"], iw, ih, s, s)
        rec = np.zeros((len(dets), 6 + 2 * 7), np.float32)
        for i, d in enumerate(dets):
            rec[i, 0], rec[i, 1] = d.conf, d.angle
            rec[i, 2:6] = d.rect.tuple()
            for k in range(d.nkp):
                rec[i, 6 + 2 * k], rec[i, 7 + 2 * k] = d.kp[k][0], d.kp[k][1]
        cases[f"{key}/want"] = rec
        print("decode case", key, "->", len(dets), "detections")
    np.savez_compressed(os.path.join(GOLD, "decode_cases.npz"), **cases)


def nms_ties():
    """Fixture nms_ties.npz: frames with more than 20 candidates of exactly equal,
    saturated confidence (logit 40 -> sigmoid 1.0f), in overlapping clusters whose members differ
    in box and keypoints, so the order inside a group changes the weighted sums' bits.  Expected
    outputs are the oracle's, i.e. ties in anchor order (a stable sort).  Rust's sort_unstable is
    stable only up to 20 elements (nms.rs:66); above that its order for these ties is NOT pinned
    by the reference: the fixture pins this build's documented rule, not the reference's."""
    cases = {}
    rng = np.random.default_rng(0x71E5)
    for kind, name, na, npar, side in ((O.FACE, "face", 896, 16, 128), (O.PALM, "palm", 2016, 18, 192)):
        for case in range(2):
            boxes = rng.normal(0, 3, size=(na, npar)).astype(np.float32)
            logits = np.full(na, -20.0, np.float32)
            for c in range(4 + case):  # clusters of 7-9 saturated candidates
                a = int(rng.integers(20, na - 20))
                members = sorted(set(rng.integers(a - 15, a + 15, size=9).tolist()))
                size = float(rng.uniform(10, 40))
                for j in members:
                    logits[j] = np.float32(40.0)
                    boxes[j, 0:2] = rng.normal(0, 1.0, 2)
                    boxes[j, 2:4] = size * rng.uniform(0.9, 1.1, 2)
            for j in rng.integers(0, na, size=3):  # a few unsaturated ones
                logits[j] = np.float32(rng.uniform(0.5, 3.0))
            img = np.array([int(rng.integers(200, 2000)), int(rng.integers(200, 2000))])
            key = f"{name}_{case}"
            cases[f"{key}/boxes"], cases[f"{key}/logits"], cases[f"{key}/img"] = boxes, logits, img
            conf = np.array([O.sigmoid(float(v)) for v in logits], np.float32)
            cand = conf[conf >= 0.5]
            _, inv, cnt = np.unique(cand.view(np.uint32), return_inverse=True, return_counts=True)
            cases[f"{key}/ties"] = np.array([len(cand), int((cnt[inv] > 1).sum())], np.int32)
            for mode in ("average", "remove"):
                dets = O.detect_post(kind, boxes, logits, int(img[0]), int(img[1]), side, side,
                                     remove=mode == "remove")
                rec = np.zeros((len(dets), 6 + 2 * 7), np.float32)
                for i, d in enumerate(dets):
                    rec[i, 0], rec[i, 1] = d.conf, d.angle
                    rec[i, 2:6] = d.rect.tuple()
                    for k in range(d.nkp):
                        rec[i, 6 + 2 * k], rec[i, 7 + 2 * k] = d.kp[k][0], d.kp[k][1]
                cases[f"{key}/want_{mode}"] = rec
            print("ties case", key, cases[f"{key}/ties"], len(cases[f"{key}/want_average"]),
                  len(cases[f"{key}/want_remove"]))
    np.savez_compressed(os.path.join(GOLD, "nms_ties.npz"), **cases)


# ------------------------------------------------------------------ SURVEY 8(f)-1 networks
NEXT_SPECS = {  # BlazeFace full range (face/detection.rs:61-94), FaceMesh V2 (mediapipe.rs:81-116)
    "face_detection_full_range": ("face_detection_full_range.onnx", 192, -1.0, 1.0),
    "face_landmarks_detector": ("face_landmarks_detector.onnx", 256, -1.0, 1.0),
    # face/eye.rs:29-64, face/landmark/multipie68.rs:46-118
    "iris_landmark": ("iris_landmark.onnx", 64, -1.0, 1.0),
    "landmarks_68_pfld": ("landmarks_68_pfld.onnx", 112, 0.0, 1.0),
    "slim_160_latest": ("slim_160_latest.onnx", 160, -1.0, 1.0),
}


def next_models():
    """next_models.npz: F2 (two seeded inputs -> f64 outputs) for both networks, plus the
    reference's qualitative model checks re-run on its own images: the full-range detector
    on the sad_linus.jpg letterbox (192^2) and FaceMesh V2 on sad_linus_cropped.jpg at
    0 / +-10 degrees (256^2).  The reference tests only ShortRangeNetwork / FaceMeshV1 with
    these images (face/detection.rs:164-173, mediapipe.rs:575-624); the same bars are applied
    here to the two networks that share their Network trait and extract code."""
    out = {}
    for mi, (name, (fn, s, lo, hi)) in enumerate(NEXT_SPECS.items()):
        net = O.Net(os.path.join(MODELS, fn), f64=True)
        rng = np.random.default_rng(0x5A525504 + mi)
        for k in range(2):
            codes = rng.integers(0, 256, size=(3, s, s), dtype=np.uint8)
            adj = np.float32((np.float32(hi) - np.float32(lo)) / np.float32(255.0))
            x = codes.astype(np.float32) * adj + np.float32(lo)
            outs = net.run(x[None], as_f64=True)
            out[f"{name}/{k}/codes"] = codes
            for oi, o in enumerate(outs):
                out[f"{name}/{k}/out{oi}"] = o.astype(np.float32)
        print("next_models:", name, [o.shape for o in outs])
    # full range on the sad_linus letterbox
    img = load_rgba("sad_linus.jpg")
    h, w = img.shape[:2]
    rect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, w, h), 192, 192)
    view = O.view_compose(O.view_full(w, h), rect)
    x = O.preproc(img, view, 192, 192, -1.0, 1.0)
    net = O.Net(os.path.join(MODELS, "face_detection_full_range.onnx"), f64=True)
    reg, cls = net.run(x[None], as_f64=True)
    dets = O.detect_post(O.FACE_FULL, reg[0].astype(np.float32), cls[0].astype(np.float32),
                         w, h, 192, 192)
    print("sad_linus full range:", [(d.conf, math.degrees(d.angle)) for d in dets])
    out["full_linus/codes"] = to_codes(x, -1.0, 1.0)
    out["full_linus/image_wh"] = np.array([w, h])
    out["full_linus/regressors"] = reg.astype(np.float32)
    out["full_linus/classificators"] = cls.astype(np.float32)
    # FaceMesh V2 on the cropped image, rotated views as in mediapipe.rs:603-624
    img = load_rgba("sad_linus_cropped.jpg")
    h, w = img.shape[:2]
    net = O.Net(os.path.join(MODELS, "face_landmarks_detector.onnx"), f64=True)
    codes, lms, flags, tongue, degs = [], [], [], [], []
    for deg in (0.0, 10.0, -10.0):
        rad = deg_to_rad_f32(abs(deg)) * (1 if deg >= 0 else -1)
        v1 = O.view_compose(O.view_full(w, h), O.RRect(O.Rect.from_top_left(0, 0, w, h), rad))
        lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, v1.rect.w, v1.rect.h), 256, 256)
        v2 = O.view_compose(v1, lrect)
        x = O.preproc(img, v2, 256, 256, -1.0, 1.0)
        lm, flag, tg = net.run(x[None], as_f64=True)
        codes.append(to_codes(x, -1.0, 1.0))
        lms.append(lm.reshape(478, 3).astype(np.float32))
        flags.append(np.float32(flag.reshape(-1)[0]))
        tongue.append(np.float32(tg.reshape(-1)[0]))
        degs.append(deg)
        d = lms[-1][263, :2] - lms[-1][33, :2]
        print("sad_linus V2", deg, "flag", O.sigmoid(flags[-1]),
              "angle", math.degrees(O.signed_angle_to((float(d[0]), float(d[1])), (1.0, 0.0))))
    out["v2_linus/codes"] = np.stack(codes)
    out["v2_linus/landmarks"] = np.stack(lms)
    out["v2_linus/flag_logit"] = np.array(flags, np.float32)
    out["v2_linus/tongue_out"] = np.array(tongue, np.float32)
    out["v2_linus/view_deg"] = np.array(degs, np.float32)
    np.savez_compressed(os.path.join(GOLD, "next_models.npz"), **out)


def main():
    if sys.argv[1:] == ["next"]:
        next_models()
        return
    if sys.argv[1:] == ["ties"]:
        nms_ties()
        return
    os.makedirs(GOLD, exist_ok=True)
    with open(os.path.join(GOLD, "reference_kat.json"), "w") as f:
        json.dump(reference_kat(), f, indent=1)
    dets = sad_linus_face()
    print("sad_linus face:", [(d.conf, math.degrees(d.angle)) for d in dets])
    sad_linus_mesh()
    models_f64()
    decode_cases()
    nms_ties()
    next_models()


if __name__ == "__main__":
    main()
