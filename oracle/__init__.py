"""CPU oracle for the Zaru detection/landmark hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
package, and only as the checker or the timed CPU baseline.  The product (``zaru_amd``)
never imports it and has no CPU fallback.

It wraps ``oracle/build/liboracle.so`` (built by ``oracle/Makefile``):
  * f32-exact restatement of preprocessing, SSD decode, NMS and landmark mapping
    (see ``oracle/geom.c`` for the reference file:line of every function);
  * a naive ONNX interpreter in f64 / f32 standing in for ONNX Runtime 1.14.8 / tract 0.20.7
    (parity of network outputs is tolerance-based: SURVEY.md §8a (iii)).
Pinning: the restatement is checked against the reference's own known-answer tests
(tests/golden/reference_kat.json) and the reference's qualitative model tests on its own
images (tests/golden/sad_linus_*.npz); see tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class Rect(C.Structure):
    _fields_ = [("cx", C.c_float), ("cy", C.c_float), ("w", C.c_float), ("h", C.c_float)]

    @staticmethod
    def from_top_left(x, y, w, h):
        return _lib().zo_rect_from_top_left(x, y, w, h)

    @staticmethod
    def from_center(x, y, w, h):
        return Rect(x, y, w, h)

    def tuple(self):
        return (self.cx, self.cy, self.w, self.h)

    def top_left(self):
        out = (C.c_float * 2)()
        _lib().zo_rect_top_left(C.byref(self), out)
        return (out[0], out[1])


class RRect(C.Structure):
    _fields_ = [("rect", Rect), ("rad", C.c_float)]


MAX_KP = 8


class Det(C.Structure):
    _fields_ = [
        ("conf", C.c_float),
        ("angle", C.c_float),
        ("rect", Rect),
        ("nkp", C.c_int32),
        ("anchor", C.c_int32),
        ("kp", (C.c_float * 2) * MAX_KP),
    ]

    def as_dict(self):
        return {
            "conf": self.conf,
            "angle": self.angle,
            "rect": self.rect.tuple(),
            "anchor": self.anchor,
            "kp": [(self.kp[k][0], self.kp[k][1]) for k in range(self.nkp)],
        }


_LIB = None


def _lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    f, u32, sz, P = C.c_float, C.c_uint32, C.c_size_t, C.c_void_p
    L.zo_rect_from_top_left.restype = Rect
    L.zo_rect_from_top_left.argtypes = [f, f, f, f]
    L.zo_rect_grow_rel.restype = Rect
    L.zo_rect_grow_rel.argtypes = [Rect, f]
    L.zo_rect_grow_to_fit_aspect.restype = Rect
    L.zo_rect_grow_to_fit_aspect.argtypes = [Rect, u32, u32]
    L.zo_rect_intersection.argtypes = [C.POINTER(Rect), C.POINTER(Rect), C.POINTER(Rect)]
    L.zo_rect_iou.restype = f
    L.zo_rect_iou.argtypes = [C.POINTER(Rect), C.POINTER(Rect)]
    L.zo_rect_top_left.argtypes = [C.POINTER(Rect), P]
    L.zo_rrect_transform_out.argtypes = [C.POINTER(RRect), f, f, P]
    L.zo_rrect_transform_in.argtypes = [C.POINTER(RRect), f, f, P]
    L.zo_rrect_bounding.argtypes = [f, P, sz, sz, C.POINTER(RRect)]
    L.zo_signed_angle_to.restype = f
    L.zo_signed_angle_to.argtypes = [f, f, f, f]
    L.zo_sigmoid.restype = f
    L.zo_sigmoid.argtypes = [f]
    L.zo_view_full.restype = RRect
    L.zo_view_full.argtypes = [u32, u32]
    L.zo_view_compose.restype = RRect
    L.zo_view_compose.argtypes = [C.POINTER(RRect), C.POINTER(RRect)]
    L.zo_view_get.restype = u32
    L.zo_view_get.argtypes = [P, u32, u32, sz, C.POINTER(RRect), u32, u32]
    L.zo_preproc.argtypes = [P, u32, u32, sz, C.POINTER(RRect), u32, u32, f, f, P]
    L.zo_anchors.restype = sz
    L.zo_anchors.argtypes = [P, sz, P]
    L.zo_extract.restype = sz
    L.zo_extract.argtypes = [C.c_int, P, P, sz, P, u32, u32, f, P, sz]
    L.zo_nms.restype = sz
    L.zo_nms.argtypes = [P, sz, f, C.c_int, P]
    L.zo_detector_map.argtypes = [P, sz, C.POINTER(Rect), u32]
    L.zo_detect_post.restype = sz
    L.zo_detect_post.argtypes = [C.c_int, P, P, sz, u32, u32, u32, u32, f, f, P, sz]
    L.zo_detect_post_mode.restype = sz
    L.zo_detect_post_mode.argtypes = [C.c_int, P, P, sz, u32, u32, u32, u32, f, f, C.c_int, P, sz]
    L.zo_estimator_map.argtypes = [P, sz, C.POINTER(Rect), u32]
    L.zo_tracker_update.restype = C.c_int
    L.zo_tracker_update.argtypes = [P, sz, C.POINTER(RRect), f, f, f, C.POINTER(RRect),
                                    C.POINTER(RRect)]
    L.zo_landmark_angle.restype = f
    L.zo_landmark_angle.argtypes = [C.c_int, P]
    L.zo_net_load.restype = P
    L.zo_net_load.argtypes = [P, sz, C.c_int]
    L.zo_net_num_outputs.restype = sz
    L.zo_net_num_outputs.argtypes = [P]
    L.zo_net_output_shape.restype = sz
    L.zo_net_output_shape.argtypes = [P, sz, P]
    L.zo_net_run.restype = C.c_int
    L.zo_net_run.argtypes = [P, P, P]
    L.zo_net_run_f64out.restype = C.c_int
    L.zo_net_run_f64out.argtypes = [P, P, P]
    L.zo_net_error.restype = C.c_char_p
    L.zo_net_tensor.restype = sz
    L.zo_jpeg_pixels.restype = C.c_int
    L.zo_jpeg_pixels.argtypes = [P, u32, u32, u32, u32, u32, P, P, P, P, P]
    L.zo_net_tensor.argtypes = [P, C.c_char_p, P, sz, P, P]
    _LIB = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------- geometry helpers
def rect_from_top_left(x, y, w, h) -> Rect:
    return _lib().zo_rect_from_top_left(x, y, w, h)


def grow_rel(r: Rect, amount: float) -> Rect:
    return _lib().zo_rect_grow_rel(r, amount)


def grow_to_fit_aspect(r: Rect, aw: int, ah: int) -> Rect:
    return _lib().zo_rect_grow_to_fit_aspect(r, aw, ah)


def iou(a: Rect, b: Rect) -> float:
    return _lib().zo_rect_iou(C.byref(a), C.byref(b))


def intersection(a: Rect, b: Rect):
    out = Rect()
    ok = _lib().zo_rect_intersection(C.byref(a), C.byref(b), C.byref(out))
    return out if ok else None


def transform_out(r: RRect, x, y):
    o = (C.c_float * 2)()
    _lib().zo_rrect_transform_out(C.byref(r), x, y, o)
    return (o[0], o[1])


def transform_in(r: RRect, x, y):
    o = (C.c_float * 2)()
    _lib().zo_rrect_transform_in(C.byref(r), x, y, o)
    return (o[0], o[1])


def rrect_bounding(rad, pts):
    a = np.ascontiguousarray(np.asarray(pts, dtype=np.float32).reshape(-1, 2))
    out = RRect()
    ok = _lib().zo_rrect_bounding(rad, _ptr(a), a.shape[0], 2, C.byref(out))
    return out if ok else None


def sigmoid(v: float) -> float:
    return _lib().zo_sigmoid(v)


def signed_angle_to(a, b) -> float:
    return _lib().zo_signed_angle_to(a[0], a[1], b[0], b[1])


# ---------------------------------------------------------------- views / preproc
def view_full(w: int, h: int) -> RRect:
    return _lib().zo_view_full(w, h)


def view_compose(parent: RRect, child) -> RRect:
    if isinstance(child, Rect):
        child = RRect(child, 0.0)
    return _lib().zo_view_compose(C.byref(parent), C.byref(child))


def view_get(img: np.ndarray, view: RRect, x: int, y: int) -> int:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    return _lib().zo_view_get(_ptr(img), w, h, w * 4, C.byref(view), x, y)


def preproc(img: np.ndarray, view: RRect, ow: int, oh: int, lo: float, hi: float) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    out = np.empty((3, oh, ow), np.float32)
    _lib().zo_preproc(_ptr(img), w, h, w * 4, C.byref(view), ow, oh, lo, hi, _ptr(out))
    return out


# ---------------------------------------------------------------- decode / NMS
FACE, PALM, FACE_FULL = 0, 1, 2
FACE_LAYERS = [(2, 16, 16), (6, 8, 8)]        # face/detection.rs:53
PALM_LAYERS = [(2, 24, 24), (6, 12, 12)]      # hand/detection.rs:117
FACE_FULL_LAYERS = [(1, 48, 48)]              # face/detection.rs:86-88
LAYERS = {FACE: FACE_LAYERS, PALM: PALM_LAYERS, FACE_FULL: FACE_FULL_LAYERS}


def anchors(layers) -> np.ndarray:
    arr = np.asarray(layers, dtype=np.uint32).reshape(-1)
    n = _lib().zo_anchors(_ptr(arr), len(layers), None)
    out = np.empty((n, 2), np.float32)
    _lib().zo_anchors(_ptr(arr), len(layers), _ptr(out))
    return out


def extract(kind, boxes, confs, in_w, in_h, thresh=0.5):
    an = anchors(LAYERS[kind])
    boxes = np.ascontiguousarray(boxes, np.float32)
    confs = np.ascontiguousarray(confs, np.float32).reshape(-1)
    out = (Det * len(an))()
    n = _lib().zo_extract(kind, _ptr(boxes), _ptr(confs), len(an), _ptr(an), in_w, in_h,
                          thresh, out, len(an))
    return [out[i] for i in range(n)]


def nms(dets, iou_thresh=0.3, mode=1):
    arr = (Det * max(1, len(dets)))(*dets)
    out = (Det * max(1, len(dets)))()
    n = _lib().zo_nms(arr, len(dets), iou_thresh, mode, out)
    return [out[i] for i in range(n)]


def detect_post(kind, boxes, confs, img_w, img_h, in_w, in_h, thresh=0.5, iou_thresh=0.3, remove=False):
    """remove: SuppressionMode::Remove (nms.rs:70-76) instead of the default Average."""
    boxes = np.ascontiguousarray(boxes, np.float32)
    confs = np.ascontiguousarray(confs, np.float32).reshape(-1)
    na = confs.shape[0]
    out = (Det * na)()
    n = _lib().zo_detect_post_mode(kind, _ptr(boxes), _ptr(confs), na, img_w, img_h, in_w, in_h,
                                   thresh, iou_thresh, 0 if remove else 1, out, na)
    return [out[i] for i in range(n)]


def estimator_map(pos: np.ndarray, view_local_rect: Rect, in_w: int) -> np.ndarray:
    p = np.ascontiguousarray(pos, np.float32).copy()
    _lib().zo_estimator_map(_ptr(p), p.shape[0], C.byref(view_local_rect), in_w)
    return p


def tracker_update(pos, view_rect: RRect, roi_rad, est_angle, padding):
    p = np.ascontiguousarray(pos, np.float32).copy()
    upd, nxt = RRect(), RRect()
    _lib().zo_tracker_update(_ptr(p), p.shape[0], C.byref(view_rect), roi_rad, est_angle,
                             padding, C.byref(upd), C.byref(nxt))
    return p, upd, nxt


FACEMESH, HAND, FACEMESH_V2 = 0, 1, 2


def landmark_angle(kind, pos) -> float:
    """Estimate::angle_radians of view-local landmarks (FACEMESH: mediapipe.rs:146-160,
    HAND: hand/landmark.rs:68-78)."""
    p = np.ascontiguousarray(pos, np.float32)
    # FaceMesh V2 uses V1's eye-corner indices (mediapipe.rs:407-421)
    return _lib().zo_landmark_angle(HAND if kind == HAND else FACEMESH, _ptr(p))


def landmark_confidence(kind, outs) -> float:
    """Confidence::confidence of the raw landmark-network outputs: FaceMesh face_flag =
    sigmoid(out1) (mediapipe.rs:60), hand presence = out1 (sigmoid inside the graph,
    hand/landmark.rs:309)."""
    v = float(np.asarray(outs[1], np.float32).reshape(-1)[0])
    return v if kind == HAND else sigmoid(v)  # V2: face_flag as V1 (mediapipe.rs:100)


# ---------------------------------------------------------------- networks
class Net:
    """Naive ONNX interpreter (batch 1); ``f64=True`` evaluates in double precision."""

    def __init__(self, onnx_path: str, f64: bool = True):
        self._bytes = open(onnx_path, "rb").read()
        buf = C.create_string_buffer(self._bytes, len(self._bytes))
        self._buf = buf
        self.f64 = f64
        self._h = _lib().zo_net_load(buf, len(self._bytes), 1 if f64 else 0)
        if not self._h:
            raise RuntimeError(_lib().zo_net_error().decode())
        self.shapes = None

    def run(self, x: np.ndarray, as_f64: bool = False):
        x = np.ascontiguousarray(x, np.float32)
        n_out = _lib().zo_net_num_outputs(self._h)
        if self.shapes is None:  # first run discovers output shapes
            ptrs = (C.c_void_p * n_out)()
            if _lib().zo_net_run(self._h, _ptr(x), ptrs):
                raise RuntimeError(_lib().zo_net_error().decode())
            shapes = []
            for i in range(n_out):
                s = np.zeros(6, np.int64)
                r = _lib().zo_net_output_shape(self._h, i, _ptr(s))
                shapes.append(tuple(int(v) for v in s[:r]))
            self.shapes = shapes
        dt = np.float64 if (as_f64 and self.f64) else np.float32
        outs = [np.empty(s, dt) for s in self.shapes]
        ptrs = (C.c_void_p * n_out)(*[o.ctypes.data for o in outs])
        fn = _lib().zo_net_run_f64out if dt == np.float64 else _lib().zo_net_run
        if fn(self._h, _ptr(x), ptrs):
            raise RuntimeError(_lib().zo_net_error().decode())
        return outs

    def tensor(self, name: str) -> np.ndarray:
        """Any intermediate tensor of the last run (f64 nets; layer bisection)."""
        shape = np.zeros(6, np.int64)
        rank = C.c_size_t(0)
        n = _lib().zo_net_tensor(self._h, name.encode(), None, 0, _ptr(shape), C.byref(rank))
        if not n:
            raise KeyError(name)
        out = np.empty(n, np.float64)
        _lib().zo_net_tensor(self._h, name.encode(), _ptr(out), n, None, None)
        return out.reshape(tuple(int(v) for v in shape[:rank.value]))


# ---------------------------------------------------------------- JPEG (libjpeg-turbo pixels)
def jpeg_pixels(coef: np.ndarray, layout: dict) -> np.ndarray:
    """libjpeg-turbo's islow IDCT + fancy upsampling + YCbCr->RGBA (oracle/jpeg.c) over the
    quantised coefficients of one frame (zaru_amd.jpeg.coefficients)."""
    coef = np.ascontiguousarray(coef, np.int16)
    bw = np.ascontiguousarray(layout["bw"], np.uint32)
    bh = np.ascontiguousarray(layout["bh"], np.uint32)
    qs = np.ascontiguousarray(layout["qsel"], np.uint32)
    q = np.ascontiguousarray(layout["quant"], np.uint16)
    out = np.empty((layout["height"], layout["width"], 4), np.uint8)
    if _lib().zo_jpeg_pixels(_ptr(coef), layout["width"], layout["height"], layout["ncomp"],
                             layout["h_samp"], layout["v_samp"], _ptr(bw), _ptr(bh), _ptr(qs),
                             _ptr(q), _ptr(out)):
        raise MemoryError("zo_jpeg_pixels")
    return out
