"""Synthetic inputs of BASELINE.json's configs, shared by the tests.

C1: one 640x480 RGBA8 frame, uniform noise from seed 1 with the reference's own FaceMesh
    test face (tests/golden/sad_linus_mesh.npz codes, 192x192) pasted at (224, 144), so the
    BlazeFace letterbox (640x640 -> 128) sees a ~38 px face as in face/detection.rs:164-173.
C2: batch 64 of [3,128,128] BlazeFace input tensors, values k*(2/255) - 1 with
    k ~ U{0..255} from numpy's PCG64 seeded 0x5A52550000000002.
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
C2_SEED = 0x5A52550000000002


def face_patch():
    codes = np.load(os.path.join(GOLDEN, "sad_linus_mesh.npz"))["codes"][0]
    img = np.full((192, 192, 4), 255, np.uint8)
    img[..., :3] = codes.transpose(1, 2, 0)
    return img


def c1_frame():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(480, 640, 4), dtype=np.uint8)
    img[144:336, 224:416] = face_patch()
    return img


def c2_batch():
    rng = np.random.default_rng(C2_SEED)
    k = rng.integers(0, 256, size=(64, 3, 128, 128), dtype=np.uint8)
    adj = np.float32(np.float32(2.0) / np.float32(255.0))
    return k.astype(np.float32) * adj + np.float32(-1.0)
