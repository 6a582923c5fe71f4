"""Decode DRI-less JPEG frames through the self-synchronising device path and report: status,
frame error flags, byte differences to libjpeg-turbo (first differing pixel, its MCU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_jpeg import encode, libjpeg_turbo_rgba, synthetic  # noqa: E402
from zaru_amd.jpeg import JpegDecoder  # noqa: E402

def noise(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


cases = [((600, 800), 100, 0, 14, noise), ((600, 800), 95, 0, 14, noise), ((600, 800), 90, 2, 14, noise),
         ((200, 200), 100, 0, 14, noise), ((64, 64), 100, 0, 14, noise)]
for (h, w), q, sub, seed, gen in cases:
    data = encode(gen(h, w, seed), quality=q, subsampling=sub)
    d = JpegDecoder(0)
    got = d.decode(data)
    want = libjpeg_turbo_rgba(data)
    diff = np.abs(got.astype(int) - want.astype(int)).max(-1)
    ys, xs = np.nonzero(diff)
    first = (int(ys[0]), int(xs[0])) if len(ys) else None
    mcu_w = 16 if sub in (1, 2) else 8
    mcu_h = 16 if sub == 2 else 8
    mcu = None if first is None else (first[0] // mcu_h) * ((w + mcu_w - 1) // mcu_w) + first[1] // mcu_w
    print((h, w), q, sub, "bytes", len(data), "segments", len(data) * 8 // 4096, "status", d.status(),
          "errors", list(d.frame_errors()), "ndiff_px", int((diff > 0).sum()), "first", first, "mcu", mcu, flush=True)
    if first is not None:
        band = [round(float((diff[r:r + mcu_h] > 0).mean()), 2) for r in range(0, h, mcu_h)]
        print("  per MCU row fraction differing:", band[:40], "...", band[-5:], flush=True)
        row0 = (diff[:mcu_h] > 0).any(0)
        print("  first MCU row: differing MCU columns", [int(x) for x in np.nonzero(row0.reshape(-1, mcu_w).any(1))[0][:30]])
        gray = (got[..., :3] == 128).all(-1)
        print("  mid-grey px", int(gray.sum()), flush=True)
    d.close()
