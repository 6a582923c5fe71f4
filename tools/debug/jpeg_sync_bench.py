"""Batches of 16 DRI-less 1080p frames through the self-synchronising device decoder (one
decoder, one stream), for rocprofv3 kernel timings of the sync passes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_jpeg import encode, synthetic  # noqa: E402
from zaru_amd._lib import DeviceBuffer, lib  # noqa: E402
from zaru_amd.jpeg import JpegDecoder  # noqa: E402

datas = [encode(synthetic(1080, 1920, 40 + i), quality=90) for i in range(16)]
bufs = [DeviceBuffer(1080 * 1920 * 4) for _ in datas]
d = JpegDecoder(0)
for it in range(6):
    t0 = time.perf_counter()
    d.decode_batch_into(datas, [b.ptr for b in bufs], [1920 * 4] * 16)
    lib().zr_stream_synchronize(None)
    print(it, "ms per 16-frame call", round((time.perf_counter() - t0) * 1e3, 2), d.status(), flush=True)
