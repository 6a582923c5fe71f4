"""Decode one DRI-less stream with ZARU_JPEG_SYNC_DUMP set (the decoder writes the first sync
frame's per-segment states) -- diagnostics for the self-synchronising decoder."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from zaru_amd.jpeg import JpegDecoder  # noqa: E402
import io  # noqa: E402
from PIL import Image  # noqa: E402

img = np.random.default_rng(14).integers(0, 256, size=(600, 800, 3), dtype=np.uint8)
b = io.BytesIO()
Image.fromarray(img).save(b, "JPEG", quality=100, subsampling=0)
d = JpegDecoder(0)
d.decode(b.getvalue())
print(d.status())
