"""Per-kernel cost of the device Huffman stage vs the restart interval: one decoder, one stream,
sequential decodes of the same 1080p frame encoded with several restart intervals.  Run under
rocprofv3 --kernel-trace --stats (or --pmc) to split the kernels."""
import io, sys, time
import numpy as np
from PIL import Image
sys.path.insert(0, '.')
import torch
from zaru_amd.jpeg import JpegDecoder

rng = np.random.default_rng(0)
yy, xx = np.mgrid[0:1080, 0:1920]
img = np.stack([(xx * 255 // 1919), (yy * 255 // 1079), ((xx + yy) % 256)], -1).astype(np.uint8)
img = np.clip(img.astype(np.int16) + rng.integers(-20, 21, img.shape), 0, 255).astype(np.uint8)
d = JpegDecoder(0)
out = torch.empty((1080, 1920 * 4), dtype=torch.uint8, device='cuda')
for blocks in [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else '1,4,16,64').split(',')]:
    b = io.BytesIO()
    Image.fromarray(img).save(b, 'JPEG', quality=90, restart_marker_blocks=blocks)
    data = b.getvalue()
    for _ in range(2):
        d.decode_into(data, out.data_ptr(), 1920 * 4)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 10
    for _ in range(n):
        d.decode_into(data, out.data_ptr(), 1920 * 4)
    torch.cuda.synchronize()
    print(f'restart {blocks} MCUs: {len(data)} B, {1e3 * (time.perf_counter() - t) / n:.3f} ms/frame, status {d.status()}', flush=True)
