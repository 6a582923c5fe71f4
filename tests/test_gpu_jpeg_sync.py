"""JPEG streams WITHOUT restart markers decoded on the device by the
self-synchronising Huffman decoder (kernels/jpeg_sync.hip, zr_jpeg.h): a lane per 4096-bit
segment of the scan, sync passes, a prefix over the lanes, a write pass.  The bar is the same as
for the other paths: RGBA byte-equal to libjpeg-turbo (Pillow), and the decoder status shows the
frames took the device path with no frame flagged.  Inputs: synthetic frames encoded by Pillow
(no DRI), from one segment to a few thousand, 4:2:0 / 4:2:2 / 4:4:4 / grayscale."""
import numpy as np
import pytest

from test_gpu_jpeg import encode, libjpeg_turbo_rgba, synthetic

pytestmark = pytest.mark.gpu


def noise(h, w, seed, gray=False):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(h, w) if gray else (h, w, 3), dtype=np.uint8)


CASES = [
    # (image, encode options, device path): scans from < 1 segment to ~4000 segments
    (lambda: synthetic(1080, 1920, 11), {"quality": 90, "subsampling": 2}, True),
    (lambda: synthetic(1080, 1920, 12), {"quality": 75, "subsampling": 0}, True),
    (lambda: synthetic(720, 1280, 13), {"quality": 95, "subsampling": 1}, True),
    (lambda: synthetic(1080, 1920, 4), {"quality": 95, "subsampling": 1}, True),
    (lambda: noise(600, 800, 14), {"quality": 95, "subsampling": 0}, True),
    (lambda: noise(300, 300, 15), {"quality": 95, "subsampling": 2}, True),
    (lambda: synthetic(61, 97, 16), {"quality": 75, "subsampling": 2}, True),
    (lambda: synthetic(16, 16, 17), {"quality": 50, "subsampling": 2}, True),
    (lambda: synthetic(33, 17, 18), {"quality": 95, "subsampling": 1}, True),
    (lambda: noise(480, 640, 19, gray=True), {"quality": 90}, True),
    (lambda: synthetic(500, 700, 20)[..., 1], {"quality": 85}, True),
    # ~700 bits per block (q100 noise): over JS_MAX_BITS_PER_BLOCK, the host decodes it
    (lambda: noise(600, 800, 14), {"quality": 100, "subsampling": 0}, False),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sync_decode_equals_libjpeg_turbo(case):
    from zaru_amd.jpeg import JpegDecoder
    make, kw, device = CASES[case]
    data = encode(make(), **kw)
    d = JpegDecoder(0)
    try:
        got = d.decode(data)
        want = libjpeg_turbo_rgba(data)
        assert got.shape == want.shape
        diff = np.abs(got.astype(int) - want.astype(int))
        assert diff.max() == 0, (case, int(diff.max()), int((diff > 0).sum()))
        assert d.status() == ((1, 0, 0) if device else (0, 1, 0)), d.status()
    finally:
        d.close()


def test_sync_batch_of_frames():
    """16 1080p frames without DRI in one zr_jpeg_decode_batch_async call (the bench's jpeg
    line shape): one set of sync launches for all of them, every frame byte-equal."""
    from zaru_amd._lib import DeviceBuffer, lib
    from zaru_amd.jpeg import JpegDecoder
    datas = [encode(synthetic(1080, 1920, 40 + i), quality=90) for i in range(16)]
    bufs = [DeviceBuffer(1080 * 1920 * 4) for _ in datas]
    d = JpegDecoder(0)
    try:
        d.decode_batch_into(datas, [b.ptr for b in bufs], [1920 * 4] * len(datas))
        lib().zr_stream_synchronize(None)
        for i, data in enumerate(datas):
            assert np.array_equal(bufs[i].download((1080, 1920, 4), "uint8"), libjpeg_turbo_rgba(data)), i
        assert d.status() == (16, 0, 0)
        assert not any(d.frame_errors())
    finally:
        d.close()


def _scan_start(data):
    i = data.index(b"\xff\xda")
    return i + 2 + int.from_bytes(data[i + 2:i + 4], "big")


def test_sync_corrupt_scan_is_flagged_and_zero_filled():
    """An invalid Huffman code in the middle of a DRI-less scan: the frame is flagged and every
    block from the bad one on is zero (libjpeg's rule after corrupt data), so the bottom MCU rows
    decode to mid-grey; nothing is read or written out of bounds."""
    from zaru_amd.jpeg import JpegDecoder
    data = bytearray(encode(synthetic(480, 640, 21), quality=90))
    k = _scan_start(data)
    mid = k + (len(data) - k) // 3
    while data[mid - 1] == 0xFF:
        mid += 1
    data[mid:mid + 16] = b"\xff\x00" * 8  # stuffed 0xFF pairs: 64 one bits, longer than any code
    d = JpegDecoder(0)
    try:
        got = d.decode(bytes(data))
        assert d.status()[2] == 1
        assert list(d.frame_errors()) == [True]
        assert (got[-16:, :, :3] == 128).all()
    finally:
        d.close()


def test_sync_switch_off_keeps_host_path():
    """ZARU_JPEG_SYNC=0 sends DRI-less streams back to the host decoder (A/B): same bytes."""
    import os
    import subprocess
    import sys
    code = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from test_gpu_jpeg import encode, synthetic, libjpeg_turbo_rgba
from zaru_amd.jpeg import JpegDecoder
data = encode(synthetic(360, 480, 5), quality=90)
d = JpegDecoder(0)
assert np.array_equal(d.decode(data), libjpeg_turbo_rgba(data))
assert d.status() == (0, 1, 0), d.status()
print("ok")
"""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, repo], env=dict(os.environ, ZARU_JPEG_SYNC="0"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
