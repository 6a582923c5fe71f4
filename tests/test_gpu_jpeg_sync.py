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
    # ~591 bits per block (q99, 80 % noise): just under the gate, the densest scan the device takes
    (lambda: dense(600, 800, 14), {"quality": 99, "subsampling": 0}, True),
]


def dense(h, w, seed):
    yy, xx = np.mgrid[0:h, 0:w]
    sm = np.stack([128 + 100 * np.sin(xx / 37.0), 128 + 100 * np.cos(yy / 23.0), 128 + 80 * np.sin((xx + yy) / 51.0)], -1)
    return np.clip(0.8 * noise(h, w, seed).astype(float) + 0.2 * sm, 0, 255).astype(np.uint8)


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


def _run_with_env(code, env):
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, repo], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


@pytest.mark.parametrize("passes", [0, 1])
def test_sync_passes_that_run_out_finish_serially(passes):
    """a valid scan whose sync passes end with lanes still out of step is finished by
    the serial kernel from the last in-step lane's exit -- byte-equal, not flagged, no zero fill.
    ZARU_JPEG_SYNC_PASSES caps the passes so that these frames (and the dense one just under the
    600 bits/block gate, where out-of-step chains are longest) really take that path."""
    code = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from test_gpu_jpeg import encode, synthetic, libjpeg_turbo_rgba
from test_gpu_jpeg_sync import dense
from zaru_amd.jpeg import JpegDecoder
d = JpegDecoder(0)
for data in (encode(synthetic(360, 480, 5), quality=90), encode(dense(240, 320, 3), quality=99, subsampling=0)):
    got = d.decode(data)
    assert np.array_equal(got, libjpeg_turbo_rgba(data))
    assert not any(d.frame_errors()), list(d.frame_errors())
print("ok", d.status())
"""
    out = _run_with_env(code, {"ZARU_JPEG_SYNC_PASSES": str(passes)})
    assert out.startswith("ok (2, 0, 0)"), out


def _blocks(img):
    h, w = img.shape[0] // 8 * 8, img.shape[1] // 8 * 8
    return img[:h, :w, 0].reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)


def check_bad_block_rule(clean, bad):
    """Grayscale frames: every 8x8 block of the corrupt decode equals the clean decode or is flat
    mid-grey (an all-zero coefficient block), the changed blocks are all flat -- the block holding
    the bad code included, with no partial decode kept -- and some block changed."""
    c, b = _blocks(clean), _blocks(bad)
    same = (c == b).all(1)
    flat = (b == 128).all(1)
    assert (~same).any()
    assert (same | flat).all(), np.flatnonzero(~(same | flat))[:8]
    assert not (flat & (c == 128).all(1)).any()  # noise: no clean block is flat by chance


def test_sync_corrupt_gray_zeroes_the_bad_block():
    from zaru_amd.jpeg import JpegDecoder
    data = encode(noise(240, 320, 23, gray=True), quality=90)
    bad = bytearray(data)
    k = _scan_start(data)
    mid = k + (len(data) - k) // 2
    while data[mid - 1] == 0xFF:
        mid += 1
    bad[mid:mid + 16] = b"\xff\x00" * 8
    d = JpegDecoder(0)
    try:
        got = d.decode(bytes(bad))
        assert list(d.frame_errors()) == [True]
        check_bad_block_rule(libjpeg_turbo_rgba(data), got)
        assert (_blocks(got)[-1] == 128).all()  # zero to the end of the frame
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
