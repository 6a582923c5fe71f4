"""the JPEG frame source (zaru_amd.jpeg over zr_jpeg_decode_async) against
libjpeg-turbo, the library behind the reference's `ZARU_JPEG_BACKEND=libjpeg-turbo` decoder
(crates/zaru-image/src/jpeg.rs:164-182: turbojpeg 0.5.3, default flags = accurate integer IDCT
and fancy upsampling, RGBA output with alpha 255).  Pillow in this image links libjpeg-turbo
and decodes with the same defaults, so it is the reference run here; the bar is byte equality.

The default backend, zune-jpeg 0.3.17 (jpeg.rs:183-205), is not installed anywhere in this
image, so parity with it is unpinned (it differs from libjpeg-turbo by +-1 in places).

Inputs are synthetic (seeded noise, gradients, a face crop of the reference's own test image),
encoded by Pillow at several sizes, qualities, chroma subsamplings and restart intervals.
Streams with restart intervals take the device Huffman path (kernels/jpeg_huff.hip); the bar
is the same byte equality.
"""
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def synthetic(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([(x * 255 // max(1, w - 1)), (y * 255 // max(1, h - 1)), ((x + y) * 7) % 256], -1)
    img = (img + rng.integers(-40, 41, size=img.shape)).clip(0, 255).astype(np.uint8)
    codes = np.load(os.path.join(REPO, "tests", "golden", "sad_linus_mesh.npz"))["codes"][0]
    ph, pw = min(192, h), min(192, w)
    img[:ph, :pw] = codes.transpose(1, 2, 0)[:ph, :pw]
    return img


def encode(img, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", **kw)
    return b.getvalue()


def libjpeg_turbo_rgba(data):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"))


@pytest.fixture(scope="module")
def dec():
    from zaru_amd.jpeg import JpegDecoder
    d = JpegDecoder(0)
    yield d
    d.close()


CASES = [
    # (h, w, quality, subsampling 0=4:4:4 1=4:2:2 2=4:2:0, extra save options)
    (1080, 1920, 90, 2, {}),
    (61, 97, 75, 2, {}),
    (33, 17, 95, 2, {}),
    (64, 64, 50, 0, {}),
    (45, 131, 85, 1, {}),
    (120, 160, 75, 2, {"restart_marker_blocks": 3}),
    (97, 203, 100, 0, {"restart_marker_rows": 1}),
    # restart intervals: the Huffman stage runs on the device, one lane per interval
    (1080, 1920, 90, 2, {"restart_marker_blocks": 1}),
    (1080, 1920, 90, 2, {"restart_marker_blocks": 4}),
    (1080, 1920, 75, 0, {"restart_marker_blocks": 7}),
    (720, 1280, 95, 1, {"restart_marker_blocks": 2}),
    # long intervals (one MCU row each: 68 lanes per frame)
    (1080, 1920, 90, 2, {"restart_marker_rows": 1}),
    (720, 1280, 95, 1, {"restart_marker_rows": 2}),
]


@pytest.mark.parametrize("h,w,q,sub,kw", CASES)
def test_decode_equals_libjpeg_turbo(dec, h, w, q, sub, kw):
    data = encode(synthetic(h, w, h * 1000 + w), quality=q, subsampling=sub, **kw)
    got = dec.decode(data)
    want = libjpeg_turbo_rgba(data)
    assert got.shape == want.shape == (h, w, 4)
    diff = np.abs(got.astype(int) - want.astype(int))
    assert diff.max() == 0, (h, w, q, sub, int(diff.max()), int((diff > 0).sum()))


def test_grayscale(dec):
    g = synthetic(70, 90, 5)[..., 0]
    data = encode(g, quality=80)
    assert np.array_equal(dec.decode(data), libjpeg_turbo_rgba(data))


def test_decoder_reuse_across_sizes(dec):
    """One decoder, shrinking and growing frames: staging reuse never leaks the previous frame."""
    for i, (h, w) in enumerate([(480, 640), (64, 48), (720, 1280), (480, 640)]):
        data = encode(synthetic(h, w, 77 + i), quality=85)
        assert np.array_equal(dec.decode(data), libjpeg_turbo_rgba(data))


def test_one_decoder_alternating_streams(dec):
    """One decoder, consecutive frames enqueued on two different streams without a host wait
    between them (INTEGRATION.md §8's per-frame stream pool): the second frame's coefficient
    upload must not overwrite buffers the first frame's kernels are still reading."""
    import ctypes as C

    from zaru_amd._lib import DeviceBuffer, check, lib
    frames = [synthetic(1080, 1920, 900 + i) for i in range(6)]
    datas = [encode(f, quality=90) for f in frames]
    streams = []
    for _ in range(2):
        sp = C.c_void_p()
        check(lib().zr_stream_create(C.byref(sp)))
        streams.append(sp.value)
    bufs = [DeviceBuffer(1080 * 1920 * 4) for _ in datas]
    try:
        for i, d in enumerate(datas):
            dec.decode_into(d, bufs[i].ptr, 1920 * 4, streams[i % 2])
        for s in streams:
            check(lib().zr_stream_synchronize(s))
        for i, d in enumerate(datas):
            got = bufs[i].download((1080, 1920, 4), "uint8")
            assert np.array_equal(got, libjpeg_turbo_rgba(d)), i
    finally:
        for s in streams:
            lib().zr_stream_destroy(s)


def test_decoded_frames_feed_the_pipeline(dec):
    """Frames decoded into HBM by the JPEG source run the config-3 pipeline exactly as frames
    uploaded from libjpeg-turbo's host decode (same bytes -> same detections and landmarks)."""
    import zaru_amd.host as H
    from zaru_amd._lib import DeviceBuffer
    imgs = [synthetic(360, 640, 900 + i) for i in range(3)]
    datas = [encode(im, quality=90) for im in imgs]
    a = DeviceBuffer(3 * 360 * 640 * 4)
    for i, d in enumerate(datas):
        dec.decode_into(d, a.ptr + i * 360 * 640 * 4, 640 * 4)
    from zaru_amd._lib import lib
    lib().zr_stream_synchronize(None)
    b = DeviceBuffer.from_array(np.stack([libjpeg_turbo_rgba(d) for d in datas]))
    forced = [[(320.0, 180.0, 200.0, 200.0, 0.0)] for _ in range(3)]
    res = []
    for buf in (a, b):
        p = H.DetectTrackPipeline("face", 0, 4, 1)
        p.run([(buf.ptr + i * 360 * 640 * 4, 640, 360, 640 * 4) for i in range(3)], forced)
        res.append([(r["frame"], r["tracked"], r["landmarks"].tobytes()) for r in (p.roi(i) for i in range(p.num_rois()))])
    assert res[0] == res[1]


@pytest.mark.parametrize("bad", [b"", b"\xff\xd8\xff\xd9", b"not a jpeg at all"])
def test_malformed_streams_are_errors(dec, bad):
    from zaru_amd._lib import ZaruError
    with pytest.raises(ZaruError):
        dec.decode(bad)


def test_truncated_scan_is_decoded_or_rejected(dec):
    """A stream cut inside the entropy-coded data: the decoder pads with zero bits (libjpeg
    warns and does the same) -- it must neither crash nor read past the buffer."""
    data = encode(synthetic(64, 64, 3), quality=90)
    cut = data[: len(data) * 2 // 3]
    from zaru_amd._lib import ZaruError
    try:
        out = dec.decode(cut)
    except ZaruError:
        return
    assert out.shape == (64, 64, 4)


def test_restart_streams_decode_on_the_device(dec):
    """Streams with >= 8 restart intervals short enough for a workgroup's LDS are entropy-decoded
    on the GPU (decoder status), with no corrupt interval flagged -- long ones (one MCU row per
    interval) too, since round 4 reads the intervals from global memory instead of staging them in
    LDS -- and so are streams without DRI (self-synchronising decoder, jpeg_sync.hip)."""
    from zaru_amd.jpeg import JpegDecoder
    d = JpegDecoder(0)
    try:
        with_rst = encode(synthetic(1080, 1920, 5), quality=90, restart_marker_blocks=4)
        long_rst = encode(synthetic(1080, 1920, 5), quality=90, restart_marker_rows=1)
        plain = encode(synthetic(1080, 1920, 5), quality=90)
        g = synthetic(200, 300, 9)[..., 0]
        gray_rst = encode(g, quality=85, restart_marker_blocks=5)
        for data in (with_rst, long_rst, plain, gray_rst):
            assert np.array_equal(d.decode(data), libjpeg_turbo_rgba(data))
        gpu, host, corrupt = d.status()
        assert (gpu, host, corrupt) == (4, 0, 0)
    finally:
        d.close()


def _scan_start(data):
    i = data.index(b"\xff\xda")
    return i + 2 + int.from_bytes(data[i + 2:i + 4], "big")


def test_restart_stream_with_fill_bytes(dec):
    """0xFF fill bytes in front of every RSTn (T.81 B.1.1.2 allows any number): the interval ends
    at the first of them, as in the host reader, and the output still equals libjpeg-turbo's."""
    from zaru_amd.jpeg import JpegDecoder
    data = encode(synthetic(480, 640, 8), quality=90, restart_marker_blocks=2)
    k = _scan_start(data)
    scan = data[k:]
    for n in range(8):
        m = bytes([0xFF, 0xD0 + n])
        scan = scan.replace(m, b"\xff\xff" + m)
    filled = data[:k] + scan
    assert len(filled) > len(data)
    d = JpegDecoder(0)
    try:
        assert np.array_equal(d.decode(filled), libjpeg_turbo_rgba(data))
        assert d.status() == (1, 0, 0)
    finally:
        d.close()


def test_restart_stream_corrupt_interval_is_flagged(dec):
    """A corrupt interval (an invalid Huffman code) is flagged by the device decoder (status
    `corrupt`), the frame still decodes without a fault, and the next good frame is clean."""
    from zaru_amd.jpeg import JpegDecoder
    data = encode(synthetic(480, 640, 8), quality=90, restart_marker_blocks=2)
    k = _scan_start(data)
    bad = bytearray(data)
    # inside the third interval, away from its markers: stuffed 0xFF pairs, i.e. a run of 64 one
    # bits -- longer than any code (T.81 C: the all-ones code is never assigned)
    r = [i for i in range(k, len(data) - 1) if data[i] == 0xFF and 0xD0 <= data[i + 1] <= 0xD7]
    p = (r[1] + r[2]) // 2
    while data[p - 1] == 0xFF:
        p += 1
    assert p + 16 < r[2]
    bad[p:p + 16] = b"\xff\x00" * 8
    d = JpegDecoder(0)
    try:
        out = d.decode(bytes(bad))
        assert out.shape == (480, 640, 4)
        assert d.status()[2] == 1
        assert list(d.frame_errors()) == [True]
        assert np.array_equal(d.decode(data), libjpeg_turbo_rgba(data))
        assert d.status()[2] == 0  # the flag is per call: the good frame after it is clean
    finally:
        d.close()


def _corrupt_third_interval(data):
    k = _scan_start(data)
    bad = bytearray(data)
    r = [i for i in range(k, len(data) - 1) if data[i] == 0xFF and 0xD0 <= data[i + 1] <= 0xD7]
    p = (r[1] + r[2]) // 2
    while data[p - 1] == 0xFF:
        p += 1
    bad[p:p + 16] = b"\xff\x00" * 8
    return bytes(bad)


def test_corrupt_interval_leaves_no_stale_coefficients(dec):
    """After a corrupt symbol the rest of the interval decodes as all-zero blocks (libjpeg-turbo's
    insufficient-data rule), never as whatever an earlier frame left in the reused coefficient
    buffer: the corrupt frame decodes the same on a decoder that just decoded another camera's
    frame as on a fresh one.  In a batch, only the corrupt frame is flagged."""
    from zaru_amd._lib import DeviceBuffer, lib
    from zaru_amd.jpeg import JpegDecoder
    other = encode(synthetic(480, 640, 31), quality=90, restart_marker_blocks=2)
    data = encode(synthetic(480, 640, 8), quality=90, restart_marker_blocks=2)
    bad = _corrupt_third_interval(data)
    fresh = JpegDecoder(0)
    used = JpegDecoder(0)
    try:
        want = fresh.decode(bad)
        used.decode(other)
        got = used.decode(bad)
        assert np.array_equal(got, want)
        # the corruption really zeroed something: not the clean decode
        assert not np.array_equal(want, libjpeg_turbo_rgba(data))
        bufs = [DeviceBuffer(480 * 640 * 4) for _ in range(3)]
        used.decode_batch_into([data, bad, other], [b.ptr for b in bufs], [640 * 4] * 3)
        lib().zr_stream_synchronize(None)
        assert list(used.frame_errors()) == [False, True, False]
        assert np.array_equal(bufs[1].download((480, 640, 4), "uint8"), want)
        assert np.array_equal(bufs[2].download((480, 640, 4), "uint8"), libjpeg_turbo_rgba(other))
    finally:
        fresh.close()
        used.close()


def test_corrupt_interval_zeroes_the_bad_block(dec):
    """the restart-interval decoder applies the sync decoder's rule -- the block holding
    the bad code is zero too, not a partial decode (grayscale noise, 2-block intervals)."""
    from test_gpu_jpeg_sync import check_bad_block_rule, noise
    data = encode(noise(240, 320, 24, gray=True), quality=90, restart_marker_blocks=8)
    bad = _corrupt_third_interval(data)
    got = dec.decode(bad)
    assert list(dec.frame_errors()) == [True]
    check_bad_block_rule(libjpeg_turbo_rgba(data), got)


def test_restart_stream_cut_mid_scan(dec):
    """A restart-interval stream cut inside the scan no longer has one RSTn per interval: it
    takes the host path, which pads with zero bits or rejects it, and never reads past the
    buffer."""
    from zaru_amd._lib import ZaruError
    data = encode(synthetic(240, 320, 4), quality=90, restart_marker_rows=1)
    cut = data[: len(data) * 2 // 3]
    try:
        out = dec.decode(cut)
    except ZaruError:
        return
    assert out.shape == (240, 320, 4)


def test_batch_decode_mixed_frames(dec):
    """zr_jpeg_decode_batch_async: frames of different sizes, subsamplings and entropy paths
    (restart intervals -> one shared device Huffman launch; no DRI -> the self-synchronising
    device decoder) in one call, each equal to libjpeg-turbo's decode."""
    from zaru_amd._lib import DeviceBuffer, lib
    from zaru_amd.jpeg import JpegDecoder
    specs = [((1080, 1920), 90, 2, {"restart_marker_blocks": 4}),
             ((480, 640), 85, 0, {}),
             ((720, 1280), 95, 1, {"restart_marker_blocks": 2}),
             ((33, 17), 90, 2, {}),
             ((1080, 1920), 90, 2, {"restart_marker_rows": 1}),
             ((240, 320), 75, 2, {"restart_marker_blocks": 1})]
    datas = [encode(synthetic(h, w, 300 + i), quality=q, subsampling=sub, **kw)
             for i, ((h, w), q, sub, kw) in enumerate(specs)]
    datas.append(encode(synthetic(200, 300, 9)[..., 0], quality=85, restart_marker_blocks=5))
    shapes = [(h, w) for (h, w), *_ in specs] + [(200, 300)]
    bufs = [DeviceBuffer(h * w * 4) for h, w in shapes]
    d = JpegDecoder(0)
    try:
        d.decode_batch_into(datas, [b.ptr for b in bufs], [w * 4 for _, w in shapes])
        lib().zr_stream_synchronize(None)
        for i, (data, (h, w)) in enumerate(zip(datas, shapes)):
            assert np.array_equal(bufs[i].download((h, w, 4), "uint8"), libjpeg_turbo_rgba(data)), i
        assert d.status() == (7, 0, 0)
    finally:
        d.close()


def test_batch_decode_rejects_a_bad_frame_before_enqueueing(dec):
    from zaru_amd._lib import DeviceBuffer, ZaruError
    from zaru_amd.jpeg import JpegDecoder
    good = encode(synthetic(64, 64, 1), quality=90, restart_marker_blocks=1)
    buf = DeviceBuffer(64 * 64 * 4 * 3)
    d = JpegDecoder(0)
    try:
        with pytest.raises(ZaruError, match="frame 1"):
            d.decode_batch_into([good, b"not a jpeg", good], [buf.ptr + i * 64 * 64 * 4 for i in range(3)], [256] * 3)
        assert d.status()[:2] == (0, 0)
        d.decode_batch_into([good] * 3, [buf.ptr + i * 64 * 64 * 4 for i in range(3)], [256] * 3)
        want = libjpeg_turbo_rgba(good)
        got = buf.download((3, 64, 64, 4), "uint8")
        for i in range(3):
            assert np.array_equal(got[i], want)
    finally:
        d.close()


def test_unaligned_output_and_odd_row_stride(dec):
    """The ABI asks only row_stride >= 4 * width: a frame buffer at an odd address with an odd
    stride takes the byte-store path of the colour stage and must hold the same pixels."""
    from zaru_amd._lib import DeviceBuffer, lib
    h, w = 37, 53
    data = encode(synthetic(h, w, 12), quality=90, restart_marker_blocks=1)
    stride = w * 4 + 3
    buf = DeviceBuffer(h * stride + 8)
    dec.decode_into(data, buf.ptr + 1, stride)
    lib().zr_stream_synchronize(None)
    raw = buf.download((h * stride + 8,), "uint8")
    got = np.stack([raw[1 + r * stride:1 + r * stride + w * 4].reshape(w, 4) for r in range(h)])
    assert np.array_equal(got, libjpeg_turbo_rgba(data))


def _with_quant(data, value):
    """The stream with every quantisation table entry set to `value` (8-bit tables)."""
    b = bytearray(data)
    i = 2
    while i + 4 <= len(b) and b[i] == 0xFF and b[i + 1] != 0xDA:
        seg = int.from_bytes(b[i + 2:i + 4], "big")
        if b[i + 1] == 0xDB:
            j = i + 4
            while j < i + 2 + seg:
                assert b[j] >> 4 == 0
                b[j + 1:j + 65] = bytes([value]) * 64
                j += 65
        i += 2 + seg
    return bytes(b)


@pytest.mark.parametrize("kw", [{}, {"restart_marker_blocks": 2}])
def test_out_of_range_coefficients_take_the_wide_idct(dec, kw):
    """A quality-100 stream re-labelled with all-255 quantisation tables dequantises past 2^15
    (no legal encoder output does): jpeg_idct_kernel's blocks fall back from int32 to 64-bit
    arithmetic, libjpeg-turbo's JLONG islow.  Checked against the oracle's 64-bit islow
    (oracle/jpeg.c) over the host decoder's coefficients of the same stream."""
    import oracle as O
    from zaru_amd import jpeg
    data = _with_quant(encode(synthetic(96, 128, 21), quality=100, **kw), 255)
    layout, coef = jpeg.coefficients(data)
    assert np.abs(coef.astype(np.int64) * 255).max() >= 1 << 15
    assert np.array_equal(dec.decode(data), O.jpeg_pixels(coef, layout))
