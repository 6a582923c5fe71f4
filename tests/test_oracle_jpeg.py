"""Pin the JPEG oracle (oracle/jpeg.c: libjpeg-turbo's islow IDCT, fancy upsampling and
YCbCr->RGBA restated as libjpeg's own row loops) and the product's host entropy decoder
(zr_jpeg_coefficients, runtime/jpeg.cpp) against libjpeg-turbo itself: Pillow in this image
links it and decodes with turbojpeg's defaults, the configuration of the reference's
libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:164-182).  CPU only; the GPU kernels are
checked against the same library in tests/test_gpu_jpeg.py."""
import io

import numpy as np
import pytest

import oracle as O
from zaru_amd import jpeg


def _img(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([(x * 255 // max(1, w - 1)), (y * 255 // max(1, h - 1)), ((x + y) * 5) % 256], -1)
    return (img + rng.integers(-50, 51, size=img.shape)).clip(0, 255).astype(np.uint8)


def _encode(img, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", **kw)
    return b.getvalue()


def _pil(data):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"))


@pytest.mark.parametrize("h,w,q,sub,kw", [
    (61, 97, 75, 2, {}), (33, 17, 95, 2, {}), (64, 64, 50, 0, {}), (45, 131, 85, 1, {}),
    (120, 160, 75, 2, {"restart_marker_blocks": 3}), (97, 203, 100, 0, {"restart_marker_rows": 1}),
    (240, 320, 30, 2, {}), (9, 9, 90, 2, {})])
def test_oracle_pixels_equal_libjpeg_turbo(h, w, q, sub, kw):
    data = _encode(_img(h, w, h * 31 + w), quality=q, subsampling=sub, **kw)
    layout, coef = jpeg.coefficients(data)
    assert (layout["width"], layout["height"]) == (w, h)
    got = O.jpeg_pixels(coef, layout)
    want = _pil(data)
    diff = np.abs(got.astype(int) - want.astype(int))
    assert diff.max() == 0, (h, w, q, sub, int(diff.max()), int((diff > 0).sum()))


def test_oracle_grayscale():
    data = _encode(_img(50, 70, 2)[..., 1], quality=85)
    layout, coef = jpeg.coefficients(data)
    assert layout["ncomp"] == 1
    assert np.array_equal(O.jpeg_pixels(coef, layout), _pil(data))


def test_coefficient_layout_420():
    layout, coef = jpeg.coefficients(_encode(_img(1080, 1920, 4), quality=90))
    # 4:2:0: MCUs of 16x16, luma 240 x 136 blocks (1080 -> 68 MCU rows), chroma 120 x 68
    assert (layout["h_samp"], layout["v_samp"]) == (2, 2)
    assert layout["bw"] == [240, 120, 120] and layout["bh"] == [136, 68, 68]
    assert coef.shape == (240 * 136 + 2 * 120 * 68, 64)
