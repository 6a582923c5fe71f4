"""The JPEG frame source's host half without a GPU: header parsing through
the C ABI and the refusal of streams outside the supported baseline subset."""
import io

import numpy as np
import pytest

from zaru_amd import jpeg
from zaru_amd._lib import ZaruError


def _encode(shape, **kw):
    from PIL import Image
    rng = np.random.default_rng(3)
    b = io.BytesIO()
    Image.fromarray(rng.integers(0, 256, size=shape, dtype=np.uint8)).save(b, "JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("shape", [(61, 97, 3), (1080, 1920, 3), (7, 5), (16, 16, 3)])
def test_info_reads_the_frame_header(shape):
    assert jpeg.info(_encode(shape, quality=80)) == (shape[1], shape[0])


def test_progressive_is_refused():
    with pytest.raises(ZaruError) as e:
        jpeg.info(_encode((32, 32, 3), progressive=True))
    assert "progressive" in str(e.value)


@pytest.mark.parametrize("cut", [2, 20, 100])
def test_truncated_headers_are_errors(cut):
    with pytest.raises(ZaruError):
        jpeg.info(_encode((40, 40, 3))[:cut])


def test_garbage_is_an_error():
    rng = np.random.default_rng(9)
    for _ in range(50):
        blob = b"\xff\xd8" + rng.integers(0, 256, size=int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
        try:
            jpeg.info(blob)
        except ZaruError:
            pass
