"""The C-ABI contract of include/zaru_hip.h under concurrency: "a session is safe to use from
several threads at once" (HandTracker workers call estimate(&self) on one shared network,
crates/zaru/src/hand/tracking.rs:165-181; NeuralNetwork is Clone + Send + Sync).

Four threads call zr_session_run and zr_cnn_estimate_views on ONE session handle, each with its
own inputs, repeatedly; every result must be bit-identical to the serial run of the same input.
ctypes releases the GIL around foreign calls, so the calls really overlap."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_concurrent_calls_on_one_session_are_bit_identical():
    from zaru_amd.nn import Cnn, ColorMapper, NeuralNetwork, model_bytes
    nn = NeuralNetwork.from_onnx(model_bytes("hand_landmark_lite")).load()
    cnn = Cnn(nn, ColorMapper.linear(0.0, 1.0))
    T, REPS = 4, 6
    rng = np.random.default_rng(41)
    xs = [rng.random((2 + t, 3, 224, 224), dtype=np.float32) for t in range(T)]
    imgs = [rng.integers(0, 256, size=(240 + 40 * t, 320, 4), dtype=np.uint8) for t in range(T)]
    views = [[(160.0, 120.0 + 10 * t, 150.0 + 5 * k, 150.0 + 5 * k, 0.2 * k - 0.3) for k in range(3)]
             for t in range(T)]
    want_run = [nn.estimate(x) for x in xs]
    want_views = [cnn.estimate_views(im, v) for im, v in zip(imgs, views)]
    errors = []
    barrier = threading.Barrier(T)

    def worker(t):
        try:
            barrier.wait()
            for rep in range(REPS):
                got = nn.estimate(xs[t]) if rep % 2 == 0 else cnn.estimate_views(imgs[t], views[t])
                want = want_run[t] if rep % 2 == 0 else want_views[t]
                for a, b in zip(got, want):
                    if not np.array_equal(a, b):
                        errors.append((t, rep))
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors


def test_errors_are_thread_local():
    """zr_last_error is per thread (anyhow::Error travels with its own Result)."""
    from zaru_amd import _lib
    L = _lib.lib()
    msgs = {}

    def bad(t):
        rc = L.zr_session_run(None, 1, None, 1, None, 1)
        msgs[t] = (rc, L.zr_last_error().decode())

    ths = [threading.Thread(target=bad, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert all(rc == -1 and "null" in m for rc, m in msgs.values())
