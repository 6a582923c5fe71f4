"""Compare a network's outputs with the fused inverted-residual form on and off (child processes,
ZARU_HIP_FORMS is per process) for a few batch sizes; prints max |diff| per output."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
model, batch, path = sys.argv[2], int(sys.argv[3]), sys.argv[4]
net = NeuralNetwork.from_onnx(model_bytes(model)).load()
s = net.inputs()[0][1]
x = np.random.default_rng(5).uniform(-1.0, 1.0, size=(batch,) + tuple(s[1:])).astype(np.float32)
np.savez(path, *net.estimate(x))
"""
model = sys.argv[1] if len(sys.argv) > 1 else "hand_landmark_lite"
for batch in [int(b) for b in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "3", "36"])]:
    res = {}
    for forms in ("", "-ir"):
        path = f"/tmp/irc_{batch}_{forms or 'def'}.npz"
        subprocess.run([sys.executable, "-c", CHILD, REPO, model, str(batch), path], check=True,
                       env=dict(os.environ, ZARU_HIP_FORMS=forms), timeout=120)
        with np.load(path) as z:
            res[forms] = [z[k] for k in z.files]
    for i, (a, b) in enumerate(zip(res[""], res["-ir"])):
        d = np.abs(a - b).reshape(batch, -1).max(axis=1)
        bad = np.nonzero(d)[0]
        print(model, "batch", batch, "out", i, "max|diff|", float(d.max()), "images differing", len(bad),
              bad[:10].tolist(), flush=True)
