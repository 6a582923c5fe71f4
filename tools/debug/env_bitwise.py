"""Bitwise comparison of one network's outputs with and without an environment setting (A/B
knobs that must not change results).  Usage: python tools/debug/env_bitwise.py <model> <size>
<batch> VAR=value"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
net = NeuralNetwork.from_onnx(model_bytes(sys.argv[3])).load()
s, b = int(sys.argv[4]), int(sys.argv[5])
x = np.random.default_rng(11).uniform(-1.0, 1.0, size=(b, 3, s, s)).astype(np.float32)
np.savez(sys.argv[2], *net.estimate(x))
"""
model, size, batch, setting = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
var, val = setting.split("=", 1)
res = []
for env in ({}, {var: val}):
    path = f"/tmp/env_bitwise_{len(res)}.npz"
    subprocess.run([sys.executable, "-c", CHILD, REPO, path, model, size, batch], env=dict(os.environ, **env),
                   check=True, timeout=110)
    res.append(np.load(path))
ok = all(np.array_equal(res[0][k], res[1][k]) for k in res[0].files)
print(model, setting, "bitwise equal" if ok else "DIFFERENT")
sys.exit(0 if ok else 1)
