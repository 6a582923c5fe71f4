"""Run one model's session on a device-resident batch a few times (for rocprofv3 kernel traces
and PMC passes on single kernels).  Usage: python tools/kernel_probe.py <model> [batch] [reps]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from zaru_amd._lib import DeviceBuffer, synchronize  # noqa: E402
from zaru_amd.nn import NeuralNetwork, model_bytes  # noqa: E402

model = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 341
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
nn = NeuralNetwork.from_onnx(model_bytes(model)).load()
shape = nn.inputs()[0][1]
x = np.random.default_rng(0).uniform(-1, 1, size=(batch,) + tuple(shape[1:])).astype(np.float32)
din = DeviceBuffer.from_array(x)
outs = [DeviceBuffer(int(np.prod(s)) * 4) for s in nn.output_shapes(batch)]
for _ in range(reps):
    nn.estimate_device(batch, din.ptr, [o.ptr for o in outs])
synchronize()
print("ok", model, batch, reps)
