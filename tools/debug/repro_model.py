"""Debug: run one model through the HIP runner with the native SIGSEGV tracer loaded."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from zaru_amd.nn import NeuralNetwork, model_bytes
ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_trace.so"))
name, s = sys.argv[1], int(sys.argv[2])
nn = NeuralNetwork.from_onnx(model_bytes(name)).load()
print("loaded", name, flush=True)
x = np.random.default_rng(0).uniform(-1, 1, (2, 3, s, s)).astype(np.float32)
outs = nn.estimate(x)
print("ok", [o.shape for o in outs], flush=True)
