"""Debug: expose intermediate tensors of an ONNX graph as extra graph outputs and compare the
HIP runner against the f64 oracle tensor by tensor (first divergent layer).
usage: bisect_outputs.py <model> <input side> [batch]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np


def varint(b, i):
    r = s = 0
    while True:
        c = b[i]; i += 1; r |= (c & 0x7f) << s; s += 7
        if c < 0x80:
            return r, i


def enc_varint(v):
    out = bytearray()
    while True:
        c = v & 0x7f; v >>= 7
        out.append(c | (0x80 if v else 0))
        if not v:
            return bytes(out)


def fields(b):
    i = 0
    while i < len(b):
        s = i
        k, i = varint(b, i); f, w = k >> 3, k & 7
        if w == 0: v, i = varint(b, i)
        elif w == 2: n, i = varint(b, i); v = b[i:i + n]; i += n
        elif w == 5: v = b[i:i + 4]; i += 4
        elif w == 1: v = b[i:i + 8]; i += 8
        yield f, w, v, b[s:i]


def with_outputs(model: bytes, names):
    """The graph truncated after the producer of the last of `names`, whose only outputs are
    `names` (no tensor may be both a graph output and consumed, so callers pass one name)."""
    out = bytearray()
    for f, w, v, raw in fields(model):
        if f == 7 and w == 2:
            g = bytearray()
            last = None
            nodes = [(ff, raw2, [x.decode() for f3, w3, x, _ in fields(v2) if f3 == 2] if ff == 1 else [])
                     for ff, ww, v2, raw2 in fields(v)]
            for k, (ff, raw2, outs) in enumerate(nodes):
                if names[-1] in outs:
                    last = k
            for k, (ff, raw2, outs) in enumerate(nodes):
                if ff == 12 or (ff == 1 and k > last):
                    continue
                g += raw2
            g = bytes(g)
            for n in names:
                vi = b"\x0a" + enc_varint(len(n)) + n.encode()
                g += b"\x62" + enc_varint(len(vi)) + vi  # field 12, wire 2
            out += b"\x3a" + enc_varint(len(g)) + g
        else:
            out += raw
    return bytes(out)


def node_outputs(model: bytes):
    g = [v for f, w, v, _ in fields(model) if f == 7][0]
    res = []
    for f, w, v, _ in fields(g):
        if f == 1:
            op = [x for ff, ww, x, _ in fields(v) if ff == 4][0].decode()
            outs = [x.decode() for ff, ww, x, _ in fields(v) if ff == 2]
            res.append((op, outs[0]))
    return res


def main():
    name, s = sys.argv[1], int(sys.argv[2])
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    import oracle as O
    from zaru_amd.nn import NeuralNetwork
    path = os.path.join(ROOT, "zaru_amd", "models", name + ".onnx")
    model = open(path, "rb").read()
    picks = [o for op, o in node_outputs(model) if op in ("Relu", "PRelu", "Add", "Resize", "Clip")]
    lo = 0.0 if name.startswith(("palm", "hand")) else -1.0
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 256, size=(batch, 3, s, s), dtype=np.uint8)
    x = codes.astype(np.float32) * np.float32((1.0 - lo) / 255.0) + np.float32(lo)
    ref = O.Net(path, f64=True)
    want = {}
    for i in range(batch):
        ref.run(x[i:i + 1], as_f64=True)
        for t in picks:
            want.setdefault(t, []).append(ref.tensor(t).reshape(-1))
    only = sys.argv[4].split(",") if len(sys.argv) > 4 else None
    for c0, t in enumerate(picks):
        if only and t not in only and str(c0) not in only:
            continue
        chunk = [t]
        m2 = with_outputs(model, chunk)
        nn = NeuralNetwork.from_onnx(m2).load()
        got = nn.estimate(x)
        for j, t in enumerate(chunk):
            g = got[-1].reshape(batch, -1)
            w = np.stack(want[t])
            err = np.abs(g - w).max(axis=1)
            print(f"{c0 + j:3d} {t:40s} {g.shape[1]:8d} maxerr/img {' '.join(f'{e:.2e}' for e in err)}  |w|max {np.abs(w).max():.2f}", flush=True)


if __name__ == "__main__":
    main()
