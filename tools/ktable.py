"""Per-kernel table of a bench.py JSON line (uncontended profiled pass): launches, ms, share,
us/launch, algorithmic TB/s and TF.  Usage: python tools/ktable.py bench.json [other.json]"""
import json
import sys


def load(f):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    return {k["kernel"]: k for k in d["kernels"]}, d


a, da = load(sys.argv[1])
b, db = load(sys.argv[2]) if len(sys.argv) > 2 else (None, None)
tot = sum(k["ms"] for k in a.values())
print(f"{sys.argv[1]}: value {da['value']}, profiled kernel ms {tot:.2f}"
      + (f"  vs {sys.argv[2]}: value {db['value']}, ms {sum(k['ms'] for k in b.values()):.2f}" if b else ""))
for name, k in sorted(a.items(), key=lambda kv: -kv[1]["ms"]):
    us = k["ms"] * 1e3 / k["launches"]
    line = (f"{name[:58]:58s} n={k['launches']:4d} {k['ms']:7.2f}ms {100 * k['ms'] / tot:5.1f}% {us:7.1f}us "
            f"{k['bytes'] / k['ms'] / 1e9:5.2f}TB/s {k['flops'] / k['ms'] / 1e9:6.1f}TF")
    if b and name in b:
        line += f"  | was {b[name]['ms'] * 1e3 / b[name]['launches']:7.1f}us"
    print(line)
