"""Per-layer kernel times of a tools/probe_times.sh trace, aligned with the compiled plan
(zr_plan_describe): the last of the probe's repetitions, one row per launch, with the layer's
algorithmic bytes (fp32 activations in + out (+ residual)) and the achieved TB/s.
Usage: python tools/layer_table.py <model> <trace_kernel_trace.csv> [batch]"""
import csv
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from zaru_amd._lib import plan_describe  # noqa: E402
from zaru_amd.nn import model_bytes  # noqa: E402

model, trace = sys.argv[1], sys.argv[2]
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 341
plan = [l for l in plan_describe(model_bytes(model)).splitlines()
        if l.split(" ", 1)[0] not in ("input", "output") and not l.endswith(" grp=0")]  # grouped into the previous launch
rows = [r for r in csv.DictReader(open(trace)) if "zr::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-len(plan):]


def dims(s):
    m = re.search(r"\[(\d+)x(\d+)x(\d+)\]", s)
    return tuple(int(x) for x in m.groups()) if m else (0, 0, 0)


tot = 0.0
out = []
for line, r in zip(plan, rows):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += us
    f = line.split()
    i = dims(line.split(" in=")[1]) if " in=" in line else (0, 0, 0)
    o = dims(line.split(" out=")[1]) if " out=" in line else (0, 0, 0)
    res = " res=1" in line or " res=2" in line
    b = 4 * batch * (i[0] * i[1] * i[2] + o[0] * o[1] * o[2] * (2 if res else 1))
    name = r["Kernel_Name"].replace("void zr::", "").split("(")[0].replace(" ", "")
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    out.append(f"{us:7.1f}us {b / us / 1e6:5.2f}TB/s wg={wg:6d}x{r['Grid_Size_Y']:>3s} {name[:40]:40s} {f[0]} {f[1][3:]} -> {f[2][4:]} {f[3]} {f[4]}")
print(f"{model} batch {batch}: {len(rows)} launches, {tot:.1f} us")
print("\n".join(out))
