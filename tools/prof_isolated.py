"""Average duration of one kernel in a rocprofv3 kernel trace, split into launches that ran alone
on the GPU (no other kernel overlapping them: the bench's stream-serialized profile pass and the
quiet moments of the timed steps) and launches that shared it with the concurrent sub-batch
streams.  bench.py's roofline times the dominant kernel uncontended, so its average is the one
to compare with the "alone" figure (plus the ~5 us of its HIP-event brackets).
Usage: python tools/prof_isolated.py <trace_kernel_trace.csv> "<kernel name substring>"
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
alone, shared = [], []
reach = []  # latest end among launches that started at or before each one
m = 0
for s, e, _, _ in iv:
    m = max(m, e)
    reach.append(m)
last = [x for x in iv if sys.argv[2] in x[2]][-1][3]  # the profile pass's stream (it runs last)
pp = []
for i, (s, e, n, q) in enumerate(iv):
    if sys.argv[2] not in n:
        continue
    overlapped = (i > 0 and reach[i - 1] > s) or (i + 1 < len(iv) and iv[i + 1][0] < e)
    (shared if overlapped else alone).append((e - s) / 1000)
    if q == last and not overlapped:
        pp.append((e - s) / 1000)
avg = lambda v: sum(v) / len(v) if v else 0.0
print(f"{sys.argv[2]}: all {len(alone) + len(shared)} launches {avg(alone + shared):.2f} us | "
      f"alone {len(alone)} {avg(alone):.2f} us | shared {len(shared)} {avg(shared):.2f} us | "
      f"alone on the last stream (profile pass) {len(pp)} {avg(pp):.2f} us")
