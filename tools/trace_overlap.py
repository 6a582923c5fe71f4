"""Concurrency summary of a rocprofv3 kernel trace (CSV): over the last `--tail` fraction of the
dispatches, wall span, summed kernel time, busy union and per-stream busy time, plus the idle
gaps.  Used to compare the pipeline's stream overlap between versions.

    python3 tools/trace_overlap.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--tail 0.3]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=float, default=0.3)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Queue_Id"],
                         r["Kernel_Name"]))
    rows.sort()
    rows = rows[int(len(rows) * (1 - a.tail)):]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    ksum = sum(e - s for s, e, *_ in rows)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, *_ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = collections.defaultdict(int)
    names = collections.Counter()
    for s, e, st, q, n in rows:
        per[(st, q)] += e - s
        if n.startswith("__amd"):
            names[n] += 1
    span = t1 - t0
    print(f"dispatches {len(rows)}  span {span / 1e6:.3f} ms  kernel sum {ksum / 1e6:.3f} ms "
          f"(x{ksum / span:.2f})  busy union {busy / 1e6:.3f} ms ({busy / span:.1%})")
    gaps.sort(reverse=True)
    print(f"idle gaps: {len(gaps)}  total {sum(gaps) / 1e6:.3f} ms  largest(us) {[round(g / 1e3, 1) for g in gaps[:8]]}")
    for k, v in sorted(per.items()):
        print(f"  stream {k[0]} queue {k[1]}: {v / 1e6:.3f} ms")
    for n, c in names.most_common():
        print(f"  runtime kernel {n}: {c}")


if __name__ == "__main__":
    main()
