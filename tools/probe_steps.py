#!/usr/bin/env python3
"""Where does a short bench run lose time?  Builds bench.py's config-3 workload, idles (as the
bench does while its CPU baseline runs), then times blocks of software-pipelined steps, each
block bracketed by a device synchronize, and prints one JSON line per block."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    idle = float(sys.argv[1]) if len(sys.argv) > 1 else 12.0
    blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    torch.cuda.set_device(0)
    import zaru_amd.host as H
    t0 = time.perf_counter()
    w = bench.Workload(H, "face", 0, 1024, 0, 16, 3, True)
    print(json.dumps({"setup_s": round(time.perf_counter() - t0, 3)}), flush=True)
    time.sleep(idle)
    for b in range(blocks):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bench.run_steps([w], per, None, 0, 1, None)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"block": b, "steps": per, "ms_per_step": round(1e3 * el / per, 3)}), flush=True)


if __name__ == "__main__":
    main()
