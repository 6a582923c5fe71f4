"""Summarise rocprofv3 --pmc counter CSVs (one or more passes) per kernel symbol: counter
totals per dispatch, averaged over dispatches.  Usage: python tools/pmc_summary.py <dir> [filter]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d, filt=None):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if filt and filt not in k:
                continue
            per[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[(k, row["Counter_Name"])].add(row["Dispatch_Id"])
    out = {}
    for k, ctr in per.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in ctr.items()}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    print(json.dumps(res, indent=1))
