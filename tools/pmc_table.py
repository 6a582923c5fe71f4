"""Per-kernel table from the rocprofv3 --pmc passes of tools/gpu_pmc.sh: average duration,
HBM traffic (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, WRITE_SIZE as is, KiB -> B),
MFMA-busy fraction of the chip (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x duration x 2.4 GHz),
wave-state fractions (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY of SQ_WAVE_CYCLES) and
LDS bank-conflict cycles per LDS instruction.  usage: pmc_table.py <pmc dir> [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CLK_GHZ, SIMDS = 2.4, 1024


def sym(name):
    """Kernel symbol without return type, namespaces and parameter list.  The parameter list is
    the first '(' outside the template arguments (those may hold casts such as '(zr::X)1')."""
    name = name.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    name = name.replace("zr::", "").replace(" ", "")
    return name or "?"


def main():
    d = sys.argv[1]
    ctr = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for row in csv.DictReader(open(f)):
            k = sym(row["Kernel_Name"])
            ctr[k][row["Counter_Name"]] += float(row["Counter_Value"])
            ctr[k]["_n_" + row["Counter_Name"]] += 1
            key = (row["Dispatch_Id"], k)
            if key not in seen and os.path.basename(f).startswith("fetch"):
                seen.add(key)
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    rows = []
    for k, c in ctr.items():
        if k.startswith("__amd") or not dur[k]:
            continue
        avg = lambda n: c[n] / max(1.0, c["_n_" + n]) if ("_n_" + n) in c else None
        us = sum(dur[k]) / len(dur[k])
        r = {"kernel": k, "dispatches": len(dur[k]), "avg_us": round(us, 2)}
        if avg("FETCH_SIZE") is not None:
            r["fetch_MB"] = round(2 * avg("FETCH_SIZE") * 1024 / 1e6, 2)
        if avg("WRITE_SIZE") is not None:
            r["write_MB"] = round(avg("WRITE_SIZE") * 1024 / 1e6, 2)
        if "fetch_MB" in r and "write_MB" in r:
            r["hbm_GBs"] = round((r["fetch_MB"] + r["write_MB"]) * 1e6 / (us * 1e-6) / 1e9, 1)
        if avg("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            r["mfma_busy"] = round(avg("SQ_VALU_MFMA_BUSY_CYCLES") / (SIMDS * us * 1e3 * CLK_GHZ), 4)
        wc = avg("SQ_WAVE_CYCLES")
        if wc:
            for n, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_ACTIVE_INST_ANY", "active")):
                if avg(n) is not None:
                    r[lab] = round(avg(n) / wc, 3)
        li = avg("SQ_INSTS_LDS")
        if li:
            r["lds_conflict_cyc_per_inst"] = round(avg("SQ_LDS_BANK_CONFLICT") / li, 3)
        rows.append(r)
    rows.sort(key=lambda r: -r["avg_us"] * r["dispatches"])
    for r in rows:
        print(json.dumps(r))
    if len(sys.argv) > 2:
        json.dump(rows, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
