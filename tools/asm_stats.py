"""Per-kernel instruction counts from a device assembly file (hipcc --cuda-device-only -S):
LDS instruction kinds, VGPR count and spills.  usage: asm_stats.py file.s [substring ...]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().splitlines()
want = sys.argv[2:]
kern, stats, meta = None, {}, {}
for line in src:
    m = re.match(r"^(_Z\w+):", line)
    if m:
        kern = m.group(1)
        stats[kern] = Counter()
        continue
    if kern and line.startswith(".Lfunc_end"):
        kern = None
        continue
    if kern:
        m = re.match(r"\s+(ds_\w+|global_load_lds\w*|v_mfma\w*)", line)
        if m:
            stats[kern][m.group(1)] += 1
cur = None
for line in src:
    m = re.match(r"\s+\.name:\s+(_Z\w+)", line)
    if m:
        cur = m.group(1)
    m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|agpr_count):\s+(\d+)", line)
    if m and cur:
        meta.setdefault(cur, {})[m.group(1)] = int(m.group(2))
for k, c in stats.items():
    if want and not all(w in k for w in want):
        continue
    print(k, meta.get(k, {}), dict(sorted(c.items())))
