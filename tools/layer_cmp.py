"""Side-by-side per-launch times (us) of the last repetition in two rocprofv3 kernel traces of
tools/kernel_probe.py (e.g. a form switched on / off).  Usage: python tools/layer_cmp.py A.csv B.csv"""
import csv,sys,os
sys.path.insert(0,os.path.dirname(os.path.abspath(__file__)))
from pmc_table import sym
def load(path,reps=5):
    rows=[r for r in csv.DictReader(open(path)) if "zr::" in r["Kernel_Name"]]
    rows.sort(key=lambda r:int(r["Start_Timestamp"]))
    n=len(rows)//reps
    out=[]
    for r in rows[-n:]:
        us=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000
        k=sym(r["Kernel_Name"])
        out.append((k,us))
    return out
a=load(sys.argv[1]); b=load(sys.argv[2])
if len(a)!=len(b):  # different launch lists (a fused form on one side): each list with its total
    for name,l in (("A",a),("B",b)):
        print(f"== {name}: {sys.argv[1] if name=='A' else sys.argv[2]}")
        for k,us in l: print(f"{us:8.1f} {k}")
        print(f"total {sum(u for _,u in l):.1f}  launches {len(l)}")
    sys.exit(0)
ta=tb=0
for (ka,ua),(kb,ub) in zip(a,b):
    ta+=ua; tb+=ub
    print(f"{ua:8.1f} {ub:8.1f} {ka[:48]:48s} {kb[:48]}")
print(f"total {ta:.1f} {tb:.1f}  launches {len(a)} {len(b)}")
