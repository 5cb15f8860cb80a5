"""Per-kernel averages of one rocprofv3 --pmc pass (its counter_collection.csv), as a small text table; the
CSV itself can be deleted on the box afterwards (it may exceed gpurun's copy-back limit).

    python scripts/pmc_sum.py <pmc outdir> [kernel substring ...] > summary.txt
"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
keys = sys.argv[2:]
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
if not files:
    sys.exit(f"no counter_collection.csv under {d}")
agg = defaultdict(lambda: defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        if keys and not any(k in n for k in keys):
            continue
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in agg.items():
    parts = [f"{c}: n={len(v)} mean={sum(v) / len(v):.6g} max={max(v):.6g}" for c, v in cs.items()]
    print(n[:120], "|", "; ".join(parts))
