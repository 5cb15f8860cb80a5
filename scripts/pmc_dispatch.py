#!/usr/bin/env python3
"""Per-dispatch counter dump of a rocprofv3 --pmc run (rocpd database), in dispatch order.

    python scripts/pmc_dispatch.py <rocprofv3 -d directory> [kernel substring]

Prints one line per dispatch: id, kernel (short), grid, duration (us) and every counter.  Used
for sweeps where one process runs several settings of the same kernel (scripts/sweep_ivf.py),
which the per-kernel averages of scripts/prof_summary.py would mix.
"""
from __future__ import annotations

import collections
import glob
import os
import sqlite3
import sys


def main(src: str, sub: str = "") -> None:
    files = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    if not files:
        sys.exit(f"no rocpd database under {src}")
    c = sqlite3.connect(files[0])
    rows = collections.OrderedDict()
    for did, kn, gs, cn, v, d in c.execute("select dispatch_id, kernel_name, grid_size, counter_name, value, duration "
                                           "from counters_collection order by dispatch_id"):
        if sub and sub not in kn:
            continue
        r = rows.setdefault(did, {"kernel": kn.replace("pyr::(anonymous namespace)::", "")[:60], "grid": gs,
                                  "us": d / 1e3, "c": collections.defaultdict(float)})
        r["c"][cn] += v
    for did, r in rows.items():
        cs = " ".join(f"{k}={v:.4g}" for k, v in sorted(r["c"].items()))
        print(f"{did} {r['kernel']} grid={r['grid']} {r['us']:.1f}us {cs}")


if __name__ == "__main__":
    main(*sys.argv[1:])
