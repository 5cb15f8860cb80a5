#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (rocprofv3 rocpd databases) into text files for profiles/.

    python scripts/prof_summary.py gpurun_out/prof_<tag> profiles/<tag>

Writes:
  kernel_stats.csv   rocprofv3 --kernel-trace --stats equivalent: per kernel symbol AND grid size
                     (the scan kernel serves k-means assignment, the coarse probe and the list scan
                     with different grids), calls, total/avg/min/max duration in ns
  counters.csv       per counter pass: mean counter value per (kernel, grid) over its dispatches
  summary.md         the list-scan launch: duration, HBM bytes (FETCH_SIZE x 2, gfx950 correction,
                     MI355X_MICROARCH.md "HBM"), VALU instruction count and issue utilisation
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sqlite3
import sys


def db(path):
    files = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    return sqlite3.connect(files[0]) if files else None


def short(name: str) -> str:
    return name.replace("pyr::(anonymous namespace)::", "")[:110]


def main(src: str, dst: str) -> None:
    os.makedirs(dst, exist_ok=True)
    kt = db(os.path.join(src, "kt"))
    rows = kt.execute("select name, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count, count(*), sum(duration), "
                      "avg(duration), min(duration), max(duration) from kernels group by name, grid_x "
                      "order by sum(duration) desc").fetchall()
    total = sum(r[7] for r in rows)
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_threads", "wg", "lds_bytes", "vgpr", "sgpr", "calls", "total_ns", "avg_ns",
                    "min_ns", "max_ns", "pct"])
        for r in rows:
            w.writerow([short(r[0])] + list(r[1:7]) + [int(r[7]), round(r[8], 1), int(r[9]), int(r[10]),
                                                       round(100.0 * r[7] / total, 2)])
    counters = {}
    for p in ("fetch", "sq", "mfma"):
        c = db(os.path.join(src, p))
        if c is None:
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        nd = collections.defaultdict(set)
        dur = collections.defaultdict(list)
        for did, kn, gs, cn, v, d in c.execute("select dispatch_id, kernel_name, grid_size, counter_name, value, "
                                               "duration from counters_collection"):
            key = (short(kn), gs)
            acc[key][cn] += v
            if did not in nd[key]:
                nd[key].add(did)
                dur[key].append(d)
        for key in acc:
            n = len(nd[key])
            counters.setdefault(key, {"dispatches": n, "avg_ns_profiled": sum(dur[key]) / n})
            for cn, v in acc[key].items():
                counters[key][cn] = v / n
    names = sorted({cn for v in counters.values() for cn in v})
    with open(os.path.join(dst, "counters.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_threads"] + names)
        for key, v in sorted(counters.items(), key=lambda kv: -kv[1].get("avg_ns_profiled", 0)):
            w.writerow(list(key) + [f"{v.get(n, ''):.6g}" if n in v else "" for n in names])
    # the dominant kernel of the timed region: the longest scan dispatch group that is not k-means (fewest calls
    # per grid is the bench's search; k-means assignment runs once per Lloyd iteration with grid = n rows)
    md = [f"# rocprofv3 summary ({os.path.basename(os.path.normpath(src))})", ""]
    md.append("| kernel | grid threads | calls | avg ms | vgpr | lds B |")
    md.append("|---|---|---|---|---|---|")
    for r in rows[:12]:
        md.append(f"| `{short(r[0])}` | {r[1]} | {r[6]} | {r[8] / 1e6:.4f} | {r[4]} | {r[3]} |")
    md.append("")
    for key, v in counters.items():
        if not any(s in key[0] for s in ("scan", "mfma_filter", "stream16_kernel")) or v.get("avg_ns_profiled", 0) < 1e6:
            continue
        line = [f"## `{key[0]}` grid {key[1]}", "",
                f"- dispatches profiled: {v['dispatches']}, avg duration under counters: "
                f"{v['avg_ns_profiled'] / 1e6:.3f} ms"]
        if "FETCH_SIZE" in v:
            hbm = v["FETCH_SIZE"] * 1024 * 2  # KB, x2 for gfx950 wide-read halving
            line.append(f"- FETCH_SIZE {v['FETCH_SIZE']:.4g} KB -> HBM read ~{hbm / 1e9:.3f} GB per launch "
                        f"(x2 gfx950 correction) = {hbm / (v['avg_ns_profiled'] * 1e-9) / 1e9:.0f} GB/s")
        if "SQ_INSTS_MFMA" in v and "GRBM_GUI_ACTIVE" in v:
            cyc = v["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs (MI355X_MICROARCH.md "DVFS give-back")
            clk = cyc / (v["avg_ns_profiled"] * 1e-9) / 1e9
            line.append(f"- SQ_INSTS_MFMA {v['SQ_INSTS_MFMA']:.4g}, SQ_VALU_MFMA_BUSY_CYCLES "
                        f"{v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.4g}, effective clock {clk:.2f} GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v and cyc > 0:
                line.append(f"- MFMA busy: {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024) * 100:.1f}% of "
                            f"1024 SIMD x GRBM_GUI_ACTIVE cycles")
        if "SQ_INSTS_VALU" in v:
            waves = v.get("SQ_WAVES", 0)
            line.append(f"- SQ_INSTS_VALU {v['SQ_INSTS_VALU']:.4g} wave-instr, SQ_WAVES {waves:.4g}, "
                        f"SQ_INSTS_LDS {v.get('SQ_INSTS_LDS', 0):.4g}, LDS bank-conflict cycles "
                        f"{v.get('SQ_LDS_BANK_CONFLICT', 0):.4g}")
            secs = v["avg_ns_profiled"] * 1e-9
            issue_cap = 1024 * 0.5 * 2.4e9 * secs  # 1024 SIMDs x 1 wave64 VALU op / 2 clk at 2.4 GHz
            line.append(f"- VALU issue utilisation vs 1 wave64 op / 2 clk / SIMD at 2.4 GHz: "
                        f"{v['SQ_INSTS_VALU'] / issue_cap * 100:.1f}%")
            if "SQ_WAVE_CYCLES" in v:
                res = v["SQ_WAVE_CYCLES"] * 4 / (1024 * 2.4e9 * secs)
                line.append(f"- mean resident waves per SIMD (SQ_WAVE_CYCLES quad-cycles): {res:.2f}")
        md += line + [""]
    with open(os.path.join(dst, "summary.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
