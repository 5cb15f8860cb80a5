"""Per-step timeline of a bench run from a rocprofv3 kernel trace (run_kernel_trace.csv).

    python scripts/kt_steps.py <kernel_trace.csv> [kernel-name substring] [--step i]

Prints, for every dispatch of the marker kernel (default: the IVF list scan), its duration and the time
since the previous one (the step period), and with --step i the kernels of step i (name, duration, gap).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = "scan_kernel<128"
    detail = None
    rest = sys.argv[2:]
    if "--step" in rest:
        i = rest.index("--step")
        detail = int(rest[i + 1])
        rest = rest[:i] + rest[i + 2:]
    if rest:
        marker = rest[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    prev = None
    for j, i in enumerate(idx):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        period = (s - prev) / 1e6 if prev is not None else 0.0
        print(f"{j:4d} {marker} dur {(e - s) / 1e6:.3f} ms  period {period:.3f} ms")
        prev = s
    if detail is not None and 0 <= detail < len(idx) - 1:
        a, b = idx[detail], idx[detail + 1]
        # from the first kernel after the previous step's last scan-relative position: print a full period
        span = rows[a - (idx[1] - idx[0]) + (b - a) // 2: b] if detail > 0 else rows[:b]
        last = None
        tot = 0.0
        for r in rows[idx[detail - 1] + 1 if detail > 0 else 0: b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"].replace("void pyr::(anonymous namespace)::", "").split("(")[0][:70]
            gap = (s - last) / 1e3 if last is not None else 0.0
            tot += (e - s) / 1e3
            print(f"  {name:70s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f} us  grid {r['Grid_Size_X']}")
            last = e
        print(f"  sum of kernel durations {tot:.1f} us")
        del span


if __name__ == "__main__":
    main()
