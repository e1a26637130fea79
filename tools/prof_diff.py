#!/usr/bin/env python3
"""Per-step kernel table from two rocprofv3 --stats runs differing only in the timed step count.
    python3 tools/prof_diff.py <dir_short> <dir_long> <extra_steps>"""
import csv, glob, sys


def stats(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        out[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    return out


def main():
    a, b, n = stats(sys.argv[1]), stats(sys.argv[2]), int(sys.argv[3])
    rows = []
    for k in b:
        c0, t0 = a.get(k, (0, 0.0))
        c1, t1 = b[k]
        if c1 - c0 > 0:
            rows.append(((t1 - t0) / n, (c1 - c0) / n, k))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    calls = sum(r[1] for r in rows)
    print(f"per replayed step over {n} extra steps: {calls:.1f} launches, {tot / 1e6:.3f} ms device time")
    print(f"{'ms/step':>9} {'share':>6} {'calls':>7} {'avg_us':>8}  kernel")
    for t, c, k in rows:
        print(f"{t / 1e6:9.3f} {t / tot:6.3f} {c:7.1f} {t / c / 1e3:8.2f}  {k[:150]}")


if __name__ == "__main__":
    main()
