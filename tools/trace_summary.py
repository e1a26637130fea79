#!/usr/bin/env python3
"""Per-step kernel summary of a rocprofv3 kernel trace: tools/trace_summary.py <run_kernel_trace.csv> <steps> [top]"""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
S = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"]
    k = "gemm3x_kernel (all instantiations)" if "gemm3x" in n else n.split("(")[0][:100]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"kernel time {tot / S:.3f} ms/step over {len(rows) / S:.0f} launches/step")
print("  ms/step calls/step    avg us  kernel")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1] / S:9.3f} {v[0] / S:10.1f} {1000 * v[1] / v[0]:9.1f}  {k}")
