#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel CSV per training step: python tools/prof_summary.py <csv> <steps>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6/steps:.1f} ms/step")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:9.2f} ms/step {int(r['Calls'])/steps:7.1f} calls/step "
          f"{float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
