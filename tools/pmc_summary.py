#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs (all dispatches, all instances) per counter name."""
import collections, csv, glob, sys

tot = collections.defaultdict(float)
disp = set()
for pat in sys.argv[1:]:
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add((f, r["Dispatch_Id"]))
for k in sorted(tot):
    print(f"{k:34s} {tot[k]:18.0f}")
