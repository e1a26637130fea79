#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: tools/bench_brief.py <file> [label]."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lab = sys.argv[2] if len(sys.argv) > 2 else d.get("config", {}).get("workload", "")
r = d.get("roofline", {})
bp = {k: v.get("TFLOP/s") for k, v in r.get("by_pass", {}).items()}
h = r.get("hbm_kernels", {})
hb = {k: (v.get("ms"), v.get("GB/s")) for k, v in h.get("by_pass", {}).items()}
print(lab, d["value"], "img/s", d["ms_per_step"], "ms", "frac", r.get("frac"), bp, "gn", h.get("ms_per_step"), hb,
      flush=True)
