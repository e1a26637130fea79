#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: tools/bench_brief.py <file> [label]. Reads the compact stdout line
(by_pass entries [launches, ms, TFLOP/s]) or a full detail record (by_pass entries as dicts)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lab = sys.argv[2] if len(sys.argv) > 2 else d.get("config", {}).get("workload", "")
r = d.get("roofline") or {}


def tf(v):
    return v[2] if isinstance(v, list) else v.get("TFLOP/s")


bp = {k: tf(v) for k, v in (r.get("by_pass") or {}).items()}
h = r.get("hbm_kernels") or {}
print(lab, d["value"], "img/s", d["ms_per_step"], "ms", "frac", r.get("frac"), bp, "gn", h.get("ms_per_step"),
      h.get("frac"), flush=True)
