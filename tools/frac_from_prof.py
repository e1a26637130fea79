#!/usr/bin/env python3
"""Recompute a bench line's GEMM-family roofline fraction from a rocprofv3 per-step kernel table.

    python3 tools/frac_from_prof.py <bench_detail.json> <prof_<cfg>_per_step.txt> [--peak TFLOPS] [--config CFG]

(--config: a config of the detail file's `configs` block -- c1, c2, c3, c5, c4x -- instead of the headline c4.)

The bench's `by_pass` entries carry each pass's algorithmic FLOPs per step (TF/s x ms); the rocprof table (tools/
prof_diff.py output: ms/step per kernel over replayed steps) gives the device time of the kernels those passes launch
-- the implicit-GEMM kernel, its split-K reducer / wgrad finish, the Winograd transforms, the fused attention and the
row softmax. frac = FLOPs / (kernel time x peak). Kernel time from rocprof counts concurrently running kernels (the
two-stream backward) in full, so this fraction is a lower bound where the streams overlap."""
import json
import re
import sys

FAMILY = re.compile(r"gemm3x_kernel|splitk_reduce|wgrad_finish|wino_|attn_small|attn_tile|softmax_rows|w_transpose|"
                    r"w_ups_dgrad|wgrad_small_cout|wgrad_direct|conv_direct|tap_select|wcls|conv_weight")


def main():
    detail, table = sys.argv[1], sys.argv[2]
    peak = float(sys.argv[sys.argv.index("--peak") + 1]) if "--peak" in sys.argv else None
    d = json.load(open(detail))
    if "--config" in sys.argv:
        d = d["configs"][sys.argv[sys.argv.index("--config") + 1]]
    r = d["roofline"]
    peak = peak or float(r["peak"])
    flops = sum(p["TFLOP/s"] * p["ms"] * 1e9 for p in r["by_pass"].values())
    fam_ms, other_ms, step_ms = 0.0, 0.0, None
    for line in open(table):
        m = re.match(r"per replayed step over .*?, ([\d.]+) ms device time", line)
        if m:
            step_ms = float(m.group(1))
        m = re.match(r"\s+([\d.]+)\s+[\d.]+\s+[\d.]+\s+[\d.]+\s+(.*)$", line)
        if m:
            if FAMILY.search(m.group(2)):
                fam_ms += float(m.group(1))
            else:
                other_ms += float(m.group(1))
    frac = flops / (fam_ms * 1e-3) / (peak * 1e12)
    print(json.dumps({"bench_frac": r["frac"], "prof_frac": round(frac, 4), "ratio": round(frac / r["frac"], 3),
                      "alg_TFLOP_per_step": round(flops / 1e12, 3), "family_ms_per_step_rocprof": round(fam_ms, 2),
                      "family_ms_per_step_bench": r.get("gemm_ms_per_step"), "other_kernels_ms": round(other_ms, 2),
                      "device_ms_per_step": step_ms, "peak_TFLOPS": peak}))


if __name__ == "__main__":
    main()
