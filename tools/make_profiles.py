#!/usr/bin/env python3
"""Turn a round-end profiling run (tools/final_prof.sh <tag>) into the committed evidence under profiles/:
  profiles/<round>_<cfg>_kernel_summary.txt  per-step kernel time of the rocprofv3 kernel trace of
      `bench.py --steps 3 --warmup 0 --no-kernel-timing` (3 steps, nothing else on the GPU), normalised by
      the 3 steps, plus the gemm3x_kernel average launch duration next to the bench's live HIP-event figure
  profiles/<round>_<cfg>_bench.json / .detail.txt  the bench line and its per-shape GEMM timings
usage: tools/make_profiles.py <run-tag> <round>"""
import collections, csv, json, os, shutil, sys

tag, rnd = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", tag)
dst = os.path.join(root, "profiles")
STEPS = 3
for cfg in ("c4", "c2", "c3", "c5", "c1"):
    bj = os.path.join(src, f"bench_{cfg}.json")
    if not os.path.exists(bj):
        continue
    line = open(bj).read().strip().splitlines()[-1]
    bench = json.loads(line)
    with open(os.path.join(dst, f"{rnd}_{cfg}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    det = [l for l in open(os.path.join(src, f"bench_{cfg}.err")) if l.startswith("[detail]")]
    with open(os.path.join(dst, f"{rnd}_{cfg}_gemm_detail.txt"), "w") as f:
        f.write("".join(det))
    tr = os.path.join(src, f"prof_{cfg}", "run_kernel_trace.csv")
    if not os.path.exists(tr):
        continue
    rows = list(csv.DictReader(open(tr)))
    # steps the profiled process executed: the 3 timed ones, plus for a graph-replayed config (c1-c3) the set-up
    # eager step (--warmup 0) and the first replay after the capture
    graphed = "graph" in str(bench.get("config", {}).get("step_launch", ""))
    STEPS = 3 + (2 if graphed else 0)
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"]
        key = "gemm3x_kernel (all tile / operand instantiations)" if "gemm3x_kernel" in name else name.split("(")[0]
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot = sum(v[1] for v in agg.values())
    HELPERS = ("splitk_reduce", "bias_reduce", "w_transpose", "w_ups_dgrad", "split_bf16", "ups_wgrad_combine",
               "tap_select", "wgrad_direct", "wgrad_small_cout")
    fam = sum(v[1] for k, v in agg.items() if k.startswith("gemm3x") or any(h in k for h in HELPERS))
    g = agg["gemm3x_kernel (all tile / operand instantiations)"]
    out = [f"rocprofv3 --kernel-trace --stats -- python3 bench.py --config {cfg} --steps 3 --warmup 0 "
           f"--no-cpu-baseline --no-kernel-timing   (round {rnd}, run {tag}; normalised by the {STEPS} steps it "
           f"executes{': 1 eager set-up + 1 replay after the capture + 3 timed replays' if graphed else ''})",
           f"kernel time {tot / STEPS:.2f} ms/step over {len(rows) / STEPS:.0f} launches/step "
           f"(bench line: {bench['ms_per_step']} ms/step wall)",
           f"gemm3x_kernel: {g[1] / STEPS:.2f} ms/step, {g[0] / STEPS:.1f} launches/step, "
           f"average {g[1] / max(g[0], 1) * 1e3:.1f} us/launch (bench live HIP events: "
           f"{(bench.get('roofline') or {}).get('avg_launch_us')} us/launch)",
           # the live HIP-event bracket is the whole conv / attention GEMM op: its helper kernels (split-K and bias
           # reducers, weight re-layouts / pre-splits, the direct small-channel wgrad kernels) run inside it
           f"conv/attention op family (gemm3x + helpers inside the live bracket): {fam / STEPS:.2f} ms/step "
           f"(bench live HIP events: {(bench.get('roofline') or {}).get('gemm_ms_per_step')} ms/step)", "",
           f"{'ms/step':>9} {'calls/step':>10} {'avg us':>9}  kernel"]
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        out.append(f"{t / STEPS:9.2f} {c / STEPS:10.1f} {t / c * 1e3:9.1f}  {k[:110]}")
    with open(os.path.join(dst, f"{rnd}_{cfg}_kernel_summary.txt"), "w") as f:
        f.write("\n".join(out) + "\n")
    print("\n".join(out[:4]))
