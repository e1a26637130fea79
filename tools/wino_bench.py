#!/usr/bin/env python3
"""Time each Winograd F(m x m, 3x3) C-ABI stage on the c4 level shapes (HIP events on the current stream): the
transforms against the HBM roofline (algorithmic bytes: every operand read once, every output written once), the
position GEMMs in executed TF/s.
usage: tools/wino_bench.py [reps] [tile]
env WB_SHAPES=i,j (indices into SHAPES) and WB_STAGES=gemm,wgemm restrict the run (PMC passes over one kernel);
WB_PREC=32-exact times the exact-fp32 arithmetic (bit-split operands, f32-input MFMA); WB_LIB=1 adds torch.bmm on the
position GEMM's shape in the arithmetic's library dtype (fp32 for 32 / 32-exact: the hipBLASLt rate on the same batched
short-K problem)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import _lib, ops

dev = torch.device("cuda:0")
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
MT = int(sys.argv[2]) if len(sys.argv) > 2 else 4
POS = (MT + 2) ** 2
PREC = os.environ.get("WB_PREC", "32")
ops.set_precision(PREC)  # 3xBF16 (the Winograd path's default arithmetic) or exact fp32
LIB = os.environ.get("WB_LIB") == "1"
SHAPES = [(256, 8, 8, 2048, 2048), (256, 16, 16, 1024, 1024), (256, 32, 32, 512, 512), (128, 64, 64, 256, 256),
          (128, 64, 64, 512, 256),
          (256, 7, 7, 512, 512), (256, 14, 14, 256, 256), (256, 28, 28, 128, 128)]  # c2 levels (WB_SHAPES=5,6,7)
if os.environ.get("WB_SHAPES"):
    SHAPES = [SHAPES[int(i)] for i in os.environ["WB_SHAPES"].split(",")]
ONLY = set(os.environ["WB_STAGES"].split(",")) if os.environ.get("WB_STAGES") else None
st = torch.cuda.current_stream().cuda_stream


def timed(fn):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / REPS


tot = {}
for nb, h, w, ci, co in SHAPES:
    t = nb * -(-h // MT) * -(-w // MT)
    x = torch.randn(nb, h, w, ci, device=dev)
    dy = torch.randn(nb, h, w, co, device=dev)
    y = torch.empty_like(dy)
    wt = torch.randn(co, 3, 3, ci, device=dev) * 0.02
    u = torch.empty(4 * POS * ci * co, dtype=torch.uint8, device=dev)
    v = torch.empty(4 * POS * t * ci, dtype=torch.uint8, device=dev)
    d = torch.empty(4 * POS * t * co, dtype=torch.uint8, device=dev)
    m = torch.empty(POS * t * co, device=dev)
    mw = torch.empty(POS * ci * co, device=dev)
    dw = torch.empty_like(wt)
    sc = torch.rand(nb, ci, device=dev) + 0.5  # GroupNorm scale / shift rows (input transform with GroupNorm+SiLU)
    sh = torch.randn(nb, ci, device=dev) * 0.1
    ws = torch.empty(_lib.query("mvae_gemm_workspace_bytes", co, ci, t, POS), dtype=torch.uint8, device=dev)
    stages = [
        ("wt_fwd", lambda: _lib.call("mvae_winograd_weight_transform", wt.data_ptr(), u.data_ptr(), ci, co, 0, MT, st),
         4.0 * co * ci * (9 + POS), 0),
        ("wt_dgrad", lambda: _lib.call("mvae_winograd_weight_transform", wt.data_ptr(), u.data_ptr(), ci, co, 1, MT,
                                       st), 4.0 * co * ci * (9 + POS), 0),
        ("in", lambda: _lib.call("mvae_winograd_input_transform", x.data_ptr(), v.data_ptr(), nb, h, w, ci, 0, MT, st),
         4.0 * (x.numel() + POS * t * ci), 0),
        ("in_gn", lambda: _lib.call("mvae_winograd_input_transform_gn", x.data_ptr(), sc.data_ptr(), sh.data_ptr(), 1,
                                    v.data_ptr(), nb, h, w, ci, MT, st), 4.0 * (x.numel() + POS * t * ci), 0),
        ("gemm", lambda: _lib.call("mvae_winograd_gemm", v.data_ptr(), u.data_ptr(), m.data_ptr(), t, ci, co, MT, st),
         4.0 * POS * (t * ci + ci * co + t * co), 2.0 * POS * t * ci * co),
        ("out", lambda: _lib.call("mvae_winograd_output_transform", m.data_ptr(), None, None, y.data_ptr(), None, nb, h,
                                  w, co, MT, st), 4.0 * (POS * t * co + y.numel()), 0),
        ("dy", lambda: _lib.call("mvae_winograd_dy_transform", dy.data_ptr(), d.data_ptr(), nb, h, w, co, 0, MT, st),
         4.0 * (dy.numel() + POS * t * co), 0),
        ("wgemm", lambda: _lib.call("mvae_winograd_wgrad_gemm", d.data_ptr(), v.data_ptr(), mw.data_ptr(), t, co, ci, MT,
                                    ws.data_ptr(), ws.numel(), st),
         4.0 * POS * (t * ci + t * co + ci * co), 2.0 * POS * t * ci * co),
        ("wout", lambda: _lib.call("mvae_winograd_wgrad_output", mw.data_ptr(), dw.data_ptr(), 0.0, co, ci, MT, st),
         4.0 * co * ci * (POS + 9), 0),
    ]
    if LIB:
        va, ub = torch.randn(POS, t, ci, device=dev), torch.randn(POS, ci, co, device=dev)
        mo = torch.empty(POS, t, co, device=dev)
        stages.append(("lib_bmm", lambda: torch.bmm(va, ub, out=mo), 0, 2.0 * POS * t * ci * co))
    row = []
    for name, fn, nbytes, flops in stages:
        if ONLY and name not in ONLY and not (name == "in" and "wgemm" in ONLY) and not (name == "dy" and "wgemm" in ONLY):
            continue
        us = timed(fn)
        tot[name] = tot.get(name, 0.0) + us
        rate = f"{flops / us / 1e6:6.1f}TF/s" if flops else f"{nbytes / us / 1e6:5.2f}TB/s"
        row.append(f"{name} {us:7.1f}us {rate}")
    print((nb, h, w, ci, co), " | ".join(row), flush=True)
    del x, dy, y, wt, u, v, d, m, mw, dw, ws, sc, sh
    torch.cuda.empty_cache()
print("total us:", {k: round(v, 1) for k, v in tot.items()})
