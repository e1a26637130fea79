"""Float64 model of larger Winograd output tiles (round 6): Cook-Toom F(m x m, 3x3) transforms for
m = 4, 6, 8 from a list of interpolation points (plus the point at infinity), applied to one conv in the arithmetics of
csrc/winograd.hip -- V / U rounded to fp32 by the transforms, then the GEMM operands as 3xBF16 (hi + lo bf16 splits, the
lo x lo product dropped), exact fp32 or bf16, M rounded to fp32 -- against the float64 direct conv. Also the GEMM MACs
per output pixel at each of c4's image widths (edge tiles count whole). CPU only; prints one line per configuration."""
import math

import torch
import torch.nn.functional as F

torch.set_default_dtype(torch.float64)


def cook_toom(points, m, r=3):
    n = m + r - 1
    at = torch.zeros(m, n)
    g = torch.zeros(n, r)
    for j in range(n - 1):
        den = math.prod(points[j] - points[q] for q in range(n - 1) if q != j)
        for i in range(m):
            at[i, j] = points[j] ** i
        for k in range(r):
            g[j, k] = points[j] ** k / den
    at[m - 1, n - 1] = 1
    g[n - 1, r - 1] = 1
    # B^T from the identity sum_j A^T[i, j] G[j, k] B^T[j, l] = [l == i + k] (least squares; residual printed)
    rows, rhs = [], []
    for i in range(m):
        for k in range(r):
            for col in range(n):
                row = torch.zeros(n, n)
                row[:, col] = at[i] * g[:, k]
                rows.append(row.flatten())
                rhs.append(1.0 if col == i + k else 0.0)
    a, b = torch.stack(rows), torch.tensor(rhs)
    sol = torch.linalg.lstsq(a, b[:, None]).solution[:, 0]
    return at, g, sol.view(n, n), float((a @ sol - b).abs().max())


def bf16(t):
    return t.to(torch.bfloat16).double()


def f32(t):
    return t.float().double()


def conv(x, w, at, g, bt, m, mode):
    a = m + 2
    n, c, h, wd = x.shape
    t = F.pad(x, (1, 1, 1, 1)).unfold(2, a, m).unfold(3, a, m)
    v = torch.einsum("ij,nctujk,lk->ntucil", bt, t, bt)
    u = torch.einsum("ij,kcjl,ml->kcim", g, w, g)
    mm = lambda p, q: torch.einsum("ntucij,kcij->ntukij", p, q)  # noqa: E731
    if mode == "f64":
        res = mm(v, u)
    else:
        v, u = f32(v), f32(u)
        if mode == "3xbf16":
            vh, uh = bf16(v), bf16(u)
            res = mm(vh, uh) + mm(vh, bf16(u - uh)) + mm(bf16(v - vh), uh)
        elif mode == "exact":
            res = mm(v, u)
        else:
            res = mm(bf16(v), bf16(u))
        res = f32(res)
    y = torch.einsum("ij,ntukjl,ml->ntukim", at, res, at)
    return y.permute(0, 3, 1, 4, 2, 5).reshape(n, -1, h, wd)


def main():
    torch.manual_seed(0)
    x = F.silu(torch.randn(2, 128, 24, 24))
    w = torch.randn(64, 128, 3, 3) / (3 * 128 ** 0.5)
    y = F.conv2d(x, w, padding=1)
    for pts in ([0, 1, -1, 2, -2], [0, 1, -1, 2, -2, .5, -.5], [0, 1, -1, .5, -.5, 1.5, -1.5],
                [0, 1, -1, 2, -2, .5, -.5, 1.5, -1.5], [0, 1, -1, 2, -2, .5, -.5, 4, -4]):
        m = len(pts) - 1
        at, g, bt, res = cook_toom(pts, m)
        errs = {mode: float((conv(x, w, at, g, bt, m, mode) - y).norm() / y.norm())
                for mode in ("f64", "exact", "3xbf16", "bf16")}
        macs = {wd: (math.ceil(wd / m) * (m + 2)) ** 2 / wd ** 2 for wd in (64, 32, 16, 8)}
        print(f"F({m}x{m}) points {pts} (B^T residual {res:.1e}): rel err " +
              " ".join(f"{k} {v:.2e}" for k, v in errs.items()) +
              " | GEMM MACs per output pixel (direct 9): " + " ".join(f"W{k} {v:.2f}" for k, v in macs.items()))


if __name__ == "__main__":
    main()
