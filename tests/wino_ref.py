"""Float64 emulation of the HIP Winograd F(m x m, 3x3) convolution (csrc/winograd.hip) for the parity tests: the same
transforms, with the GEMM operands (V, U, D') rounded the way the kernels round them before the GEMM -- `rnd` maps a
float64 tensor to the values the GEMM multiplies (identity for exact fp32, bf16 round-to-nearest-even for the bf16 mode).
Test infrastructure only: it restates the algorithm in float64 so a bf16 Winograd conv (whose transform-domain rounding
differs from a direct bf16 conv's) can be checked to fp32-accumulation accuracy instead of at the bf16 algorithm error.

Shapes: x [N, C, H, W] float64, w [K, C, 3, 3]; tiles cover the image from the top-left corner (edge tiles zero-filled /
cut), padding 1."""
import torch


def bt(m):
    if m == 2:
        rows = [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]]
    else:
        rows = [[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]]
    return torch.tensor(rows, dtype=torch.float64)


def gm(m):
    if m == 2:
        rows = [[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]]
    else:
        rows = [[.25, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
                [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]]
    return torch.tensor(rows, dtype=torch.float64)


def at(m):
    if m == 2:
        rows = [[1, 1, 1, 0], [0, 1, -1, -1]]
    else:
        rows = [[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]]
    return torch.tensor(rows, dtype=torch.float64)


def bf16(t):
    return t.to(torch.bfloat16).double()


def ident(t):
    return t


def filters(w, m, rnd):
    """U [K, C, a, a] = rnd(G g G^T)."""
    g = gm(m)
    return rnd(torch.einsum("ij,kcjl,ml->kcim", g, w.double(), g))


def dgrad_weights(w):
    """The input gradient's filters g'(c, k)[r][s] = g(k, c)[2-r][2-s]: a [C, K, 3, 3] weight."""
    return w.flip(2, 3).transpose(0, 1)


def rows(x, w, bias, ns, oh, ow, m, rnd):
    """Output rows y[ns, :, oh, ow] ([len, K]) of the Winograd conv of x with w (+ bias)."""
    a = m + 2
    B, A = bt(m), at(m)
    u = filters(w, m, rnd)  # [K, C, a, a]
    n, c, h, wd = x.shape
    th, tw = -(-h // m), -(-wd // m)
    xp = torch.nn.functional.pad(x.double(), (1, 1 + tw * m - wd, 1, 1 + th * m - h))
    ti, tj = torch.div(oh, m, rounding_mode="floor"), torch.div(ow, m, rounding_mode="floor")
    ar = torch.arange(a)
    hh = (ti[:, None] * m + ar[None, :])[:, :, None].expand(-1, a, a)
    ww = (tj[:, None] * m + ar[None, :])[:, None, :].expand(-1, a, a)
    p = xp[ns[:, None, None], :, hh, ww].permute(0, 3, 1, 2)  # [S, C, a, a]
    v = rnd(torch.einsum("ij,scjk,lk->scil", B, p, B))
    mm = torch.einsum("scij,kcij->skij", v, u)
    y = torch.einsum("ij,skjl,ml->skim", A, mm, A)  # [S, K, m, m]
    r = y[torch.arange(len(ns)), :, oh % m, ow % m]
    return r + bias.double()[None, :] if bias is not None else r


def conv(x, w, m, rnd, chunk=8):
    """The whole output [N, K, H, W] (small problems)."""
    a = m + 2
    B, A = bt(m), at(m)
    u = filters(w, m, rnd)
    n, c, h, wd = x.shape
    th, tw = -(-h // m), -(-wd // m)
    xp = torch.nn.functional.pad(x.double(), (1, 1 + tw * m - wd, 1, 1 + th * m - h))
    ys = []
    for b0 in range(0, n, chunk):
        pt = xp[b0:b0 + chunk].unfold(2, a, m).unfold(3, a, m)  # [n, C, th, tw, a, a]
        v = rnd(torch.einsum("ij,nctwjk,lk->nctwil", B, pt, B))
        mm = torch.einsum("nctwij,kcij->nktwij", v, u)
        y = torch.einsum("ij,nktwjl,ml->nktwim", A, mm, A)
        ys.append(y.permute(0, 1, 2, 4, 3, 5).reshape(y.shape[0], -1, th * m, tw * m)[:, :, :h, :wd])
    return torch.cat(ys)


def wgrad(x, dy, m, rnd, cols=None, chunk=8):
    """dW [K', C, 3, 3] = G^T [sum_t rnd(A D_t A^T) (.) rnd(B^T X_t B)] G over every tile t (the output channels
    `cols` of dy only, when given)."""
    a = m + 2
    B, A, g = bt(m), at(m), gm(m)
    n, c, h, wd = x.shape
    th, tw = -(-h // m), -(-wd // m)
    xp = torch.nn.functional.pad(x.double(), (1, 1 + tw * m - wd, 1, 1 + th * m - h))
    d = dy.double() if cols is None else dy[:, cols].double()
    dp = torch.nn.functional.pad(d, (0, tw * m - wd, 0, th * m - h))
    mm = torch.zeros(d.shape[1], c, a, a, dtype=torch.float64)
    for b0 in range(0, n, chunk):
        pt = xp[b0:b0 + chunk].unfold(2, a, m).unfold(3, a, m)
        v = rnd(torch.einsum("ij,nctwjk,lk->nctwil", B, pt, B))
        dt = dp[b0:b0 + chunk].unfold(2, m, m).unfold(3, m, m)  # [n, K', th, tw, m, m]
        dd = rnd(torch.einsum("ji,nktwjl,lm->nktwim", A, dt, A))  # A D A^T with A = (A^T)^T: [a, a]
        mm += torch.einsum("nktwij,nctwij->kcij", dd, v)
    return torch.einsum("ji,kcjl,lm->kcim", g, mm, g)


UPS_TAP = ((0, 1, 1), (1, 1, 2))  # embedded tap of original tap r for output parity p (csrc/winograd.hip ups_tap)


def ups_class_kernels(w):
    """The Upsample conv's four class kernels K_pq [4, K, C, 3, 3] (float64) of w [K, C, 3, 3]: output pixel
    (2i + p, 2j + q) of nearest-x2 + 3x3 / pad-1 conv = the 3x3 / pad-1 conv of the low-resolution input with K_pq."""
    w = w.double()
    kc = torch.zeros(4, *w.shape, dtype=torch.float64)
    for pq in range(4):
        p, q = pq >> 1, pq & 1
        for r in range(3):
            for s in range(3):
                kc[pq, :, :, UPS_TAP[p][r], UPS_TAP[q][s]] += w[:, :, r, s]
    return kc


def ups_conv(x, w, m, rnd):
    """Winograd emulation of the Upsample conv: [N, K, 2H, 2W]."""
    kc = ups_class_kernels(w)
    n, c, h, wd = x.shape
    y = torch.zeros(n, w.shape[0], 2 * h, 2 * wd, dtype=torch.float64)
    for pq in range(4):
        y[:, :, pq >> 1::2, pq & 1::2] = conv(x, kc[pq], m, rnd)
    return y


def ups_dgrad(dy, w, m, rnd):
    """... its input gradient [N, C, H, W]: sum over the classes of the class sub-images of dy through the flipped,
    transposed class kernels."""
    kc = ups_class_kernels(w)
    return sum(conv(dy[:, :, pq >> 1::2, pq & 1::2], dgrad_weights(kc[pq]), m, rnd) for pq in range(4))


def ups_wgrad(x, dy, m, rnd):
    """... its weight gradient [K, C, 3, 3]: each class kernel's Winograd gradient, summed onto the taps it was built
    from."""
    dw = torch.zeros(dy.shape[1], x.shape[1], 3, 3, dtype=torch.float64)
    for pq in range(4):
        dk = wgrad(x, dy[:, :, pq >> 1::2, pq & 1::2], m, rnd)
        p, q = pq >> 1, pq & 1
        for r in range(3):
            for s in range(3):
                dw[:, :, r, s] += dk[:, :, UPS_TAP[p][r], UPS_TAP[q][s]]
    return dw
