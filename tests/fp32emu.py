"""fp32 emulation of the tone-bank detectors, operation for operation.

Test infrastructure: the derived error bounds of
audio-network_amd/csrc/error_model.cpp are checked on the CPU against this
emulation (tests/test_error_bound.py), and the emulation is tied to the
kernels by a GPU test that requires the kernels' fp32 powers to equal it bit
for bit (tests/test_gpu_error_model.py). Every operation below is the one the
kernel issues, in the kernel's order:

  goertzel.hip  a = x - s2; s = fma(c, s1, a)   (Reinsch: t = fma(sg, d, x),
                d = fma(lam, s, t), s = fma(sg, s, d)); rotation
                'ws'   (re, im) = fma(-(Bx, By), s2, (Ax, Ay) * s1)   (K >= 3, n = 1024)
                'fmaf' re = fma(Ax, s1, -(Bx * s2))                    (K <= 2, n != 1024)
  fold.hip      the same chain over the folded window; F16 combines the two
                fold halves exactly (Z0 = E + O, Z8 = E - O) and sums over 8
                lanes; the C rotation `Ax * s1 - Bx * s2` is emulated as the
                compiler contracts it ('c': fma(Ax, s1, -(Bx * s2)))
  residue.hip   the 8-point class butterflies (exact integer adds, the 1/sqrt 2
                products as FMAs), the chain on both components, the 4-term
                rotation by FMAs
  window_sum.h  the reduce-scatter over the 16 lanes of a row (row_mirror,
                row_half_mirror, quad_perm [2,3,0,1], [1,0,3,2]), then
                P = re^2 + im^2 as sq + dpp(sq)
  group_sum     v += dpp(v) over xor 1, xor 2, half mirror, mirror, xor 16,
                xor 32; P = fma(re, re, im * im)

fma32 is correctly rounded: the product of two floats is exact in double, the
sum's TwoSum error decides the rare double-rounding case at a float midpoint.
"""
import numpy as np

F32 = np.float32
F64 = np.float64


def fma32(a, b, c):
    """Correctly rounded fp32 a * b + c (broadcasting)."""
    a = np.asarray(a, F32).astype(F64)
    b = np.asarray(b, F32).astype(F64)
    c = np.asarray(c, F32).astype(F64)
    p = a * b                      # exact: 24 + 24 bits
    s = p + c
    bp = s - c
    ap = s - bp
    e = (p - bp) + (c - ap)        # p + c == s + e exactly (TwoSum)
    r = s.astype(F32)
    other = np.nextafter(r, np.where(s > r.astype(F64), F32(np.inf), F32(-np.inf)).astype(F32))
    mid = (r.astype(F64) + other.astype(F64)) * 0.5 == s
    fix = mid & (e != 0)
    if np.any(fix):
        r = np.where(fix, np.where(e > 0, np.maximum(r, other), np.minimum(r, other)), r)
    return r.astype(F32)


def chain_plain(xs, c):
    """s = fma(c, s1, x - s2) over the last axis; returns (s1, s2)."""
    c = F32(c)
    s1 = np.zeros(xs.shape[:-1], F32)
    s2 = np.zeros(xs.shape[:-1], F32)
    for i in range(xs.shape[-1]):
        a = (xs[..., i] - s2).astype(F32)
        s = fma32(c, s1, a)
        s2, s1 = s1, s
    return s1, s2


def chain_reinsch(xs, lam, sg):
    lam, sg = F32(lam), F32(sg)
    s = np.zeros(xs.shape[:-1], F32)
    d = np.zeros(xs.shape[:-1], F32)
    for i in range(xs.shape[-1]):
        t = fma32(sg, d, xs[..., i])
        dd = fma32(lam, s, t)
        s = fma32(sg, s, dd)
        d = dd
    return s, d


def rotate(s1, s2, r, mode):
    """r: [..., 4] float32 {Ax, Ay, Bx, By} broadcast against s1."""
    ax, ay, bx, by = (r[..., i] for i in range(4))
    if mode == "ws":
        re = fma32(-bx, s2, (ax * s1).astype(F32))
        im = fma32(-by, s2, (ay * s1).astype(F32))
    elif mode in ("fmaf", "c"):
        re = fma32(ax, s1, -((bx * s2).astype(F32)))
        im = fma32(ay, s1, -((by * s2).astype(F32)))
    else:
        raise ValueError(mode)
    return re, im


_LANES = np.arange(16)
# window_sum.h stage partners (lane bit B): row_mirror, row_half_mirror, quad_perm
_WS_PARTNER = {3: 15 - _LANES, 2: (_LANES & 8) | (7 - (_LANES & 7)), 1: _LANES ^ 2, 0: _LANES ^ 1}


def ws_reduce(v, stages=(3, 2, 1, 0)):
    """window_sum.h reduce-scatter: v [W, 16, V] lane lists -> lane j holds
    value (j mod VS) in v[:, j, 0] (and value 16 + j in v[:, j, 16] if V = 32)."""
    v = v.astype(F32).copy()
    V = v.shape[2]
    VS = min(V, 16)
    for B in stages:
        pt = _WS_PARTNER[B]
        if (1 << B) >= VS:
            v = (v + v[:, pt, :]).astype(F32)
            continue
        bit = ((_LANES >> B) & 1).astype(bool)[None, :]
        new = v.copy()
        for e in range(V):
            if e & (1 << B):
                continue
            f = e | (1 << B)
            keep = np.where(bit, v[:, :, f], v[:, :, e])
            send = np.where(bit, v[:, :, e], v[:, :, f])
            new[:, :, e] = (keep + send[:, pt]).astype(F32)
        v = new
    return v


def ws_powers(re, im):
    """re, im [W, 16, K] lane partials (lane = segment) -> P [W, K] as the
    window_sum.h epilogue computes them."""
    W, _, K = re.shape
    KP = 1 if K <= 1 else 2 if K <= 2 else 4 if K <= 4 else 8 if K <= 8 else 16
    v = np.zeros((W, 16, 2 * KP), F32)
    v[:, :, 0:2 * K:2] = re
    v[:, :, 1:2 * K:2] = im
    v = ws_reduce(v)
    P = np.zeros((W, K), F32)
    for lst in (0, 16) if 2 * KP > 16 else (0,):
        sq = (v[:, :, lst] * v[:, :, lst]).astype(F32)
        p = (sq + sq[:, _LANES ^ 1]).astype(F32)
        VS = min(2 * KP, 16)
        for j in range(0, VS, 2):
            t = j // 2 + (8 if lst else 0)
            if t < K:
                P[:, t] = p[:, j]
    return P


def group_sum(v, log2g):
    """v [W, G, ...] over the G = 2^log2g lanes of a window -> lane 0's total."""
    G = 1 << log2g
    lanes = np.arange(G)
    partners = [lanes ^ 1, lanes ^ 2, (lanes & ~7) | (7 - (lanes & 7)), (lanes & ~15) | (15 - (lanes & 15)),
                lanes ^ 16, lanes ^ 32]
    v = v.astype(F32)
    for s in range(log2g):
        v = (v + v[:, partners[s]]).astype(F32)
    return v[:, 0]


def fmaf_power(re, im):
    return fma32(re, re, (im * im).astype(F32))


def _windows(x, n, hop, W):
    idx = np.arange(W)[:, None] * hop + np.arange(n)[None, :]
    return x[idx]


def detector_powers(info, x, n, hop, W, K):
    """The fp32 tone powers [W, K] (caller's tone order) the detector of plan
    `info` (audio_network_amd.plan_info) computes for W windows of x."""
    xw = _windows(np.asarray(x), n, hop, W).astype(np.int64)
    method, log2g = info["method"], info["log2g"]
    G = 1 << log2g
    rot = info["rot"]
    coef, sgn = info["coef"], info["sgn"]
    slot_tone = info["slot_tone"]
    P = np.zeros((W, K), F32)
    if method == 1:  # plain bank
        seg = xw.reshape(W, G, 64).astype(F32)
        ws = log2g == 4 and K >= 3
        re = np.zeros((W, G, K), F32)
        im = np.zeros((W, G, K), F32)
        for k in range(K):
            if info["reinsch"]:
                s1, s2 = chain_reinsch(seg, coef[k], sgn[k])
            else:
                s1, s2 = chain_plain(seg, coef[k])
            r = rot[k * G:(k + 1) * G][None, :, :]
            re[:, :, k], im[:, :, k] = rotate(s1, s2, r, "ws" if ws else "fmaf")
        if ws:
            return ws_powers(re, im)
        for k in range(K):
            P[:, k] = fmaf_power(group_sum(re[:, :, k], log2g), group_sum(im[:, :, k], log2g))
        return P
    if method == 3:  # fold
        xf = xw.reshape(W, 8, n // 8).sum(axis=1)
        if info["f16"]:
            z0 = (xf[:, :64] + xf[:, 64:]).astype(F32)
            z8 = (xf[:, :64] - xf[:, 64:]).astype(F32)
            re = np.zeros((W, 16, 4), F32)
            im = np.zeros((W, 16, 4), F32)
            for sl in range(8):
                z = (z0 if sl < 4 else z8).reshape(W, 8, 8)
                s1, s2 = chain_plain(z, coef[sl])
                r = rot[sl * 16:sl * 16 + 8][None, :, :]
                a, b = rotate(s1, s2, r, "ws")
                lanes = slice(0, 8) if sl < 4 else slice(8, 16)
                re[:, lanes, sl % 4] = a
                im[:, lanes, sl % 4] = b
            v = np.zeros((W, 16, 8), F32)
            v[:, :, 0::2] = re
            v[:, :, 1::2] = im
            v = ws_reduce(v, stages=(2, 1, 0))
            sq = (v[:, :, 0] * v[:, :, 0]).astype(F32)
            p = (sq + sq[:, _LANES ^ 1]).astype(F32)
            for j in range(0, 16, 2):
                P[:, slot_tone[j // 2]] = p[:, j]
            return P
        seg = xf.reshape(W, G, 8).astype(F32)
        re = np.zeros((W, G, K), F32)
        im = np.zeros((W, G, K), F32)
        for k in range(K):
            s1, s2 = chain_plain(seg, coef[k])
            r = rot[k * G:(k + 1) * G][None, :, :]
            re[:, :, k], im[:, :, k] = rotate(s1, s2, r, "c")
        if log2g == 4:
            return ws_powers(re, im)
        for k in range(K):
            P[:, k] = fmaf_power(group_sum(re[:, :, k], log2g), group_sum(im[:, :, k], log2g))
        return P
    if method == 4:  # residue
        Pn = n // 8
        xs = xw.reshape(W, 8, Pn).astype(F32)          # xs[:, m, r] = x[r + m P]
        xl = xs.reshape(W, 8, G, 8)                     # [W, m, lane j, i]
        x = [xl[:, m] for m in range(8)]                # [W, G, 8] each
        a0, a2 = (x[0] + x[4]).astype(F32), (x[2] + x[6]).astype(F32)
        d0, d2 = (x[0] - x[4]).astype(F32), (x[2] - x[6]).astype(F32)
        a1, a3 = (x[1] + x[5]).astype(F32), (x[3] + x[7]).astype(F32)
        d1, d3 = (x[1] - x[5]).astype(F32), (x[3] - x[7]).astype(F32)
        e0, e1 = (a0 + a2).astype(F32), (a0 - a2).astype(F32)
        e2, e3 = (a1 + a3).astype(F32), (a1 - a3).astype(F32)
        u, v = (d1 - d3).astype(F32), (d1 + d3).astype(F32)
        kr = F32(0.70710678118654752)
        cls = {0: ((e0 + e2).astype(F32), (e0 - e2).astype(F32)),
               1: (fma32(u, kr, d0), fma32(v, -kr, -d2)),
               2: (fma32(u, -kr, d0), fma32(v, -kr, d2)),
               3: (e1, e3)}
        re = np.zeros((W, G, K), F32)
        im = np.zeros((W, G, K), F32)
        for sl in range(K):
            lo, hi = cls[int(info["zcls"][sl])]
            s1l, s2l = chain_plain(lo, coef[sl])
            s1h, s2h = chain_plain(hi, coef[sl])
            c12 = rot[(sl * G + np.arange(G)) * 2][None]
            c34 = rot[(sl * G + np.arange(G)) * 2 + 1][None]
            xr = (c12[..., 0] * s1l).astype(F32)
            xi = (c12[..., 1] * s1l).astype(F32)
            xr, xi = fma32(c12[..., 2], s1h, xr), fma32(c12[..., 3], s1h, xi)
            xr, xi = fma32(c34[..., 0], s2l, xr), fma32(c34[..., 1], s2l, xi)
            xr, xi = fma32(c34[..., 2], s2h, xr), fma32(c34[..., 3], s2h, xi)
            re[:, :, sl], im[:, :, sl] = xr, xi
        if log2g == 4:
            Ps = ws_powers(re, im)
        else:
            Ps = np.stack([fmaf_power(group_sum(re[:, :, k], log2g), group_sum(im[:, :, k], log2g))
                           for k in range(K)], axis=1)
        for sl in range(K):
            P[:, slot_tone[sl]] = Ps[:, sl]
        return P
    raise ValueError(f"method {method}")


def energies(x, n, hop, W):
    """(raw sum x^2, folded sum xf^2) per window, exact."""
    xw = _windows(np.asarray(x), n, hop, W).astype(np.int64)
    xf = xw.reshape(W, 8, n // 8).sum(axis=1)
    return (xw * xw).sum(axis=1).astype(F64), (xf * xf).sum(axis=1).astype(F64)


def exact_dft_mag(x, n, hop, W, omegas):
    """|X(w)| per window and frequency in long double (|X| only)."""
    xw = _windows(np.asarray(x), n, hop, W).astype(np.longdouble)
    t = np.arange(n, dtype=np.longdouble)
    out = np.zeros((W, len(omegas)), F64)
    for k, w in enumerate(omegas):
        ph = np.longdouble(w) * t
        re = xw @ np.cos(ph)
        im = xw @ np.sin(ph)
        out[:, k] = np.sqrt(re * re + im * im).astype(F64)
    return out
