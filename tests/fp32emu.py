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
  fold.hip      the same chain over the folded window, rotation 'fmaf'; F16
                combines the two fold halves exactly (Z0 = E + O, Z8 = E - O),
                rotation 'ws', and sums over 8 lanes
  residue.hip   the 8-point class butterflies (exact integer adds, the 1/sqrt 2
                products as FMAs), the chain on both components, the 4-term
                rotation by FMAs
  window_sum.h  the reduce-scatter over the 16 lanes of a row (row_mirror,
                row_half_mirror, quad_perm [2,3,0,1], [1,0,3,2]), then
                P = fma(re, re, im^2) (im^2 from the partner lane)
  group_sum     v += dpp(v) over xor 1, xor 2, half mirror, mirror, xor 16,
                xor 32; P = fma(re, re, im * im)

fma32 is correctly rounded: the product of two floats is exact in double, the
sum's TwoSum error decides the rare double-rounding case at a float midpoint.
"""
import numpy as np

F32 = np.float32
F64 = np.float64
PI_L = np.longdouble("3.14159265358979323846264338327950288")  # pi to long double precision


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
    elif mode == "fmaf":
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
        a = v[:, :, lst]
        sq = (a * a).astype(F32)
        p = fma32(a, a, sq[:, _LANES ^ 1])
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
            p = fma32(v[:, :, 0], v[:, :, 0], sq[:, _LANES ^ 1])
            for j in range(0, 16, 2):
                P[:, slot_tone[j // 2]] = p[:, j]
            return P
        seg = xf.reshape(W, G, 8).astype(F32)
        re = np.zeros((W, G, K), F32)
        im = np.zeros((W, G, K), F32)
        for k in range(K):
            s1, s2 = chain_plain(seg, coef[k])
            r = rot[k * G:(k + 1) * G][None, :, :]
            re[:, :, k], im[:, :, k] = rotate(s1, s2, r, "fmaf")
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
        ph = np.asarray(w, np.longdouble) * t
        re = xw @ np.cos(ph)
        im = xw @ np.sin(ph)
        out[:, k] = np.sqrt(re * re + im * im).astype(F64)
    return out


# ---------------------------------------------------------------------------
# fft_quad.hip (the shipped FUSED 4 kernel), operation for operation: complex
# values as (re, im) pairs of float32 arrays.

def _c(re, im):
    return (np.asarray(re, F32), np.asarray(im, F32))


def _add(a, b):
    return ((a[0] + b[0]).astype(F32), (a[1] + b[1]).astype(F32))


def _sub(a, b):
    return ((a[0] - b[0]).astype(F32), (a[1] - b[1]).astype(F32))


def _add_mj(x, y):   # x + (-j) y
    return ((x[0] + y[1]).astype(F32), (x[1] - y[0]).astype(F32))


def _sub_mj(x, y):   # x - (-j) y
    return ((x[0] - y[1]).astype(F32), (x[1] + y[0]).astype(F32))


def _bfly(x, y, w):
    """QTB_T / QTB_U / QTB_V: t = fma(y, w.x, x); u = x + w y by
    fma(y.yx, (-w.y, w.y), t); v = fma(x, 2, -u)."""
    wr, wi = w
    t = (fma32(y[0], wr, x[0]), fma32(y[1], wr, x[1]))
    u = (fma32(y[1], -wi, t[0]), fma32(y[0], wi, t[1]))
    v = (fma32(x[0], F32(2), -u[0]), fma32(x[1], F32(2), -u[1]))
    return u, v


def _mjw(w):          # -j w, as the QTB_TM / QTB_UM operand modifiers read it
    return (w[1], -w[0])


_W32 = [(F32(np.cos(2 * np.pi * j / 32)), F32(-np.sin(2 * np.pi * j / 32))) for j in range(32)]


def _w32(e):
    return _W32[e % 32]


def _dft4_triv(x):
    a0, a1 = _add(x[0], x[2]), _sub(x[0], x[2])
    c0, c1 = _add(x[1], x[3]), _sub(x[1], x[3])
    return [_add(a0, c0), _add_mj(a1, c1), _sub(a0, c0), _sub_mj(a1, c1)]


def _dft4_geo(x, w, w2):
    """Geometric DFT-4 of (x0, w x1, w^2 x2, w^3 x3) in two fused stages
    (dft4_fused_k / dft4_fused_v / dft4x2_fused_v): a = x0 +- w^2 x2,
    c = x1 +- w^2 x3, X0 / X2 = a0 +- w c0, X1 / X3 = a1 +- (-j w) c1."""
    a0, a1 = _bfly(x[0], x[2], w2)
    c0, c1 = _bfly(x[1], x[3], w2)
    X0, X2 = _bfly(a0, c0, w)
    X1, X3 = _bfly(a1, c1, _mjw(w))
    return [X0, X1, X2, X3]


def _dft8(x):
    """dftf<8, ., 4>: two DFT-4 (even / odd i1), then dft8_last."""
    e = _dft4_triv([x[0], x[2], x[4], x[6]])
    o = _dft4_triv([x[1], x[3], x[5], x[7]])
    u0, v0 = _add(e[0], o[0]), _sub(e[0], o[0])
    u1, v1 = _bfly(e[1], o[1], _w32(4))
    u2, v2 = _add_mj(e[2], o[2]), _sub_mj(e[2], o[2])
    u3, v3 = _bfly(e[3], o[3], _w32(12))
    return [u0, u1, u2, u3, v0, v1, v2, v3]


def _dft32(a):
    """dftf<32, 1, 4> over a[0..31]: a DFT-8 over i1 per column i2 < 4, then per
    k1 the geometric DFT-4 over i2 with ratio W32^k1; natural order out."""
    cols = [_dft8([a[i2 + 4 * i1] for i1 in range(8)]) for i2 in range(4)]
    out = [None] * 32
    for k1 in range(8):
        y = [cols[i2][k1] for i2 in range(4)]
        if k1 == 0:
            X = _dft4_triv(y)
        elif k1 == 4:   # w^2 = -j: dft4_fused_kq
            a0, a1 = _add_mj(y[0], y[2]), _sub_mj(y[0], y[2])
            c0, c1 = _add_mj(y[1], y[3]), _sub_mj(y[1], y[3])
            X0, X2 = _bfly(a0, c0, _w32(4))
            X1, X3 = _bfly(a1, c1, _w32(12))
            X = [X0, X1, X2, X3]
        else:           # dft4_fused_k: w^2 = W32^{2 k1}, w = W32^k1, -j w = W32^{k1 + 8}
            a0, a1 = _bfly(y[0], y[2], _w32(2 * k1))
            c0, c1 = _bfly(y[1], y[3], _w32(2 * k1))
            X0, X2 = _bfly(a0, c0, _w32(k1))
            X1, X3 = _bfly(a1, c1, _w32(k1 + 8))
            X = [X0, X1, X2, X3]
        for k2 in range(4):
            out[k1 + 8 * k2] = X[k2]
    return out


def _tw512(e):
    e = np.asarray(e) & 511
    ang = -2.0 * np.pi * e / 512.0
    return (np.cos(ang).astype(F32), np.sin(ang).astype(F32))


def fft_spectrum(x, hop, W):
    """|X_b|^2, b = 0..512, of W 1024-sample windows as fft1024_quad_kernel
    computes them (float32 [W, 513])."""
    xw = _windows(np.asarray(x), 1024, hop, W).astype(F32)
    z = (xw[:, 0::2], xw[:, 1::2])                      # z[n] = x[2n] + i x[2n+1]
    # lane t: a[n1] = z[t + 16 n1]; arrays [W, 16] per n1
    a = [(z[0][:, n1 * 16:(n1 + 1) * 16], z[1][:, n1 * 16:(n1 + 1) * 16]) for n1 in range(32)]
    A = _dft32(a)                                        # A[k1][:, t] = DFT-32 of lane t at k1
    t = np.arange(16)
    cols = [t, np.where(t == 0, 16, 32 - t)]             # lane t': columns t' and k1b
    Z = []
    for col in cols:
        # b[n2] = A_{n2}[col] for lane t': the transpose
        Ak_re = np.stack([A[k][0] for k in range(32)], axis=1)   # [W, 32 (k1), 16 (t)]
        Ak_im = np.stack([A[k][1] for k in range(32)], axis=1)
        b = [(Ak_re[:, col, n2], Ak_im[:, col, n2]) for n2 in range(16)]  # [W, 16 lanes t']
        v, v2 = _tw512(4 * col), _tw512(8 * col)
        y = [None] * 16
        for i2 in range(4):       # inner geometric DFT-4 over i1 (rows i2 + 4 i1), ratio v
            X = _dft4_geo([b[i2 + 4 * i1] for i1 in range(4)], v, v2)
            for k1 in range(4):
                y[i2 + 4 * k1] = X[k1]
        out = [None] * 16
        for k1 in range(4):       # outer over i2, ratio g = W512^{col + 32 k1}
            g, g2 = _tw512(col + 32 * k1), _tw512(2 * (col + 32 * k1))
            X = _dft4_geo([y[4 * k1 + i2] for i2 in range(4)], g, g2)
            for k2 in range(4):
                out[k1 + 4 * k2] = X[k2]
        Z.append(out)             # Z[sl][k2] = Z[col + 32 k2]
    # real post-pass: pair j of lane t: P = Z[kP], Q = Z[512 - kP]
    P_out = np.zeros((W, 513), F32)
    ang = -2.0 * np.pi * np.arange(512) / 1024.0
    t1024 = (np.cos(ang).astype(F32), np.sin(ang).astype(F32))
    l0 = t == 0
    for j in range(16):
        Pr, Pi = Z[0][j]
        Qr, Qi = Z[1][15 - j]
        if j < 8:   # lane 0: column 16's Z[16 + 32 j]
            Pr = np.where(l0, Z[1][j][0], Pr)
            Pi = np.where(l0, Z[1][j][1], Pi)
        else:       # lane 0: Z[32 (16 - j)]
            Qr = np.where(l0, Z[0][16 - j][0], Qr)
            Qi = np.where(l0, Z[0][16 - j][1], Qi)
        kP = np.where(l0 & (j < 8), 16 + 32 * j, t + 32 * j)
        Wr = (F32(0.5) * t1024[0][kP]).astype(F32)
        Wi = (F32(0.5) * t1024[1][kP]).astype(F32)
        S = ((Pr + Qr).astype(F32), (Pi - Qi).astype(F32))
        D = ((Pi + Qi).astype(F32), (Qr - Pr).astype(F32))
        tt = ((D[1] * Wi).astype(F32), (D[1] * Wr).astype(F32))
        T = (fma32(D[0], Wr, -tt[0]), fma32(D[0], Wi, tt[1]))
        R0 = (fma32(S[0], F32(0.5), T[0]), fma32(S[0], F32(0.5), -T[0]))
        R1 = (fma32(S[1], F32(0.5), T[1]), fma32(S[1], F32(0.5), -T[1]))
        sq = ((R1[0] * R1[0]).astype(F32), (R1[1] * R1[1]).astype(F32))
        pw = (fma32(R0[0], R0[0], sq[0]), fma32(R0[1], R0[1], sq[1]))
        rows = np.arange(W)[:, None]
        P_out[rows, kP[None, :].repeat(W, 0)] = pw[0]
        P_out[rows, (512 - kP)[None, :].repeat(W, 0)] = pw[1]
    z0 = Z[0][0]                  # lane 0: Z[0]
    px = ((z0[0] + z0[1]).astype(F32), (z0[0] - z0[1]).astype(F32))
    P_out[:, 0] = (px[0][:, 0] * px[0][:, 0]).astype(F32)
    P_out[:, 512] = (px[1][:, 0] * px[1][:, 0]).astype(F32)
    return P_out
