"""Second, independent restatement of the reference path in numpy float32 --
tests only. It exists to catch transcription errors in the C oracle: the two
are written separately (vectorised numpy here, scalar C there) from the same
reference lines and must agree bit for bit. Slow; small inputs only.

numpy >= 2 (NEP 50): Python scalars are "weak", so float32 op Python-scalar
stays float32 and every operation below rounds once in float32.
"""
import math

import numpy as np

f32 = np.float32


def reflect101(i, n):
    if n == 1:
        return 0
    i = -i if i < 0 else i
    return 2 * n - 2 - i if i >= n else i


def sobel(img):
    """cv::Sobel ksize 3 scale 1/8 reflect-101 (src/main.cpp:19-20,34-35)."""
    H, W = img.shape
    xi = np.arange(W)
    xm = np.array([reflect101(x - 1, W) for x in xi])
    xp = np.array([reflect101(x + 1, W) for x in xi])
    R = img[:, xp] - img[:, xm]
    S = img * f32(0.25) + (img[:, xm] + img[:, xp]) * f32(0.125)
    yi = np.arange(H)
    ym = np.array([reflect101(y - 1, H) for y in yi])
    yp = np.array([reflect101(y + 1, H) for y in yi])
    dx = R * f32(0.25) + (R[ym] + R[yp]) * f32(0.125)
    dy = S[yp] - S[ym]
    return dx.astype(f32), dy.astype(f32)


def pyramid(img, C):
    levels = []
    for l in range(C + 1):
        if l == 0:
            gx, gy = sobel(img)
            lev = np.sqrt(gx * gx + gy * gy)
        else:
            p = levels[-1][0]
            lev = (((p[0::2, 0::2] + p[0::2, 1::2]) + p[1::2, 0::2]) + p[1::2, 1::2]) * f32(0.25)
        dx, dy = sobel(lev)
        levels.append((lev.astype(f32), dx, dy))
    return levels


def eigen_sum(x):
    """Eigen 3.3 SSE redux order over a float32 vector."""
    x = np.asarray(x, f32)
    n = x.size
    if n < 4:
        r = x[0]
        for i in range(1, n):
            r = r + x[i]
        return r
    a = (n // 4) * 4
    a2 = (n // 8) * 8
    p0 = x[0:4].copy()
    if a > 4:
        p1 = x[4:8].copy()
        for i in range(8, a2, 8):
            p0 = p0 + x[i:i + 4]
            p1 = p1 + x[i + 4:i + 8]
        p0 = p0 + p1
        if a > a2:
            p0 = p0 + x[a2:a2 + 4]
    r = (p0[0] + p0[2]) + (p0[1] + p0[3])
    for i in range(a, n):
        r = r + x[i]
    return r


def lu_solve(h00, h01, h10, h11, b0, b1):
    a00, a01, a10, a11, c0, c1 = h00, h01, h10, h11, b0, b1
    if abs(a10) > abs(a00):
        a00, a10 = a10, a00
        a01, a11 = a11, a01
        c0, c1 = c1, c0
    l10 = a10 / a00 if a00 != 0 else a10
    a11 = a11 - l10 * a01
    c1 = c1 - l10 * c0
    c1 = c1 / a11
    c0 = c0 - c1 * a01
    c0 = c0 / a00
    return c0, c1


def search_level(dxp, dyp, I1p, pad, W, H, ps, st, it, norm, init, I0p=None):
    """One PatchGrid level over padded planes; init: dict id -> (u, v) or None.
    I0p (padded frame-0 level image) given: paper mode,
    b = sum(g*I1n) - sum(g*Tn) with Tn the (mean-normalised) template."""
    npw = int(math.ceil(f32(W) / f32(st)))
    nph = int(math.ceil(f32(H) / f32(st)))
    offw = (W - (npw - 1) * st) // 2
    offh = (H - (nph - 1) * st) // 2
    hp = ps // 2
    thr = f32(ps) / f32(2)
    lb = -f32(ps) / f32(2)
    ubw = f32(W + ps // 2 - 2)
    ubh = f32(H + ps // 2 - 2)
    us = np.zeros((npw * nph, 2), f32)
    for gx in range(npw):
        for gy in range(nph):
            pid = gx * nph + gy
            rx, ry = f32(gx * st + offw), f32(gy * st + offh)
            px, py = int(rx) + pad, int(ry) + pad
            gdx = dxp[py - hp:py + hp, px - hp:px + hp].reshape(-1)
            gdy = dyp[py - hp:py + hp, px - hp:px + hp].reshape(-1)
            h00 = eigen_sum(gdx * gdx)
            h01 = eigen_sum(gdx * gdy)
            h11 = eigen_sum(gdy * gdy)
            h10 = h01
            if h00 * h11 - h10 * h01 == 0:
                h00 = f32(float(h00) + 1e-10)
                h11 = f32(float(h11) + 1e-10)
            bt0 = bt1 = None
            if I0p is not None:
                tn = I0p[py - hp:py + hp, px - hp:px + hp].reshape(-1).astype(f32)
                if norm:
                    tn = tn - eigen_sum(tn) / f32(ps * ps)
                bt0, bt1 = eigen_sum(gdx * tn), eigen_sum(gdy * tn)
            iu, iv = init(pid, rx, ry) if init else (f32(0), f32(0))
            u0, u1 = iu, iv
            sx, sy = rx + u0, ry + u1

            def oob(x, y):
                return x < lb or y < lb or x > ubw or y > ubh

            def warp(x, y):
                l, k = np.floor(x), np.floor(y)
                a, b = x - l, y - k
                w0, w1, w2, w3 = (1 - a) * (1 - b), a * (1 - b), b * (1 - a), a * b
                X = int(np.ceil(x + f32(1e-5))) + pad
                Y = int(np.ceil(y + f32(1e-5))) + pad
                A = I1p[Y - hp:Y + hp, X - hp:X + hp]
                B = I1p[Y - hp:Y + hp, X - hp - 1:X + hp - 1]
                Cc = I1p[Y - hp - 1:Y + hp - 1, X - hp:X + hp]
                D = I1p[Y - hp - 1:Y + hp - 1, X - hp - 1:X + hp - 1]
                r = (((w3 * A + w2 * B) + w1 * Cc) + w0 * D).reshape(-1).astype(f32)
                if norm:
                    r = r - eigen_sum(r) / f32(ps * ps)
                return r

            if not oob(sx, sy):
                r = warp(sx, sy)
                counter = 0
                while True:
                    counter += 1
                    b0 = eigen_sum(gdx * r)
                    b1 = eigen_sum(gdy * r)
                    if bt0 is not None:
                        b0, b1 = b0 - bt0, b1 - bt1
                    d0, d1 = lu_solve(h00, h01, h10, h11, b0, b1)
                    u0, u1 = u0 - d0, u1 - d1
                    qx, qy = rx + u0, ry + u1
                    ex, ey = sx - qx, sy - qy
                    nrm = np.sqrt(ex * ex + ey * ey)
                    if nrm > thr or oob(qx, qy) or nrm != nrm:
                        u0, u1 = iu, iv
                        break
                    if counter > it:
                        break
                    r = warp(qx, qy)
            us[pid] = (u0, u1)
    return us, (npw, nph, offw, offh)


def densify(us, geom, W, H, ps, st):
    npw, nph, offw, offh = geom
    f = np.zeros((H, W, 2), f32)
    w = np.zeros((H, W), f32)
    hp = ps // 2
    for gx in range(npw):
        for gy in range(nph):
            u = us[gx * nph + gy] * f32(0.5)
            rx, ry = gx * st + offw, gy * st + offh
            x0, x1 = max(rx - hp, 0), min(rx + hp, W)
            y0, y1 = max(ry - hp, 0), min(ry + hp, H)
            w[y0:y1, x0:x1] = w[y0:y1, x0:x1] + f32(0.5)
            f[y0:y1, x0:x1] = f[y0:y1, x0:x1] + u
    m = w > 0
    f[m] = f[m] / w[m][:, None]
    return f


def bilinear_replicate(I, X, Y):
    """I sampled at float32 arrays (X, Y): bilinear, replicate border, the
    position clamped to [-1, W] x [-1, H] first."""
    H, W = I.shape
    X = np.minimum(np.maximum(X, f32(-1)), f32(W)).astype(f32)
    Y = np.minimum(np.maximum(Y, f32(-1)), f32(H)).astype(f32)
    fx0, fy0 = np.floor(X), np.floor(Y)
    xa, ya = fx0.astype(np.int64), fy0.astype(np.int64)
    fx, fy = X - fx0, Y - fy0
    c0, c1 = np.clip(xa, 0, W - 1), np.clip(xa + 1, 0, W - 1)
    r0, r1 = np.clip(ya, 0, H - 1), np.clip(ya + 1, 0, H - 1)
    top = (f32(1) - fx) * I[r0, c0] + fx * I[r0, c1]
    bot = (f32(1) - fx) * I[r1, c0] + fx * I[r1, c1]
    return ((f32(1) - fy) * top + fy * bot).astype(f32)


def densify_paper(us, geom, I0, I1, W, H, ps, st):
    """Paper-mode densification: votes weighted by
    1 / max(1, |I1(x + u) - I0(x)|), patch-id order; I0/I1 unpadded level images."""
    npw, nph, offw, offh = geom
    f = np.zeros((H, W, 2), f32)
    w = np.zeros((H, W), f32)
    hp = ps // 2
    for gx in range(npw):
        for gy in range(nph):
            u = us[gx * nph + gy]
            rx, ry = gx * st + offw, gy * st + offh
            x0, x1 = max(rx - hp, 0), min(rx + hp, W)
            y0, y1 = max(ry - hp, 0), min(ry + hp, H)
            yy, xx = np.mgrid[y0:y1, x0:x1]
            d = bilinear_replicate(I1, xx.astype(f32) + u[0], yy.astype(f32) + u[1]) - I0[y0:y1, x0:x1]
            c = (f32(1) / np.maximum(f32(1), np.abs(d))).astype(f32)
            w[y0:y1, x0:x1] = w[y0:y1, x0:x1] + c
            f[y0:y1, x0:x1, 0] = f[y0:y1, x0:x1, 0] + c * u[0]
            f[y0:y1, x0:x1, 1] = f[y0:y1, x0:x1, 1] + c * u[1]
    m = w > 0
    f[m] = f[m] / w[m][:, None]
    return f


def atan2_dis(y, x):
    """The float atan2 restatement both the oracle and the kernel use (ARM
    optimized-routines atanf polynomial after reduction to [0, 1])."""
    f32 = np.float32
    y = np.asarray(y, f32)
    x = np.asarray(x, f32)
    ax, ay = np.abs(x), np.abs(y)
    mx, mn = np.maximum(ax, ay), np.minimum(ax, ay)
    with np.errstate(invalid="ignore", divide="ignore"):
        t = np.where(mx > 0, mn / np.where(mx > 0, mx, f32(1)), f32(0)).astype(f32)
    z = t * t
    p = f32(float.fromhex("0x1.01fd88p-8"))
    for c in ("-0x1.4c3c60p-6", "0x1.93a2c0p-5", "-0x1.491f0ep-4", "0x1.bd7368p-4", "-0x1.24051ep-3",
              "0x1.99935ep-3", "-0x1.55555p-2"):
        p = p * z + f32(float.fromhex(c))
    r = t + (t * z) * p
    r = np.where(ay > ax, f32(1.57079637) - r, r)
    r = np.where((x < 0) | ((x == 0) & np.signbit(x)), f32(3.14159274) - r, r)
    return np.where(np.signbit(y), -r, r).astype(f32)


def flow_color(flow, maxmotion=-1.0):
    """Vectorised float32 restatement of draw_optical_flow / compute_color
    (src/color_coding.cpp:13-117), independent of the C oracle."""
    f32 = np.float32
    wheel = []
    for i in range(15):
        wheel.append((255, 255 * i // 15, 0))
    for i in range(6):
        wheel.append((255 - 255 * i // 6, 255, 0))
    for i in range(4):
        wheel.append((0, 255, 255 * i // 4))
    for i in range(11):
        wheel.append((0, 255 - 255 * i // 11, 255))
    for i in range(13):
        wheel.append((255 * i // 13, 0, 255))
    for i in range(6):
        wheel.append((255, 0, 255 - 255 * i // 6))
    wheel = np.array(wheel, np.int64)
    ncols = len(wheel)
    x = flow[..., 0].astype(f32)
    y = flow[..., 1].astype(f32)
    with np.errstate(invalid="ignore", over="ignore"):
        ok = ~np.isnan(x) & ~np.isnan(y) & (np.abs(x) < f32(1e9)) & (np.abs(y) < f32(1e9))
        if maxmotion <= 0:
            r = np.sqrt(x[ok] * x[ok] + y[ok] * y[ok])
            maxrad = max(f32(1), r.max() if r.size else f32(1))
        else:
            maxrad = f32(maxmotion)
        fx = np.where(ok, x, f32(0)) / f32(maxrad)
        fy = np.where(ok, y, f32(0)) / f32(maxrad)
        rad = np.sqrt(fx * fx + fy * fy)
        a = atan2_dis(-fy, -fx) / f32(3.14159274)
        fk = (a + f32(1)) / f32(2) * f32(ncols - 1)
        k0 = fk.astype(np.int64)
        k1 = (k0 + 1) % ncols
        fr = fk - k0.astype(f32)
        out = np.zeros(flow.shape[:-1] + (3,), np.uint8)
        for b in range(3):
            c0 = wheel[k0, b].astype(f32) / f32(255)
            c1 = wheel[k1, b].astype(f32) / f32(255)
            col = (f32(1) - fr) * c0 + fr * c1
            col = np.where(rad <= f32(1), f32(1) - rad * (f32(1) - col), col * f32(0.75))
            out[..., 2 - b] = np.where(ok, (f32(255) * col).astype(np.int64), 0).astype(np.uint8)
    return out
