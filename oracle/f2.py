"""TEST INFRASTRUCTURE ONLY -- numpy oracle for SURVEY.md §8 f2 (the steps either side of the
DIB-R path in the training loop, examples/tutorial/ian_dibr.py:248-265):

  * ``mask_iou`` / ``mask_iou_backward``   <- kaolin/metrics/render.py:18-40 and its torch
    autograd (MulBackward, SumBackward, DivBackward, MeanBackward, RsubBackward);
  * ``texture_mapping`` / ``texture_mapping_backward``  <- kaolin/render/mesh/utils.py:23-76:
    clamp, affine map to [-1, 1], y flip, then ``grid_sample(align_corners=False,
    padding_mode='border')`` restated from ATen's grid_sampler_2d (the source-index / border-clip
    / nearest / bilinear formulas and their backward, including clip_coordinates_set_grad).

Only tests/ (and the smoke / cpu_baseline legs) use this module.  Pinned against the reference's
own test literals and against the reference functions run on seeded inputs
(tests/golden/f2.npz, written by tests/golden/make_golden_f2.py).
"""
import numpy as np


def mask_iou(lhs, rhs):
    """render.py:32-41; sums in float64 (the reference's fp32 sums differ by rounding only)."""
    dt = lhs.dtype.type
    B = lhs.shape[0]
    mul = lhs * rhs
    add = lhs + rhs
    up = np.sum(mul.reshape(B, -1).astype(np.float64), axis=1).astype(dt)
    down = np.sum((add - mul).reshape(B, -1).astype(np.float64), axis=1).astype(dt)
    iou = up / (down + dt(1e-10))
    loss = dt(1.0) - dt(np.sum(iou, dtype=dt) / dt(B))
    return loss, np.stack([up, down], axis=1)


def mask_iou_backward(grad, lhs, rhs, stats):
    dt = lhs.dtype.type
    B = lhs.shape[0]
    gi = -(dt(grad) / dt(B))
    U = stats[:, 0].reshape(B, 1, 1)
    Dp = stats[:, 1].reshape(B, 1, 1) + dt(1e-10)
    gu = gi / Dp
    gd = -gi * U / (Dp * Dp)
    gm = gu - gd
    return gm * rhs + gd, gm * lhs + gd


def _source(g, size):
    """grid_sampler_compute_source_index(_set_grad), align_corners=False, border padding."""
    dt = g.dtype.type
    x = ((g + dt(1)) * dt(size) - dt(1)) / dt(2)
    mult = np.full_like(x, dt(size) / dt(2))
    lo = x <= 0
    hi = x >= size - 1
    mult[lo | hi] = 0
    x = np.where(lo, dt(0), np.where(hi, dt(size - 1), x))
    return x, mult


def _coords(uv, Wt, Ht):
    dt = uv.dtype.type
    u, v = uv[..., 0], uv[..., 1]
    uc = np.clip(u, dt(0), dt(1))
    vc = np.clip(v, dt(0), dt(1))
    gx = uc * dt(2) - dt(1)
    gy = -(vc * dt(2) - dt(1))
    ix, mx = _source(gx, Wt)
    iy, my = _source(gy, Ht)
    cu = (u >= 0) & (u <= 1)
    cv = (v >= 0) & (v <= 1)
    return ix, iy, mx, my, cu, cv


def _taps(ix, iy, Wt, Ht):
    x0 = np.floor(ix).astype(np.int64)
    y0 = np.floor(iy).astype(np.int64)
    x1, y1 = x0 + 1, y0 + 1
    dt = ix.dtype.type
    ex, wx = x1.astype(dt) - ix, ix - x0.astype(dt)
    ey, wy = y1.astype(dt) - iy, iy - y0.astype(dt)
    taps = [(x0, y0, ex * ey), (x1, y0, wx * ey), (x0, y1, ex * wy), (x1, y1, wx * wy)]
    return [(x, y, w, (x >= 0) & (x < Wt) & (y >= 0) & (y < Ht)) for x, y, w in taps], \
        (ex, wx, ey, wy)


def texture_mapping(uv, tex, mode):
    """uv (B, ..., 2), tex (Bt, C, Ht, Wt), Bt in {1, B} -> (B, ..., C)."""
    B = uv.shape[0]
    C, Ht, Wt = tex.shape[1:]
    flat = uv.reshape(B, -1, 2)
    ix, iy, *_ = _coords(flat, Wt, Ht)
    texb = np.broadcast_to(tex, (B, C, Ht, Wt))
    bidx = np.arange(B).reshape(B, 1)
    out = np.zeros((B, flat.shape[1], C), dtype=tex.dtype)
    if mode == 'nearest':
        x = np.rint(ix).astype(np.int64)
        y = np.rint(iy).astype(np.int64)
        ok = (x >= 0) & (x < Wt) & (y >= 0) & (y < Ht)
        for c in range(C):
            out[..., c] = np.where(ok, texb[bidx, c, np.clip(y, 0, Ht - 1),
                                            np.clip(x, 0, Wt - 1)], 0)
    else:
        taps, _ = _taps(ix, iy, Wt, Ht)
        for c in range(C):
            acc = np.zeros(ix.shape, dtype=tex.dtype)
            for x, y, w, ok in taps:
                v = texb[bidx, c, np.clip(y, 0, Ht - 1), np.clip(x, 0, Wt - 1)]
                acc = np.where(ok, acc + v * w, acc)
            out[..., c] = acc
    return out.reshape(*uv.shape[:-1], C)


def texture_mapping_backward(grad_out, uv, tex, mode):
    """(grad_uv, grad_tex) of texture_mapping; grad_tex has tex's shape (summed over views
    when tex has batch 1)."""
    B = uv.shape[0]
    C, Ht, Wt = tex.shape[1:]
    dt = tex.dtype.type
    flat = uv.reshape(B, -1, 2)
    go = grad_out.reshape(B, -1, C)
    ix, iy, mx, my, cu, cv = _coords(flat, Wt, Ht)
    texb = np.broadcast_to(tex, (B, C, Ht, Wt))
    gt = np.zeros((B, C, Ht, Wt), dtype=np.float64)
    bidx = np.broadcast_to(np.arange(B).reshape(B, 1), ix.shape)
    guv = np.zeros(flat.shape, dtype=tex.dtype)
    if mode == 'nearest':
        x = np.rint(ix).astype(np.int64)
        y = np.rint(iy).astype(np.int64)
        ok = (x >= 0) & (x < Wt) & (y >= 0) & (y < Ht)
        for c in range(C):
            np.add.at(gt, (bidx[ok], c, y[ok], x[ok]), go[..., c][ok])
    else:
        taps, (ex, wx, ey, wy) = _taps(ix, iy, Wt, Ht)
        gix = np.zeros(ix.shape, dtype=tex.dtype)
        giy = np.zeros(ix.shape, dtype=tex.dtype)
        # d(weight)/d(ix), d(weight)/d(iy) per tap (nw, ne, sw, se): the ATen backward's terms
        dxs = [(-1, ey), (1, ey), (-1, wy), (1, wy)]
        dys = [(-1, ex), (-1, wx), (1, ex), (1, wx)]
        for c in range(C):
            g = go[..., c]
            for (x, y, w, ok), (sx, fx), (sy, fy) in zip(taps, dxs, dys):
                xc, yc = np.clip(x, 0, Wt - 1), np.clip(y, 0, Ht - 1)
                np.add.at(gt, (bidx[ok], c, yc[ok], xc[ok]), (w * g)[ok])
                v = texb[bidx, c, yc, xc]
                gix = np.where(ok, gix + dt(sx) * (v * fx * g), gix)
                giy = np.where(ok, giy + dt(sy) * (v * fy * g), giy)
        guv[..., 0] = np.where(cu, (mx * gix) * dt(2), 0)
        guv[..., 1] = np.where(cv, -(my * giy) * dt(2), 0)
    if tex.shape[0] == 1 and B > 1:
        gt = gt.sum(axis=0, keepdims=True)
    return guv.reshape(uv.shape), gt.astype(tex.dtype)
