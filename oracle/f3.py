"""TEST INFRASTRUCTURE ONLY -- numpy oracle for SURVEY.md §8 f3, deftet_sparse_render
(kaolin/render/mesh/deftet.py:269-330 + deftet_cuda.cu:31-190):

  * ``deftet_forward(px, ranges, fvz, fvi, feat, knum, eps)`` -> (interp, face_idx, weights)
      per pixel, faces in index order: half-open box of the corner min / max (deftet.py:287-289,
      deftet_cuda.cu:114-126), eps-normalised barycentric weights with copysignf(float eps,
      norm) (:128-147), all three >= 0, depth w0*az + w1*bz + w2*cz in [min, max) (:150-160);
      the first knum hits by face index (:165-183), then sorted by depth descending (deftet.py:
      300-303 -- a stable sort here; the reference's torch.argsort is not stable, so tied depths
      are unpinned), w2 = (face != -1) - (w0 + w1) (:304), features w0*f0 + w1*f1 + w2*f2 (:305-313).
  * the backward is ``oracle.rasterize_backward`` on the (pixel, slot) samples as a P x knum image
    (deftet_cuda.cu:238-402 is rasterization_cuda.cu:238-402's math).

Pinned by tests/test_oracle_f3.py against the reference's literals (test_deftet.py:118-135) and its
naive renderer's outputs (tests/golden/deftet.npz, tests/golden/make_golden_f3.py).
"""
import numpy as np


def deftet_forward_raw(px, ranges, fvz, fvi, bbox, knum, eps=1e-8):
    """The reference's op form (deftet.cpp:48-106, deftet_cuda.cu:31-190): the caller's boxes
    bbox (B, F, 4) = (xmin, ymin, xmax, ymax) for the half-open test, and per pixel the first knum
    hits in face-index order, unsorted -> face_idx (-1), pixel_depths (-inf), w0 (0), w1 (0)."""
    B, P = px.shape[:2]
    face_idx = np.full((B, P, knum), -1, np.int64)
    depths = np.full((B, P, knum), -np.inf, fvi.dtype)
    w0o = np.zeros((B, P, knum), fvi.dtype)
    w1o = np.zeros((B, P, knum), fvi.dtype)
    for b in range(B):
        hit, depth, w0, w1, _ = _hits(px[b], ranges[b], fvz[b], fvi[b], eps, bbox[b])
        for p in range(P):
            fs = np.nonzero(hit[p])[0][:knum]
            n = fs.size
            face_idx[b, p, :n] = fs
            depths[b, p, :n] = depth[p, fs]
            w0o[b, p, :n] = w0[p, fs]
            w1o[b, p, :n] = w1[p, fs]
    return face_idx, depths, w0o, w1o


def _hits(px, ranges, fvz, v, eps, bbox=None):
    """(P, F) hit mask, depth, w0, w1, w2 of one view (deftet_cuda.cu:114-160)."""
    dt = v.dtype.type
    eps32 = np.float32(eps)
    with np.errstate(invalid='ignore', divide='ignore', over='ignore'):
        ax, ay, bx, by, cx, cy = (v[:, i // 2, i % 2][None, :] for i in range(6))
        if bbox is None:
            xmin, xmax = v[:, :, 0].min(axis=1)[None], v[:, :, 0].max(axis=1)[None]
            ymin, ymax = v[:, :, 1].min(axis=1)[None], v[:, :, 1].max(axis=1)[None]
        else:
            xmin, ymin, xmax, ymax = (bbox[None, :, i] for i in range(4))
        x0 = px[:, 0][:, None]
        y0 = px[:, 1][:, None]
        inbox = (x0 >= xmin) & (x0 < xmax) & (y0 >= ymin) & (y0 < ymax)
        aex, aey, bex, bey = ax - x0, ay - y0, bx - x0, by - y0
        cex, cey = cx - x0, cy - y0
        w0_ = bex * cey - bey * cex
        w1_ = cex * aey - cey * aex
        w2_ = aex * bey - aey * bex
        norm = w0_ + w1_ + w2_
        ne = np.copysign(eps32, norm.astype(np.float32)).astype(dt)
        w0 = w0_ / (norm + ne)
        w1 = w1_ / (norm + ne)
        w2 = w2_ / (norm + ne)
        depth = w0 * fvz[None, :, 0] + w1 * fvz[None, :, 1] + w2 * fvz[None, :, 2]
        hit = inbox & (w0 >= 0) & (w1 >= 0) & (w2 >= 0) & \
            (depth < ranges[:, 1][:, None]) & (depth >= ranges[:, 0][:, None])
    return hit, depth, w0, w1, w2


def deftet_forward(px, ranges, fvz, fvi, feat, knum, eps=1e-8):
    dt = fvi.dtype.type
    B, P = px.shape[:2]
    F, D = fvi.shape[1], feat.shape[-1]
    eps32 = np.float32(eps)
    interp = np.zeros((B, P, knum, D), fvi.dtype)
    face_idx = np.full((B, P, knum), -1, np.int64)
    weights = np.zeros((B, P, knum, 3), fvi.dtype)
    with np.errstate(invalid='ignore', divide='ignore', over='ignore'):
        for b in range(B):
            v = fvi[b]
            ax, ay, bx, by, cx, cy = (v[:, i // 2, i % 2][None, :] for i in range(6))
            xmin, xmax = v[:, :, 0].min(axis=1)[None], v[:, :, 0].max(axis=1)[None]
            ymin, ymax = v[:, :, 1].min(axis=1)[None], v[:, :, 1].max(axis=1)[None]
            x0 = px[b, :, 0][:, None]
            y0 = px[b, :, 1][:, None]
            inbox = (x0 >= xmin) & (x0 < xmax) & (y0 >= ymin) & (y0 < ymax)
            aex, aey, bex, bey = ax - x0, ay - y0, bx - x0, by - y0
            cex, cey = cx - x0, cy - y0
            w0_ = bex * cey - bey * cex
            w1_ = cex * aey - cey * aex
            w2_ = aex * bey - aey * bex
            norm = w0_ + w1_ + w2_
            ne = np.copysign(eps32, norm.astype(np.float32)).astype(dt)
            w0 = w0_ / (norm + ne)
            w1 = w1_ / (norm + ne)
            w2 = w2_ / (norm + ne)
            z = fvz[b]
            depth = w0 * z[None, :, 0] + w1 * z[None, :, 1] + w2 * z[None, :, 2]
            hit = inbox & (w0 >= 0) & (w1 >= 0) & (w2 >= 0) & \
                (depth < ranges[b, :, 1][:, None]) & (depth >= ranges[b, :, 0][:, None])
            for p in range(P):
                fs = np.nonzero(hit[p])[0][:knum]
                if fs.size == 0:
                    continue
                order = np.argsort(-depth[p, fs], kind='stable')
                fs = fs[order]
                n = fs.size
                a0, a1 = w0[p, fs], w1[p, fs]
                a2 = dt(1) - (a0 + a1)
                face_idx[b, p, :n] = fs
                weights[b, p, :n] = np.stack([a0, a1, a2], axis=-1)
                c = feat[b, fs]  # (n, 3, D)
                interp[b, p, :n] = a0[:, None] * c[:, 0] + a1[:, None] * c[:, 1] + \
                    a2[:, None] * c[:, 2]
    return interp, face_idx, weights
