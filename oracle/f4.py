"""TEST INFRASTRUCTURE ONLY -- numpy oracle for SURVEY.md §8 f4, the nvdiffrast_fwd data path
(kaolin/render/mesh/rasterization.py:145-241) after the external forward:

  * ``rast_interpolate(rast, feat)`` -> (interp, face_idx, weights):
      face_idx = rast[..., 3].long() - 1                                  (:207)
      weights  = cat(rast[..., :2], 1 - sum(rast[..., :2]))               (:213-216)
      interp   = nvdiff.interpolate(features, rast, tri)[0] with tri = arange(3F).reshape(F, 3)
                 (:204-206): u * a0 + v * a1 + w2 * a2 of the triangle's corner attributes, 0
                 on empty pixels.
The backward is rasterize_backward on (face_idx, weights) -- oracle.rasterize_backward.

nvdiffrast is a dependency the reference imports optionally (rasterization.py:24-29) and is not
present here (no version pinned by the reference): its interpolation is restated from its
published definition (barycentric interpolation with b2 = 1 - b0 - b1), with b2 written as the
reference's own weights expression 1 - (u + v); that choice is documented in DESIGN.md.
Parity for this row is pinned through the reference's rasterize goldens: a rast buffer holding the
reference forward's barycentrics reproduces its features (tests/test_oracle_f4.py).
"""
import numpy as np


def rast_interpolate(rast, feat):
    dt = feat.dtype.type
    B, H, W, _ = rast.shape
    F, D = feat.shape[1], feat.shape[3]
    rast = rast.astype(feat.dtype)
    u, v, tid = rast[..., 0], rast[..., 1], rast[..., 3]
    w2 = dt(1) - (u + v)
    weights = np.stack([u, v, w2], axis=-1)
    ok = (tid >= 1) & (tid <= F)
    face_idx = np.where(ok, np.trunc(np.where(ok, tid, 1)).astype(np.int64) - 1, -1)
    f = np.clip(face_idx, 0, max(F - 1, 0))
    bidx = np.arange(B).reshape(B, 1, 1)
    a = feat[bidx, f]  # (B, H, W, 3, D)
    interp = u[..., None] * a[..., 0, :] + v[..., None] * a[..., 1, :] + w2[..., None] * a[..., 2, :]
    interp = np.where(ok[..., None], interp, dt(0))
    return interp.astype(feat.dtype), face_idx, weights
