"""Texel-tile load of the texture_mapping backward at the bench_rows workload (diagnostic):
samples per 32 x 32 texel tile and per texel of the C3 render's uvs, per view.
python tools/tex_tile_hist.py   (GPU)
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaolin_amd import workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization, prepare_vertices  # noqa: E402

DEV = 'cuda'


def main():
    B, H, W, Ht, Wt, T = 8, 512, 512, 512, 512, 32
    verts, faces, face_uvs = workloads.uv_sphere(250, 101, seed=0)
    cams = workloads.orbit_cameras(B, 0.3).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    with torch.no_grad():
        fvc, fvi, nrm = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                         camera_transform=cams)
        uvs = face_uvs.to(DEV).unsqueeze(0).repeat(B, 1, 1, 1)
        interp, _, face_idx = dibr_rasterization(H, W, fvc[..., 2], fvi, uvs, nrm[..., 2])
    out = {}
    for b in range(B):
        m = face_idx[b] >= 0
        uv = interp[b][m].clamp(0, 1)
        ix = torch.floor(uv[:, 0] * Wt - 0.5).long().clamp(0, Wt - 1)
        iy = torch.floor((1 - uv[:, 1]) * Ht - 0.5).long().clamp(0, Ht - 1)
        tile = torch.bincount((iy // T) * (Wt // T) + ix // T, minlength=(Ht // T) * (Wt // T))
        texel = torch.bincount(iy * Wt + ix, minlength=Ht * Wt)
        nz = tile[tile > 0].float()
        out[b] = {'samples': int(m.sum()), 'tiles_hit': int((tile > 0).sum()),
                  'tile_max': int(tile.max()), 'tile_mean': round(float(nz.mean()), 1),
                  'tile_p99': int(torch.quantile(nz, 0.99)), 'texel_max': int(texel.max()),
                  'texels_hit': int((texel > 0).sum())}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
