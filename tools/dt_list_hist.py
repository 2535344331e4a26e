"""Cell-list lengths of the DefTet forward at the bench_rows workload (diagnostic): per pixel, the
length of its cell's face list (kd_dt_bin's 64 x 64 grid over [-1, 1]^2) and the walk steps of
64 faces it takes.   python tools/dt_list_hist.py   (GPU)
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaolin_amd import workloads  # noqa: E402
from kaolin_amd.render.mesh import prepare_vertices  # noqa: E402

DEV = 'cuda'


def main():
    H = W = 512
    G = 64
    verts, faces, _ = workloads.uv_sphere(250, 101, seed=0)
    cams = workloads.orbit_cameras(8, 0.3).to(DEV)[:1]
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    with torch.no_grad():
        _, fvi, _ = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                     camera_transform=cams)
    v = fvi[0]
    cell = lambda x: ((x + 1) * (G // 2)).clamp(0, G - 1).floor().long()  # noqa: E731
    cx0, cx1 = cell(v[:, :, 0].min(1).values), cell(v[:, :, 0].max(1).values)
    cy0, cy1 = cell(v[:, :, 1].min(1).values), cell(v[:, :, 1].max(1).values)
    cnt = torch.zeros(G * G, device=DEV, dtype=torch.long)
    span = int(max((cx1 - cx0).max(), (cy1 - cy0).max())) + 1
    for dy in range(span):
        for dx in range(span):
            m = (cx0 + dx <= cx1) & (cy0 + dy <= cy1)
            cnt.index_add_(0, ((cy0 + dy) * G + cx0 + dx)[m], torch.ones_like(cx0[m]))
    xs = (2 * torch.arange(W, device=DEV) + 1 - W) / W
    ys = (H - 2 * torch.arange(H, device=DEV) - 1.) / H
    pc = (cell(ys).reshape(-1, 1) * G + cell(xs).reshape(1, -1)).reshape(-1)
    nl = cnt[pc].float()
    steps = torch.ceil(nl / 64)
    box = (cx1 - cx0 + 1) * (cy1 - cy0 + 1)
    print(json.dumps({'faces': int(v.shape[0]), 'cells_per_face_mean': float(box.float().mean()),
                      'cells_per_face_max': int(box.max()), 'nl_mean': float(nl.mean()),
                      'nl_p50': float(nl.median()), 'nl_max': float(nl.max()),
                      'steps_mean': float(steps.mean()), 'px_nl_gt_64': float((nl > 64).float().mean())}))


if __name__ == '__main__':
    main()
