"""Synthetic DIB-R workloads and the plain-PyTorch camera / mesh helpers around
the hot path (harness, not accelerated):

  prepare_vertices  <- kaolin/render/mesh/utils.py:128-175
  perspective_camera / generate_perspective_projection / generate_transformation_matrix
                    <- kaolin/render/camera/legacy.py:85-158
  index_vertices_by_faces <- kaolin/ops/mesh/mesh.py:24-45
  face_normals      <- kaolin/ops/mesh/trianglemesh.py:313-336

Meshes are deterministic (CPU torch.Generator), no downloads.
"""
import math

import torch


def uv_sphere(n_lon, n_lat, seed=0, dtype=torch.float32):
    """2 poles + (n_lat-1) rings x n_lon vertices, radius 1 + 0.05 N(0,1); fan triangles at the
    poles (no degenerate faces); F = 2 n_lon (n_lat-1), outward CCW winding.
    Returns (vertices (V,3), faces (F,3) int64, face_uvs (F,3,2))."""
    g = torch.Generator().manual_seed(seed)
    theta = torch.arange(1, n_lat, dtype=torch.float64) * (math.pi / n_lat)  # polar angle
    phi = torch.arange(n_lon, dtype=torch.float64) * (2 * math.pi / n_lon)
    st, ct = torch.sin(theta)[:, None], torch.cos(theta)[:, None]
    ring = torch.stack([st * torch.cos(phi)[None], ct.expand(-1, n_lon),
                        -st * torch.sin(phi)[None]], dim=-1).reshape(-1, 3)
    verts = torch.cat([torch.tensor([[0., 1., 0.]], dtype=torch.float64), ring,
                       torch.tensor([[0., -1., 0.]], dtype=torch.float64)], dim=0)
    radius = 1. + 0.05 * torch.randn(verts.shape[0], 1, generator=g, dtype=torch.float64)
    verts = verts * radius
    V = verts.shape[0]
    top, bot = 0, V - 1

    def rid(i, j):  # ring i (0..n_lat-2), lon j
        return 1 + i * n_lon + (j % n_lon)

    faces = []
    for j in range(n_lon):
        faces.append((top, rid(0, j), rid(0, j + 1)))
    for i in range(n_lat - 2):
        for j in range(n_lon):
            a, b, c, d = rid(i, j), rid(i + 1, j), rid(i + 1, j + 1), rid(i, j + 1)
            faces.append((a, b, c))
            faces.append((a, c, d))
    for j in range(n_lon):
        faces.append((bot, rid(n_lat - 2, j + 1), rid(n_lat - 2, j)))
    faces = torch.tensor(faces, dtype=torch.long)
    # uv = (phi / 2pi, theta / pi) per face corner
    vu = torch.zeros(V, 2, dtype=torch.float64)
    vu[1:-1, 0] = (phi[None, :].expand(n_lat - 1, -1).reshape(-1)) / (2 * math.pi)
    vu[1:-1, 1] = (theta[:, None].expand(-1, n_lon).reshape(-1)) / math.pi
    vu[-1, 1] = 1.
    face_uvs = vu[faces]
    return verts.to(dtype), faces, face_uvs.to(dtype)


def soup(num_faces, seed=3, dtype=torch.float32, batch=1):
    """Clustered random triangle soup: centres ~ N(0, 0.25^2) clipped to
    [-0.95, 0.95]^2, corners centre + U(-s, s)^2 with s = 2/sqrt(F), z = U(-4,-2) per face +
    U(-0.05, 0.05) per corner, random winding.  Returns (fvz (B,F,3), fvi (B,F,3,2),
    normals_z (B,F))."""
    g = torch.Generator().manual_seed(seed)
    s = 2. / math.sqrt(num_faces)
    c = (torch.randn(batch, num_faces, 1, 2, generator=g, dtype=torch.float64) * 0.25)
    c = c.clamp(-0.95, 0.95)
    fvi = c + (torch.rand(batch, num_faces, 3, 2, generator=g, dtype=torch.float64) * 2 - 1) * s
    fvz = (-2. - 2. * torch.rand(batch, num_faces, 1, generator=g, dtype=torch.float64)) + \
        (torch.rand(batch, num_faces, 3, generator=g, dtype=torch.float64) - 0.5) * 0.1
    e1 = fvi[..., 1, :] - fvi[..., 0, :]
    e2 = fvi[..., 2, :] - fvi[..., 0, :]
    nz = e1[..., 0] * e2[..., 1] - e1[..., 1] * e2[..., 0]
    return fvz.to(dtype), fvi.to(dtype), nz.to(dtype)


# --------------------------------------------------------------------------------------------
# camera / mesh helpers (restated; legacy.py / mesh.py / trianglemesh.py / utils.py)
# --------------------------------------------------------------------------------------------
def generate_perspective_projection(fovyangle, ratio=1.0, dtype=torch.float32):
    tanfov = math.tan(fovyangle / 2.0)
    return torch.tensor([[1.0 / (ratio * tanfov)], [1.0 / tanfov], [-1]], dtype=dtype)


def generate_transformation_matrix(camera_position, look_at, camera_up_direction):
    z_axis = camera_position - look_at
    z_axis = z_axis / z_axis.norm(dim=1, keepdim=True)
    up = camera_up_direction
    if up.shape[0] < z_axis.shape[0]:
        up = up.repeat(z_axis.shape[0], 1)
    x_axis = torch.cross(up, z_axis, dim=1)
    x_axis = x_axis / x_axis.norm(dim=1, keepdim=True)
    y_axis = torch.cross(z_axis, x_axis, dim=1)
    rot = torch.stack([x_axis, y_axis, z_axis], dim=2)
    trans = -camera_position.unsqueeze(1) @ rot
    return torch.cat([rot, trans], dim=1)


def perspective_camera(points, camera_proj):
    projected = points * camera_proj.view(-1, 1, 3)
    return projected[:, :, :2] / projected[:, :, 2:3]


def index_vertices_by_faces(vertices_features, faces):
    """(B, V, C) x (F, 3) -> (B, F, 3, C); its backward is the face->vertex scatter-add."""
    B = vertices_features.shape[0]
    return torch.index_select(vertices_features, 1, faces.reshape(-1)).reshape(
        B, faces.shape[0], faces.shape[1], vertices_features.shape[-1])


def face_normals(face_vertices, unit=False):
    e1 = face_vertices[:, :, 1] - face_vertices[:, :, 0]
    e2 = face_vertices[:, :, 2] - face_vertices[:, :, 0]
    n = torch.cross(e1, e2, dim=2)
    if unit:  # ops/mesh/trianglemesh.py:333-335 (length + 1e-10, not F.normalize)
        n = n / (n.norm(dim=2, keepdim=True) + 1e-10)
    return n


def prepare_vertices(vertices, faces, camera_proj, camera_transform):
    padded = torch.nn.functional.pad(vertices, (0, 1), mode='constant', value=1.)
    vertices_camera = padded @ camera_transform
    vertices_image = perspective_camera(vertices_camera, camera_proj)
    face_vertices_camera = index_vertices_by_faces(vertices_camera, faces)
    face_vertices_image = index_vertices_by_faces(vertices_image, faces)
    normals = face_normals(face_vertices_camera, unit=True)
    return face_vertices_camera, face_vertices_image, normals


def orbit_cameras(num_views, elevation=0.3, distance=3., first_view=0, total_views=None,
                  dtype=torch.float32):
    """Views b = first_view.. first_view+num_views-1 of `total_views` cameras at azimuth
    2*pi*b/total, given elevation / distance, looking at the origin, up (0,1,0)."""
    total = total_views or num_views
    b = torch.arange(first_view, first_view + num_views, dtype=torch.float64)
    az = 2 * math.pi * b / total
    pos = torch.stack([distance * math.cos(elevation) * torch.sin(az),
                       torch.full_like(az, distance * math.sin(elevation)),
                       distance * math.cos(elevation) * torch.cos(az)], dim=1)
    look = torch.zeros_like(pos)
    up = torch.tensor([[0., 1., 0.]], dtype=torch.float64)
    return generate_transformation_matrix(pos, look, up).to(dtype)


def sphere_views(n_lon, n_lat, height, width, batch, device, dtype=torch.float32, seed=0,
                 elevation=0.3, first_view=0, total_views=None):
    """A uv_sphere seen by `batch` orbit cameras, fovy pi/4.  Returns a dict with vertices, faces,
    face_uvs (B,F,3,2), the camera and the per-view DIB-R inputs (fvz, fvi, normals_z, feats)."""
    verts, faces, face_uvs = uv_sphere(n_lon, n_lat, seed, dtype)
    cam = orbit_cameras(batch, elevation, first_view=first_view, total_views=total_views,
                        dtype=dtype).to(device)
    proj = generate_perspective_projection(math.pi / 4, dtype=dtype).to(device)
    verts = verts.to(device)
    faces = faces.to(device)
    fvc, fvi, nrm = prepare_vertices(verts.unsqueeze(0).repeat(batch, 1, 1), faces, proj, cam)
    uvs = face_uvs.to(device).unsqueeze(0).repeat(batch, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1)
    return dict(vertices=verts, faces=faces, cam=cam, proj=proj, fvz=fvc[..., 2].contiguous(),
                fvi=fvi.contiguous(), normals_z=nrm[..., 2].contiguous(), feats=feats,
                height=height, width=width)


def view_grads(first_view, num_views, height, width, feat_dim, seed=1, dtype=torch.float32):
    """Upstream gradients of the bench step (g_feat ~ U(0,1), g_soft ~ U(0,1)),
    drawn per GLOBAL view index, so a view gets the same numbers however the views are sharded.
    Returns (g_feat (B, H, W, D), g_soft (B, H, W)) on the CPU."""
    gf, gs = [], []
    for v in range(first_view, first_view + num_views):
        g = torch.Generator().manual_seed(seed * 1000003 + 2 * v)
        gf.append(torch.rand((height, width, feat_dim), generator=g, dtype=dtype))
        g = torch.Generator().manual_seed(seed * 1000003 + 2 * v + 1)
        gs.append(torch.rand((height, width), generator=g, dtype=dtype))
    if not gf:
        return (torch.empty((0, height, width, feat_dim), dtype=dtype),
                torch.empty((0, height, width), dtype=dtype))
    return torch.stack(gf), torch.stack(gs)
