"""GPU parity for SURVEY.md §8 f2: mask_iou (kd_metrics.hip) and texture_mapping (kd_texture.hip)
against the oracle (oracle/f2.py), the reference's golden fixtures (tests/golden/f2.npz) and, at
full size, the reference's torch composition (kaolin/render/mesh/utils.py:64-76 and
kaolin/metrics/render.py:32-41 restated in torch, fp64).

Bars: texture_mapping forward and uv gradient bit-exact vs the oracle (same IEEE op sequence);
texture gradient (float atomics, any order) to rtol 1e-5 / atol 1e-6 (fp32), 1e-12 (fp64);
mask_iou (fp64 sums instead of the reference's fp32 sums) to rtol 1e-5 (fp32), 1e-12 (fp64).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import f2

pytestmark = pytest.mark.gpu

DEV = 'cuda'
DT = {'f32': torch.float32, 'f64': torch.float64}
MODES = ['nearest', 'bilinear']


@pytest.fixture(scope='module', autouse=True)
def _native():
    import kaolin_amd  # noqa: F401
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()


@pytest.fixture(scope='module')
def g():
    return load_golden('f2.npz')


def T(a, dt=None):
    t = torch.as_tensor(np.ascontiguousarray(a)).to(DEV)
    return t if dt is None else t.to(dt)


def N(t):
    return t.detach().cpu().numpy()


def tol(k):
    return dict(rtol=1e-5, atol=1e-6) if k == 'f32' else dict(rtol=1e-12, atol=1e-13)


def _native_loaded():
    from kaolin_amd import _lib
    return _lib._lib is not None


# ------------------------------------------------------------------------------------------
# mask_iou
# ------------------------------------------------------------------------------------------
def torch_mask_iou(l, r):
    """kaolin/metrics/render.py:32-41 restated in torch (the reference composition)."""
    B = l.shape[0]
    mul = l * r
    add = l + r
    up = torch.sum(mul.reshape(B, -1), dim=1)
    down = torch.sum((add - mul).reshape(B, -1), dim=1)
    return 1.0 - torch.mean(up / (down + 1e-10))


@pytest.mark.parametrize('k', ['f32', 'f64'])
def test_mask_iou_reference_case(g, k):
    from kaolin_amd.metrics.render import mask_iou
    loss = mask_iou(T(g['t_lhs'], DT[k]), T(g['t_rhs'], DT[k]))
    assert loss.shape == ()
    assert torch.allclose(loss.cpu(), torch.tensor([0.3105], dtype=DT[k]))  # test_render.py:51
    np.testing.assert_allclose(N(loss), g[f't_iou_{k}'], **tol(k))
    assert _native_loaded()


@pytest.mark.parametrize('k', ['f32', 'f64'])
def test_mask_iou_golden_grads(g, k):
    from kaolin_amd.metrics.render import mask_iou
    l = T(g[f'r_iou_l_{k}']).requires_grad_(True)
    r = T(g[f'r_iou_r_{k}']).requires_grad_(True)
    loss = mask_iou(l, r)
    gl, gr = torch.autograd.grad(loss, [l, r], torch.tensor(0.75, dtype=DT[k], device=DEV))
    np.testing.assert_allclose(N(loss), g[f'r_iou_loss_{k}'], **tol(k))
    np.testing.assert_allclose(N(gl), g[f'r_iou_gl_{k}'], **tol(k))
    np.testing.assert_allclose(N(gr), g[f'r_iou_gr_{k}'], **tol(k))
    # and the oracle on the same inputs (bit-level formula, same fp64 sums up to order)
    lo, st = f2.mask_iou(g[f'r_iou_l_{k}'], g[f'r_iou_r_{k}'])
    ol, orr = f2.mask_iou_backward(0.75, g[f'r_iou_l_{k}'], g[f'r_iou_r_{k}'], st)
    np.testing.assert_allclose(N(loss), lo, **tol(k))
    np.testing.assert_allclose(N(gl), ol, **tol(k))
    np.testing.assert_allclose(N(gr), orr, **tol(k))


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('shape', [(1, 1, 1), (2, 3, 5), (300, 7, 9), (8, 512, 512),
                                   (3, 1021, 1023), (1, 2048, 2048)])
def test_mask_iou_sizes(k, shape):
    """Scalar and 16-byte paths, many views (finisher loops), full-size images."""
    from kaolin_amd.metrics.render import mask_iou
    gen = torch.Generator(device='cpu').manual_seed(sum(shape))
    l = torch.rand(shape, generator=gen, dtype=torch.float64)
    r = (torch.rand(shape, generator=gen, dtype=torch.float64) > 0.3).double()
    ref = torch_mask_iou(l, r)
    lt, rt = l.to(DEV, DT[k]).requires_grad_(True), r.to(DEV, DT[k]).requires_grad_(True)
    loss = mask_iou(lt, rt)
    loss.backward()
    lr, rr = l.clone().requires_grad_(True), r.clone().requires_grad_(True)
    torch_mask_iou(lr, rr).backward()
    t = dict(rtol=2e-5, atol=1e-6) if k == 'f32' else dict(rtol=1e-11, atol=1e-14)
    np.testing.assert_allclose(N(loss), ref.numpy(), **t)
    np.testing.assert_allclose(N(lt.grad), lr.grad.numpy(), **t)
    np.testing.assert_allclose(N(rt.grad), rr.grad.numpy(), **t)


def test_mask_iou_misaligned_and_one_sided():
    """Inputs that are views at an odd offset (scalar path) and a gradient for one input only."""
    from kaolin_amd.metrics.render import mask_iou
    gen = torch.Generator(device='cpu').manual_seed(5)
    lv = torch.rand((2 * 64 * 64 + 1,), generator=gen, dtype=torch.float64).to(DEV)[1:]
    lv = lv.reshape(2, 64, 64)  # misaligned by 8 bytes
    r = torch.rand((2, 64, 64), generator=gen, dtype=torch.float64).to(DEV).requires_grad_(True)
    loss = mask_iou(lv, r)
    loss.backward()
    ref_r = r.detach().cpu().clone().requires_grad_(True)
    ref = torch_mask_iou(lv.cpu(), ref_r)
    ref.backward()
    np.testing.assert_allclose(N(loss), ref.detach().numpy(), rtol=1e-12)
    np.testing.assert_allclose(N(r.grad), ref_r.grad.numpy(), rtol=1e-11, atol=1e-15)


def test_mask_iou_rejects_bad_input():
    from kaolin_amd.metrics.render import mask_iou
    with pytest.raises(RuntimeError):
        mask_iou(torch.zeros((2, 3, 3), device=DEV, dtype=torch.float16),
                 torch.zeros((2, 3, 3), device=DEV, dtype=torch.float16))
    with pytest.raises(RuntimeError):
        mask_iou(torch.zeros((2, 3, 3), device=DEV), torch.zeros((2, 3, 3)))


# ------------------------------------------------------------------------------------------
# texture_mapping
# ------------------------------------------------------------------------------------------
def torch_texture_mapping(uv, tex, mode):
    """kaolin/render/mesh/utils.py:59-76 restated in torch (the reference composition)."""
    B = uv.shape[0]
    C = tex.shape[1]
    t = uv.reshape(B, -1, 1, 2)
    t = torch.clamp(t, 0., 1.)
    t = t * 2 - 1
    t = torch.stack([t[..., 0], -t[..., 1]], dim=-1)
    r = torch.nn.functional.grid_sample(tex, t, mode=mode, align_corners=False,
                                        padding_mode='border')
    return r.permute(0, 2, 3, 1).reshape(B, *uv.shape[1:-1], C)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_reference_cases(g, k, mode):
    from kaolin_amd.render.mesh import texture_mapping
    for tname in ('tex1', 'tex3'):
        out = texture_mapping(T(g['t_sparse'], DT[k]), T(g[f't_{tname}'], DT[k]), mode=mode)
        assert out.shape == (2, 4, g[f't_{tname}'].shape[1])
        np.testing.assert_array_equal(N(out), g[f't_sparse_{tname}_{mode}_{k}'])
    out = texture_mapping(T(g['t_dense'], DT[k]), T(g['t_tex3'], DT[k]), mode=mode)
    np.testing.assert_array_equal(N(out), g[f't_dense_tex3_{mode}_{k}'])


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_golden_and_oracle(g, k, mode):
    from kaolin_amd.render.mesh import texture_mapping
    uv, tex, go = g[f'r_tex_uv_{k}'], g[f'r_tex_map_{k}'], g[f'r_tex_go_{k}']
    u, t = T(uv).requires_grad_(True), T(tex).requires_grad_(True)
    out = texture_mapping(u, t, mode=mode)
    gu, gt = torch.autograd.grad(out, [u, t], T(go))
    # reference outputs (torch CPU run of the reference function)
    np.testing.assert_allclose(N(out), g[f'r_tex_out_{mode}_{k}'], **tol(k))
    np.testing.assert_allclose(N(gt), g[f'r_tex_gmap_{mode}_{k}'], **tol(k))
    gtol = dict(rtol=1e-4, atol=2e-5) if k == 'f32' else tol(k)
    np.testing.assert_allclose(N(gu), g[f'r_tex_guv_{mode}_{k}'], **gtol)
    # oracle: forward and uv gradient are the same op sequence -> bit-exact
    np.testing.assert_array_equal(N(out), f2.texture_mapping(uv, tex, mode))
    ou, ot = f2.texture_mapping_backward(go, uv, tex, mode)
    np.testing.assert_array_equal(N(gu), ou)
    np.testing.assert_allclose(N(gt), ot, **tol(k))


@pytest.mark.parametrize('mode', MODES)
def test_texture_shared_map(g, mode):
    """Batch-1 texture shared by every view == the reference's repeat (gradient summed)."""
    from kaolin_amd.render.mesh import texture_mapping
    uv, tex, go = g['r_tex_uv_f32'], g['r_tex_map_f32'][:1], g['r_tex_go_f32']
    u = T(uv)
    t1 = T(tex).requires_grad_(True)
    out = texture_mapping(u, t1, mode=mode)
    out.backward(T(go))
    t2 = T(tex).requires_grad_(True)
    out2 = texture_mapping(u, t2.repeat(uv.shape[0], 1, 1, 1), mode=mode)
    out2.backward(T(go))
    np.testing.assert_array_equal(N(out), N(out2))
    np.testing.assert_allclose(N(t1.grad), N(t2.grad), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_full_size_vs_torch(k, mode):
    """C3 render size (8 x 512 x 512 uvs) into a 512 x 512 RGB texture (ian_dibr.py:38, 112),
    against the reference torch composition on the GPU."""
    from kaolin_amd.render.mesh import texture_mapping
    gen = torch.Generator(device='cpu').manual_seed(7)
    uv = (torch.rand((8, 512, 512, 2), generator=gen) * 1.1 - 0.05).to(DEV, DT[k])
    tex = torch.rand((8, 3, 512, 512), generator=gen).to(DEV, DT[k])
    go = torch.rand((8, 512, 512, 3), generator=gen).to(DEV, DT[k])
    u, t = uv.clone().requires_grad_(True), tex.clone().requires_grad_(True)
    out = texture_mapping(u, t, mode=mode)
    gu, gt = torch.autograd.grad(out, [u, t], go)
    u2, t2 = uv.clone().requires_grad_(True), tex.clone().requires_grad_(True)
    ref = torch_texture_mapping(u2, t2, mode)
    ru, rt = torch.autograd.grad(ref, [u2, t2], go, allow_unused=True)
    t = dict(rtol=1e-5, atol=1e-5) if k == 'f32' else dict(rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(N(out), N(ref), **t)
    np.testing.assert_allclose(N(gt), N(rt), **t)
    if mode == 'bilinear':
        gtol = dict(rtol=1e-3, atol=2e-3) if k == 'f32' else dict(rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(N(gu), N(ru), **gtol)
    else:
        assert float(gu.abs().max()) == 0.0


def test_texture_edge_cases():
    from kaolin_amd.render.mesh import texture_mapping
    tex = torch.rand((2, 1, 4, 5), device=DEV)
    # empty sample set
    out = texture_mapping(torch.zeros((2, 0, 2), device=DEV), tex, mode='bilinear')
    assert out.shape == (2, 0, 1)
    # 1x1 texture, NaN / inf / out-of-range uvs stay in range
    one = torch.rand((2, 3, 1, 1), device=DEV)
    uv = torch.tensor([[[float('nan'), 0.5], [float('inf'), -float('inf')], [-3., 7.]]] * 2,
                      device=DEV)
    for mode in MODES:
        out = texture_mapping(uv, one, mode=mode)
        assert torch.equal(out, one[:, :, 0, 0].unsqueeze(1).expand(2, 3, 3))
    with pytest.raises(RuntimeError):
        texture_mapping(torch.zeros((2, 4, 2), device=DEV), tex, mode='bicubic')
    with pytest.raises(RuntimeError):
        texture_mapping(torch.zeros((3, 4, 2), device=DEV), tex, mode='nearest')


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_coherent_uvs_vs_torch(k, mode):
    """Smooth uv fields (the LDS-summed texture gradient of 16 x 16 sample blocks) with a masked
    background (zero gradient, uv = 0), odd image sizes (partial blocks), a shared texture."""
    from kaolin_amd.render.mesh import texture_mapping
    gen = torch.Generator(device='cpu').manual_seed(11)
    B, h, w = 3, 77, 101
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h, dtype=torch.float64),
                            torch.linspace(0, 1, w, dtype=torch.float64), indexing='ij')
    uv = torch.stack([0.2 + 0.6 * xx + 0.05 * torch.sin(7 * yy),
                      0.1 + 0.7 * yy + 0.05 * torch.cos(5 * xx)], -1)
    uv = uv.unsqueeze(0).repeat(B, 1, 1, 1) + 0.01 * torch.rand((B, h, w, 2), generator=gen,
                                                               dtype=torch.float64)
    mask = ((xx - 0.5) ** 2 + (yy - 0.5) ** 2 < 0.16).unsqueeze(-1)
    uv = torch.where(mask, uv, torch.zeros_like(uv))
    go = torch.rand((B, h, w, 3), generator=gen, dtype=torch.float64) * mask
    for tb in (B, 1):
        tex = torch.rand((tb, 3, 64, 48), generator=gen, dtype=torch.float64)
        u, t = uv.to(DEV, DT[k]).requires_grad_(True), tex.to(DEV, DT[k]).requires_grad_(True)
        out = texture_mapping(u, t, mode=mode)
        gu, gt = torch.autograd.grad(out, [u, t], go.to(DEV, DT[k]))
        u2 = uv.clone().requires_grad_(True)
        t2 = tex.clone().requires_grad_(True)
        ref = torch_texture_mapping(u2, t2.expand(B, -1, -1, -1), mode)
        ru, rt = torch.autograd.grad(ref, [u2, t2], go, allow_unused=True)
        t_ = dict(rtol=1e-5, atol=1e-5) if k == 'f32' else dict(rtol=1e-11, atol=1e-11)
        if mode == 'nearest':
            # uvs on a linspace grid land on exact texel halves, where ATen's CPU kernel and the
            # restated formula may round the source index differently: check the oracle
            ou = uv.to(DT[k]).numpy()
            np.testing.assert_array_equal(N(out), f2.texture_mapping(ou, N(t), mode))
            _, ot = f2.texture_mapping_backward(go.to(DT[k]).numpy(), ou, N(t), mode)
            np.testing.assert_allclose(N(gt), ot, **t_)
            continue
        np.testing.assert_allclose(N(out), ref.detach().numpy(), **t_)
        np.testing.assert_allclose(N(gt), rt.numpy(), **t_)
        if mode == 'bilinear':
            gtol = dict(rtol=1e-3, atol=1e-3) if k == 'f32' else dict(rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(N(gu), ru.numpy(), **gtol)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_tiled_heavy_tiles_and_large_texture(k, mode):
    """The texel-tile backward's chunking: a magnified region where one 32 x 32 texel tile gets
    ~40k samples (40 chunks of 1024) next to a spread of samples, and a 2080 x 2080 texture
    (65 x 65 tiles, past the 4096-tile LDS table: the per-block kernel), against the torch
    composition."""
    from kaolin_amd.render.mesh import texture_mapping
    gen = torch.Generator(device='cpu').manual_seed(13)
    B = 2
    hot = 0.30 + 0.02 * torch.rand((B, 40000, 2), generator=gen, dtype=torch.float64)
    spread = torch.rand((B, 9000, 2), generator=gen, dtype=torch.float64)
    for hw, uv in ((96, torch.cat([hot, spread], 1)), (2080, spread)):
        tex = torch.rand((B, 3, hw, hw), generator=gen, dtype=torch.float64)
        go = torch.rand(uv.shape[:2] + (3,), generator=gen, dtype=torch.float64)
        u, t = uv.to(DEV, DT[k]).requires_grad_(True), tex.to(DEV, DT[k]).requires_grad_(True)
        gu, gt = torch.autograd.grad(texture_mapping(u, t, mode=mode), [u, t], go.to(DEV, DT[k]))
        # the reference in the same dtype (f32 uvs round to texels on their own)
        u2 = uv.to(DEV, DT[k]).requires_grad_(True)
        t2 = tex.to(DEV, DT[k]).requires_grad_(True)
        ref = torch_texture_mapping(u2, t2, mode)
        ru, rt = torch.autograd.grad(ref, [u2, t2], go.to(DEV, DT[k]), allow_unused=True)
        # f32: bilinear weights come from ix = ((g + 1) W - 1) / 2, whose ulp grows with the
        # texture width (~1.2e-4 at 2080); torch's kernel may contract it differently
        scale = float(rt.abs().max())
        tol = (dict(rtol=1e-4, atol=1e-5 * scale + 8 * hw * 2.0 ** -23) if k == 'f32'
               else dict(rtol=1e-10, atol=1e-11 * scale))
        np.testing.assert_allclose(N(gt), N(rt), **tol)
        if mode == 'bilinear':
            # the coordinate gradient carries a factor W / 2 (1040 at 2080 texels)
            su = float(ru.abs().max())
            gtol = (dict(rtol=1e-3, atol=2e-3 + 1e-4 * su) if k == 'f32'
                    else dict(rtol=1e-9, atol=1e-9 + 1e-12 * su))
            np.testing.assert_allclose(N(gu), N(ru), **gtol)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_tiled_abi_matches_block(k, mode):
    """kd_texture_mapping_backward_tiled_* (the texel-tile lists; texture_mapping itself runs the
    per-block kernel) called through the C ABI against the product's backward: a magnified
    region of ~40k samples in one tile next to spread samples, per-view and shared textures."""
    from kaolin_amd import _C, _lib
    gen = torch.Generator(device='cpu').manual_seed(17)
    B, C, hw = 2, 3, 96
    uv = torch.cat([0.30 + 0.02 * torch.rand((B, 40000, 2), generator=gen, dtype=torch.float64),
                    torch.rand((B, 9000, 2), generator=gen, dtype=torch.float64) * 1.1 - 0.05], 1)
    go = torch.rand(uv.shape[:2] + (C,), generator=gen, dtype=torch.float64)
    go[:, ::7] = 0.0  # samples with a zero incoming gradient are not listed
    for tb in (B, 1):
        tex = torch.rand((tb, C, hw, hw), generator=gen, dtype=torch.float64).to(DEV, DT[k])
        u, g_ = uv.to(DEV, DT[k]).contiguous(), go.to(DEV, DT[k]).contiguous()
        gc_ref, gt_ref = _C.texture_mapping_backward(g_, u, tex, mode)
        N_ = u.shape[1]
        bs = 0 if tb == 1 else C * hw * hw
        nb = _lib.texture_backward_workspace_size(B, N_, hw, hw, tb == 1)
        ws = torch.empty((nb,), dtype=torch.uint8, device=DEV)
        gt = torch.empty((tb, C, hw, hw), dtype=DT[k], device=DEV)
        gc = torch.empty_like(u)
        _lib.call(f'kd_texture_mapping_backward_tiled_{k}', B, N_, C, hw, hw, u.data_ptr(),
                  tex.data_ptr(), bs, {'nearest': 0, 'bilinear': 1}[mode], g_.data_ptr(),
                  gt.data_ptr(), gc.data_ptr(), ws.data_ptr(), nb,
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        scale = float(gt_ref.abs().max())
        tol = dict(rtol=1e-4, atol=1e-5 * scale) if k == 'f32' else dict(rtol=1e-10,
                                                                          atol=1e-11 * scale)
        np.testing.assert_allclose(N(gt), N(gt_ref), **tol)
        np.testing.assert_array_equal(N(gc), N(gc_ref))
