"""View sharding across GPUs (one process per GPU), the one exchange step of the path, and the
DIB-R training step that bench.py times and the multi-process tests run.

The reference has no distributed code.  DIB-R views are independent through the
whole forward and the per-view backward kernels (no cross-view terms: rasterization_cuda.cu:62,
dibr_soft_mask_cuda.cu:47-51), so views are sharded in contiguous blocks and the only exchange is
the sum over views of the shared mesh parameters' gradients -- the ``.repeat(batch_size, 1, 1)``
backward of the reference training loop (examples/tutorial/ian_dibr.py:208-229) -- done as ONE
bucketed all-reduce (RCCL over xGMI with backend "nccl"; gloo on CPU for tests).

``dibr_step`` is that training step (prepare_vertices -> dibr_rasterization -> backward ->
all-reduce); ``GraphedStep`` captures its GPU part (everything up to the all-reduce) in one HIP
graph, so a step costs one graph launch plus one collective however few views a rank holds.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* when
    WORLD_SIZE > 1.  Returns (rank, world_size, local_rank)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        kw = {}
        if backend == 'nccl':
            torch.cuda.set_device(local)
            kw['device_id'] = torch.device('cuda', local)
        dist.init_process_group(backend=backend, init_method='env://', rank=rank,
                                world_size=world, **kw)
    return rank, world, local


def shard_views(total_views, rank, world):
    """Contiguous block of views for `rank`: (first_view, num_views).  Remainders go to the
    lowest ranks, so every view is rendered exactly once."""
    base, rem = divmod(total_views, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def _distributed(group=None):
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def allreduce_grads_(tensors, group=None):
    """Sum `tensors` (e.g. shared-parameter .grad) over all ranks in place, as one flat bucket
    (one collective per step).  No-op when not distributed."""
    tensors = [t for t in tensors if t is not None]
    if not tensors or not _distributed(group):
        return tensors
    if len(tensors) == 1 and tensors[0].is_contiguous():  # in place: no pack / unpack kernels
        dist.all_reduce(tensors[0], op=dist.ReduceOp.SUM, group=group)
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
    return tensors


class EarlyReduce:
    """Overlap for shared parameters whose gradients are final before the end of the backward
    (e.g. a texture, whose gradient comes out of texture_mapping's backward before the DIB-R
    backward runs): a post-accumulate hook marks a parameter ready as soon as autograd has
    written its gradient, and the asynchronous all-reduces are issued in the FIXED order of
    `params` (a parameter starts once it and every parameter before it are ready), so every rank
    issues the same collectives in the same order whatever order its hooks fire in; the
    collectives run on RCCL's stream while the rest of the backward runs on the compute stream.
    ``flush()`` issues whatever is left -- a parameter this rank produced no gradient for (e.g. a
    rank holding no views) contributes zeros -- and ``wait()`` joins them.  A caller that issues
    collectives of its own after the backward (the vertex gradient's bucket) calls ``flush()``
    first, so that every rank issues the shared reductions before its own, in the same order,
    whichever hooks fired on it."""

    def __init__(self, params, group=None):
        self.group = group
        self.params = list(params)
        self.works = []
        self.handles = []
        self.ready = [False] * len(self.params)
        self.next = 0
        if _distributed(group):
            for i, p in enumerate(self.params):
                self.handles.append(p.register_post_accumulate_grad_hook(
                    lambda _p, i=i: self._hook(i)))

    def _issue(self, i):
        p = self.params[i]
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        self.works.append(dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group,
                                          async_op=True))

    def _hook(self, i):
        self.ready[i] = True
        while self.next < len(self.params) and self.ready[self.next]:
            self._issue(self.next)
            self.next += 1

    def flush(self):
        """Issue every parameter not issued yet (zeros for a gradient this rank never produced)."""
        if self.handles:
            while self.next < len(self.params):
                self._issue(self.next)
                self.next += 1

    def wait(self):
        self.flush()
        for w in self.works:
            w.wait()
        self.works = []

    def remove(self):
        for h in self.handles:
            h.remove()
        self.handles = []


class GradBucket:
    """The step's exchange: the shared parameters' gradients summed over the ranks as ONE flat
    all-reduce per dtype (one in the DIB-R step: vertices and features share a dtype; a mixed
    set keeps each gradient's precision instead of casting it into one buffer).  The flat
    buffers are allocated once; ``pack()`` copies the gradients into them (on the current
    stream: inside a captured HIP graph these copies are graph nodes) and ``reduce()`` runs the
    collectives (RCCL over xGMI with backend "nccl", in the fixed order of the parameters' first
    dtype occurrence) and copies the sums back.  A single contiguous gradient of its dtype is
    reduced in place (no copies).  Parameters without a gradient on this rank contribute zeros,
    so every rank issues the same collectives."""

    def __init__(self, params, group=None):
        self.params = list(params)
        self.group = group
        self.flat = {}  # dtype -> flat buffer
        groups = {}
        for i, p in enumerate(self.params):
            groups.setdefault(p.dtype, []).append(i)
        self.groups = list(groups.items())  # [(dtype, [param indices])], first-occurrence order

    def _grads(self):
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        return [p.grad for p in self.params]

    @staticmethod
    def _in_place(gs):
        return len(gs) == 1 and gs[0].is_contiguous()

    def pack(self):
        if not self.params or not _distributed(self.group):
            return
        grads = self._grads()
        for dt, idx in self.groups:
            gs = [grads[i] for i in idx]
            if self._in_place(gs):
                continue
            n = sum(g.numel() for g in gs)
            flat = self.flat.get(dt)
            if flat is None or flat.numel() != n or flat.device != gs[0].device:
                flat = self.flat[dt] = torch.empty(n, device=gs[0].device, dtype=dt)
            off = 0
            for g in gs:
                flat[off:off + g.numel()].copy_(g.reshape(-1))
                off += g.numel()

    def reduce(self):
        if not self.params or not _distributed(self.group):
            return
        grads = self._grads()
        for dt, idx in self.groups:
            gs = [grads[i] for i in idx]
            if self._in_place(gs):
                dist.all_reduce(gs[0], op=dist.ReduceOp.SUM, group=self.group)
                continue
            flat = self.flat[dt]
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            off = 0
            for g in gs:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()

    def __call__(self):
        self.pack()
        self.reduce()


def dibr_forward_backward(vertices, faces, camera_proj, camera_transform, face_features, height,
                          width, grad_interp, grad_soft, sigmainv=7000., boxlen=0.02, knum=30,
                          prepare=None, render=None, gt_mask=None, iou='fused',
                          fused_vertices=True):
    """The GPU part of one DIB-R training step on this rank's views: project the
    shared mesh to the rank's cameras (``prepare_vertices``, utils.py:128-175), render
    (``dibr_rasterization``, dibr.py:119-209, valid faces = normals z >= 0) and back-propagate
    the fixed upstream gradients ``[grad_interp, grad_soft]`` into ``vertices.grad`` (summed over
    the rank's views) and the features' gradient.

    vertices (V, 3) leaf, faces (F, 3) int64, camera_transform (B_rank, 4, 3), face_features
    (B_rank, F, 3, D) or (1, F, 3, D) shared.  `prepare` / `render` default to the HIP kernels
    (kaolin_amd.render.mesh); the CPU tests pass oracle-backed ones with the same signatures.
    With gt_mask (B_rank, H, W) the soft mask's gradient is that of the DIB-R silhouette loss
    mask_iou(soft_mask, gt_mask) (metrics/render.py:18-40, ian_dibr.py:264-265) instead of
    grad_soft: fused into the renderer (iou='fused', dibr_rasterization_with_mask_iou) or as the
    composition dibr_rasterization + mask_iou (iou='compose').
    fused_vertices (default; HIP kernels, no gt_mask): ``dibr_rasterization_from_vertices``, one
    node whose forward projects the vertices inside the binning launch (no kd_prepare_fwd), instead
    of prepare_vertices + dibr_rasterization.  C3, same box (profiles/r04/ab_vp*.txt): 0.2963 ->
    0.2949 ms per step at 8 views, 0.1082 -> 0.1056 at 1 view.
    Returns face_idx (B_rank, H, W)."""
    B = camera_transform.shape[0]
    if fused_vertices and gt_mask is None and prepare is None and render is None:
        from .render.mesh import dibr_rasterization_from_vertices
        feats = face_features if face_features.shape[0] == B else \
            face_features.expand(B, *face_features.shape[1:])
        interp, soft, face_idx = dibr_rasterization_from_vertices(
            height, width, vertices.unsqueeze(0), faces, camera_proj, camera_transform, feats,
            sigmainv, boxlen, knum)
        torch.autograd.backward([interp, soft], [grad_interp, grad_soft])
        return face_idx
    if prepare is None or render is None:
        from .render.mesh import dibr_rasterization, prepare_vertices
        prepare = prepare or prepare_vertices
        render = render or dibr_rasterization
    fvc, fvi, nrm = prepare(vertices.unsqueeze(0), faces, camera_proj,
                            camera_transform=camera_transform)
    feats = face_features if face_features.shape[0] == B else \
        face_features.expand(B, *face_features.shape[1:])
    if gt_mask is not None:
        from .render.mesh import dibr_rasterization_with_mask_iou
        from .metrics.render import mask_iou
        one = torch.ones((), device=gt_mask.device, dtype=gt_mask.dtype)
        if iou == 'fused':
            interp, soft, face_idx, loss = dibr_rasterization_with_mask_iou(
                height, width, fvc[..., 2], fvi, feats, nrm[..., 2], gt_mask, sigmainv, boxlen,
                knum)
        else:
            interp, soft, face_idx = render(height, width, fvc[..., 2], fvi, feats, nrm[..., 2],
                                            sigmainv, boxlen, knum)
            loss = mask_iou(soft, gt_mask)
        torch.autograd.backward([interp, loss], [grad_interp, one])
        return face_idx
    interp, soft, face_idx = render(height, width, fvc[..., 2], fvi, feats, nrm[..., 2],
                                    sigmainv, boxlen, knum)
    torch.autograd.backward([interp, soft], [grad_interp, grad_soft])
    return face_idx


def dibr_step(vertices, faces, camera_proj, camera_transform, face_features, height, width,
              grad_interp, grad_soft, sigmainv=7000., boxlen=0.02, knum=30, shared=(),
              group=None, prepare=None, render=None):
    """One DIB-R training step: ``dibr_forward_backward`` then the step's one exchange, a single
    bucketed all-reduce of the shared parameters' gradients (vertices + `shared`, e.g. a feature
    table shared by every view).  `shared` parameters are reduced early and asynchronously when
    their gradients are final before the vertex gradient (``EarlyReduce``).  The caller resets
    the .grad fields between steps (as an optimizer's zero_grad would)."""
    early = EarlyReduce(shared, group)
    try:
        face_idx = dibr_forward_backward(vertices, faces, camera_proj, camera_transform,
                                         face_features, height, width, grad_interp, grad_soft,
                                         sigmainv, boxlen, knum, prepare, render)
        late = [vertices] + [p for p in shared if not early.handles]
        early.flush()  # the shared reductions first on every rank, whichever hooks fired
        GradBucket(late, group)()
        early.wait()
    finally:
        early.remove()
    return face_idx


class GraphedStep:
    """``dibr_step`` with its GPU part captured once in a HIP graph (torch.cuda.CUDAGraph over
    the library's stream-ordered launches) and replayed; the step's exchange (``GradBucket``: the
    shared gradients packed into one flat buffer -- the packing copies are captured in the graph
    -- and one all-reduce) stays an eager RCCL call after the replay.  Inputs and the .grad
    tensors are static: the replay overwrites the gradients in place (they are None at capture,
    so the captured backward assigns instead of accumulating).  `warmup` eager steps on a side
    stream come first (they also build the per-topology vertex->face table, a one-time host
    copy).  Every replay restarts the library's device state (pool counters, the record cursor,
    the zeroed-on-the-side gradient buffers) inside the graph: tests/test_gpu_graphed_step.py
    compares replays with eager steps."""

    def __init__(self, params, fn, params_to_reduce=None, group=None, warmup=3):
        self.params = list(params)  # every parameter whose .grad the step writes
        self.reduce = self.params if params_to_reduce is None else list(params_to_reduce)
        self.fn = fn
        self.group = group
        self.bucket = GradBucket(self.reduce, group)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._clear()
                fn()
                self.bucket.pack()
        torch.cuda.current_stream().wait_stream(s)
        self._clear()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn()
            self.bucket.pack()

    def _clear(self):
        for p in self.params:
            p.grad = None

    def replay(self):
        """The GPU part of the step (one graph launch)."""
        self.graph.replay()
        return self.out

    def exchange(self):
        """The step's all-reduce (eager RCCL), after the replay."""
        self.bucket.reduce()

    def __call__(self):
        self.replay()
        self.exchange()
        return self.out
