// kd_prepare.hip -- the DIB-R step's upstream projection and its face->vertex backward, fused
// (SURVEY.md §8 f1).
//
// Reference: kaolin/render/mesh/utils.py:128-175 (prepare_vertices) composes
//   vertices_camera = pad(vertices, 1) @ camera_transform                 (utils.py:164-167)
//   vertices_image  = perspective_camera(vertices_camera, camera_proj)    (legacy.py:120-139)
//   face_vertices_* = index_vertices_by_faces(..., faces)                 (ops/mesh/mesh.py:24-45)
//   face_normals    = cross(v1 - v0, v2 - v0) / (|.| + 1e-10)             (trianglemesh.py:313-336)
// as ~15 PyTorch kernels forward and ~25 backward, the largest being the index_add that scatters
// the (B, F, 3, C) face-corner gradients back onto the vertices (one float atomic per corner
// coordinate).  Here:
//   kd_prepare_fwd  one thread per (view, face): transform, project, gather and normal in
//                   registers, write the three outputs once.
//   kd_prepare_bwd  one thread per incident (face, corner) entry of the vertex -> corner CSR
//                   (built once per topology): projection / normal / gather backward and the
//                   transposed camera transform, summed over the views when the vertices are
//                   shared; workgroups take whole vertices (ranges computed once per
//                   topology), sum each vertex's entries in LDS and store it once.
#include "../../include/kaolin_dibr.h"
#include "kd_capi.hpp"
#include "kd_common.hpp"
#include "kd_prep.hpp"
#include "kd_tile.hpp"

namespace kd {

// One thread per (view, face) row; the rows' outputs (9 + 6 + 3 values each) are assembled in
// LDS and written by the workgroup as contiguous, coalesced runs.
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_prepare_fwd(PrepArgs<T> a, T *fvc, T *fvi, T *nrm) {
  __shared__ __align__(16) T s_c[kBlock * 9];
  __shared__ __align__(16) T s_i[kBlock * 6];
  __shared__ __align__(16) T s_n[kBlock * 3];
  const int64_t total = (int64_t)a.B * a.F;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock; i0 < total; i0 += (int64_t)gridDim.x * kBlock) {
    const int64_t i = i0 + threadIdx.x;
    const int rows = (int)min((int64_t)kBlock, total - i0);
    if (i < total) {
      T c[3][3], fi[6], n[3];
      prep_face<T>(a, i, c, fi, n);
      prep_stage<T>(c, fi, n, s_c, s_i, s_n);
    }
    __syncthreads();
    lds_to_global<T>(fvc + i0 * 9, s_c, rows * 9);
    lds_to_global<T>(fvi + i0 * 6, s_i, rows * 6);
    lds_to_global<T>(nrm + i0 * 3, s_n, rows * 3);
    __syncthreads();
  }
}

// Gradient of one face corner w.r.t. its camera-space position: the gather (grad_fvc), the
// projection (grad_fvi) and the unit normal (grad_nrm, which depends on all three corners).
template <typename T>
__device__ __forceinline__ void corner_grad(const T c[3][3], int k, const T proj[3],
                                            const T *gc, const T *gi, const T *gn, T g[3]) {
  g[0] = gc ? gc[0] : (T)0;
  g[1] = gc ? gc[1] : (T)0;
  g[2] = gc ? gc[2] : (T)0;
  if (gi) {  // x = P0 cx / (P2 cz), y = P1 cy / (P2 cz)
    const T pz = c[k][2] * proj[2];
    const T x = c[k][0] * proj[0] / pz, y = c[k][1] * proj[1] / pz;
    g[0] += gi[0] * proj[0] / pz;
    g[1] += gi[1] * proj[1] / pz;
    g[2] -= (gi[0] * x + gi[1] * y) / c[k][2];
  }
  if (gn) {  // n = r / (|r| + 1e-10), r = e1 x e2, e1 = c1 - c0, e2 = c2 - c0
    const T e1[3] = {c[1][0] - c[0][0], c[1][1] - c[0][1], c[1][2] - c[0][2]};
    const T e2[3] = {c[2][0] - c[0][0], c[2][1] - c[0][1], c[2][2] - c[0][2]};
    const T r[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                    e1[0] * e2[1] - e1[1] * e2[0]};
    const T len = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const T d = len + (T)1e-10;
    const T rg = r[0] * gn[0] + r[1] * gn[1] + r[2] * gn[2];
    const T s = len > (T)0 ? rg / (len * d * d) : (T)0;
    const T gr[3] = {gn[0] / d - r[0] * s, gn[1] / d - r[1] * s, gn[2] / d - r[2] * s};
    // (a x b) . g = a . (b x g) = b . (g x a)
    const T ge1[3] = {e2[1] * gr[2] - e2[2] * gr[1], e2[2] * gr[0] - e2[0] * gr[2],
                      e2[0] * gr[1] - e2[1] * gr[0]};
    const T ge2[3] = {gr[1] * e1[2] - gr[2] * e1[1], gr[2] * e1[0] - gr[0] * e1[2],
                      gr[0] * e1[1] - gr[1] * e1[0]};
#pragma unroll
    for (int j = 0; j < 3; ++j) g[j] += k == 1 ? ge1[j] : k == 2 ? ge2[j] : -(ge1[j] + ge2[j]);
  }
}

// corner_grad with only the projection's incoming gradient (grad_fvc = grad_nrm = NULL): the
// same operations in the same order on the corner's own camera-space point, so the same bits.
template <typename T>
__device__ __forceinline__ void corner_grad_gi(const T ck[3], const T proj[3], T gi0, T gi1,
                                               T g[3]) {
  g[0] = (T)0;
  g[1] = (T)0;
  g[2] = (T)0;
  const T pz = ck[2] * proj[2];
  const T x = ck[0] * proj[0] / pz, y = ck[1] * proj[1] / pz;
  g[0] += gi0 * proj[0] / pz;
  g[1] += gi1 * proj[1] / pz;
  g[2] -= (gi0 * x + gi1 * y) / ck[2];
}

// One thread per incident (face, corner) entry of the CSR (entries grouped by vertex) and vertex
// batch: the corner's gradient, transformed back to world space, summed over the views it
// covers.  Workgroup k takes the entries [blocks[k], blocks[k+1]): whole vertices, at most 256
// entries, or one vertex alone when it has more (then its entries are walked in 256-entry
// rounds, each thread summing its own).  A vertex's entries are summed in LDS and stored once --
// no memset, no global atomics.  The workgroups past the last range (blockIdx.x >= nblk) write
// the zero gradient of vertices without incident faces.
//
// FROM_V (the DIB-R node's backward: grad_fvi only): the corner's camera-space point is
// recomputed from the vertex per view (cam_point, the forward's own arithmetic: the bits of fvc)
// instead of gathering the face's 9 camera coordinates from fvc for every (entry, view) -- the
// entry's vertex is loaded once, the view loop gathers only the corner's 8-byte grad_fvi.
template <typename T, bool FROM_V = false>
__global__ __launch_bounds__(kBlock) void kd_prepare_bwd(PrepArgs<T> a, const T *fvc,
                                                         const T *gfvc, const T *gfvi,
                                                         const T *gnrm, const int64_t *adj_off,
                                                         const int32_t *adj,
                                                         const int32_t *blocks, int nblk,
                                                         T *gvert, const int32_t *adj_v = nullptr) {
  __shared__ T s_acc[kBlock][3];
  __shared__ int64_t s_vid[kBlock];
  __shared__ int s_scan[4];
  const int bv = blockIdx.y;
  T *gv = gvert + (int64_t)bv * a.V * 3;
  if ((int)blockIdx.x >= nblk) {  // isolated vertices
    const int64_t v = (int64_t)(blockIdx.x - nblk) * kBlock + threadIdx.x;
    if (v < a.V && adj_off[v] == adj_off[v + 1]) {
      gv[v * 3 + 0] = (T)0;
      gv[v * 3 + 1] = (T)0;
      gv[v * 3 + 2] = (T)0;
    }
    return;
  }
  // XCD-aware: workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8), so XCD x takes the
  // contiguous band of ranges [x q + min(x, r), ...) (nblk = 8 q + r): neighbouring vertices,
  // whose faces' corner rows (in every view) overlap, share one L2
  int rb = blockIdx.x;
  if (nblk >= 64) {
    const int x = rb & 7, j = rb >> 3, q = nblk >> 3, r = nblk & 7;
    rb = x * q + min(x, r) + j;
  }
  const int64_t e0 = blocks[rb], e1 = blocks[rb + 1];
  const bool valid = e0 + threadIdx.x < e1;
  int64_t v = -1;
  T g3[3] = {0, 0, 0};
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kBlock) {
    const int32_t fc = adj[e];
    const int64_t f = fc / 3;
    const int k = fc - (int)f * 3;
    // (F, 3) row-major: entry fc = 3 f + k (one vertex per multi-round range); FROM_V reads the
    // entry's vertex directly (adj_v) instead of through the face row
    v = FROM_V ? (int64_t)adj_v[e] : a.faces[fc];
    const int b0 = a.Bv == 1 ? 0 : bv, b1 = a.Bv == 1 ? a.B : bv + 1;
    if constexpr (FROM_V) {
      const T *pv = a.vertices + ((int64_t)bv * a.V + v) * 3;  // (bv = 0 when Bv == 1)
      const T p[3] = {pv[0], pv[1], pv[2]};
      for (int b = b0; b < b1; ++b) {
        const int64_t row = (int64_t)b * a.F + f;
        const T *tf = a.tf + (int64_t)b * 12;
        T ck[3], g[3];
        cam_point<T>(tf, p, ck);
        const T *gi = gfvi + row * 6 + k * 2;
        corner_grad_gi<T>(ck, a.proj, gi[0], gi[1], g);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          g3[q] += tf[q * 3 + 0] * g[0] + tf[q * 3 + 1] * g[1] + tf[q * 3 + 2] * g[2];
      }
      continue;
    }
    for (int b = b0; b < b1; ++b) {
      const int64_t row = (int64_t)b * a.F + f;
      T c[3][3];
      const T *pc = fvc + row * 9;
#pragma unroll
      for (int q = 0; q < 9; ++q) c[q / 3][q % 3] = pc[q];
      T g[3];
      corner_grad<T>(c, k, a.proj, gfvc ? gfvc + row * 9 + k * 3 : nullptr,
                     gfvi ? gfvi + row * 6 + k * 2 : nullptr, gnrm ? gnrm + row * 3 : nullptr, g);
      // cam_j = sum_i p_i tf[i][j] + tf[3][j]  ->  dL/dp_i = sum_j tf[i][j] g_j
      const T *tf = a.tf + (int64_t)b * 12;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        g3[q] += tf[q * 3 + 0] * g[0] + tf[q * 3 + 1] * g[1] + tf[q * 3 + 2] * g[2];
    }
  }
  // segments of equal vertex inside the workgroup (entries are grouped by vertex)
  s_vid[threadIdx.x] = v;
  __syncthreads();
  const bool start = valid && (threadIdx.x == 0 || s_vid[threadIdx.x - 1] != v);
  int nseg;
  const int seg = wg_exclusive_scan(start ? 1 : 0, s_scan, nseg) + (start ? 0 : -1);
  if (threadIdx.x < nseg) {
    s_acc[threadIdx.x][0] = (T)0;
    s_acc[threadIdx.x][1] = (T)0;
    s_acc[threadIdx.x][2] = (T)0;
  }
  __syncthreads();
  if (valid) {
    if (start) s_vid[kBlock - 1 - seg] = v;  // segment -> vertex (upper half of the array)
    atomicAdd(&s_acc[seg][0], g3[0]);
    atomicAdd(&s_acc[seg][1], g3[1]);
    atomicAdd(&s_acc[seg][2], g3[2]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nseg * 3; i += kBlock) {
    const int sg = i / 3, q = i - sg * 3;
    gv[s_vid[kBlock - 1 - sg] * 3 + q] = s_acc[sg][q];
  }
}

template <typename T>
static int prep_fwd(int B, int Bv, int64_t V, int64_t F, const T *vert, const int64_t *faces,
                    const T *proj, const T *tf, T *fvc, T *fvi, T *nrm, void *stream);
template <typename T>
int prep_vertices_forward(int B, int Bv, int64_t V, int64_t F, const T *vert, const int64_t *faces,
                          const T *proj, const T *tf, T *fvc, T *fvi, T *nrm, void *stream) {
  return prep_fwd<T>(B, Bv, V, F, vert, faces, proj, tf, fvc, fvi, nrm, stream);
}
template int prep_vertices_forward<float>(int, int, int64_t, int64_t, const float *,
                                          const int64_t *, const float *, const float *, float *,
                                          float *, float *, void *);
template int prep_vertices_forward<double>(int, int, int64_t, int64_t, const double *,
                                           const int64_t *, const double *, const double *,
                                           double *, double *, double *, void *);

template <typename T>
static int prep_fwd(int B, int Bv, int64_t V, int64_t F, const T *vert, const int64_t *faces,
                    const T *proj, const T *tf, T *fvc, T *fvi, T *nrm, void *stream) {
  KD_CHECK_ARG(B >= 0 && V >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(Bv == 1 || Bv == B, "vertex batch must be 1 or the view count");
  const int64_t total = (int64_t)B * F;
  if (total == 0) return KD_OK;
  PrepArgs<T> a{B, Bv, V, F, vert, faces, proj, tf};
  const unsigned blocks = (unsigned)std::min<int64_t>((total + kBlock - 1) / kBlock, 65536);
  {
    ProfScope prof(K_PREPARE_FWD, (hipStream_t)stream);
    hipLaunchKernelGGL(kd_prepare_fwd<T>, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, a,
                       fvc, fvi, nrm);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "prepare fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
static int prep_bwd(int B, int Bv, int64_t V, int64_t F, const int64_t *faces, const T *proj,
                    const T *tf, const T *fvc, const T *gfvc, const T *gfvi, const T *gnrm,
                    const int64_t *adj_off, const int32_t *adj, const int32_t *blocks,
                    int64_t nblk, T *gvert, void *stream, const T *vert = nullptr,
                    const int32_t *adj_v = nullptr) {
  KD_CHECK_ARG(!vert || (!gfvc && !gnrm && gfvi && adj_v),
               "from vertices: only the grad_fvi form (grad_fvc and grad_normals NULL), with "
               "adj_vertex");
  KD_CHECK_ARG(B >= 0 && V >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(Bv == 1 || Bv == B, "vertex batch must be 1 or the view count");
  KD_CHECK_ARG(F * 3 < (1ll << 31), "too many faces");
  const int64_t total = (int64_t)Bv * V;
  if (total == 0) return KD_OK;
  if (F == 0 || B == 0) {
    hipError_t e0 = zero_words(gvert, sizeof(T) * total * 3, (hipStream_t)stream);
    if (e0 != hipSuccess) return set_error(KD_ERR_LAUNCH, "memset: %s", hipGetErrorString(e0));
    return KD_OK;
  }
  KD_CHECK_ARG(adj_off && adj && blocks && nblk >= 1, "vertex adjacency and its ranges required");
  const int64_t nz = (V + kBlock - 1) / kBlock;
  KD_CHECK_ARG(nblk + nz < (1ll << 31), "too many faces");
  PrepArgs<T> a{B, Bv, V, F, vert, faces, proj, tf};
  {
    ProfScope prof(K_PREPARE_BWD, (hipStream_t)stream);
    if (vert)
      hipLaunchKernelGGL((kd_prepare_bwd<T, true>), dim3((unsigned)(nblk + nz), Bv), dim3(kBlock),
                         0, (hipStream_t)stream, a, fvc, gfvc, gfvi, gnrm, adj_off, adj, blocks,
                         (int)nblk, gvert, adj_v);
    else
      hipLaunchKernelGGL((kd_prepare_bwd<T, false>), dim3((unsigned)(nblk + nz), Bv),
                         dim3(kBlock), 0, (hipStream_t)stream, a, fvc, gfvc, gfvi, gnrm, adj_off,
                         adj, blocks, (int)nblk, gvert);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "prepare bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

extern "C" {

int kd_prepare_vertices_forward_f32(int B, int Bv, int64_t V, int64_t F, const float *vertices,
                                    const int64_t *faces, const float *camera_proj,
                                    const float *camera_transform, float *fvc, float *fvi,
                                    float *normals, void *stream) {
  return prep_fwd<float>(B, Bv, V, F, vertices, faces, camera_proj, camera_transform, fvc, fvi,
                         normals, stream);
}
int kd_prepare_vertices_forward_f64(int B, int Bv, int64_t V, int64_t F, const double *vertices,
                                    const int64_t *faces, const double *camera_proj,
                                    const double *camera_transform, double *fvc, double *fvi,
                                    double *normals, void *stream) {
  return prep_fwd<double>(B, Bv, V, F, vertices, faces, camera_proj, camera_transform, fvc, fvi,
                          normals, stream);
}
int kd_prepare_vertices_backward_f32(int B, int Bv, int64_t V, int64_t F, const int64_t *faces,
                                     const float *camera_proj, const float *camera_transform,
                                     const float *fvc, const float *grad_fvc,
                                     const float *grad_fvi, const float *grad_normals,
                                     const int64_t *adj_offsets, const int32_t *adj,
                                     const int32_t *adj_ranges, int64_t num_ranges,
                                     float *grad_vertices, void *stream) {
  return prep_bwd<float>(B, Bv, V, F, faces, camera_proj, camera_transform, fvc, grad_fvc,
                         grad_fvi, grad_normals, adj_offsets, adj, adj_ranges, num_ranges,
                         grad_vertices, stream);
}
int kd_prepare_vertices_backward_f64(int B, int Bv, int64_t V, int64_t F, const int64_t *faces,
                                     const double *camera_proj, const double *camera_transform,
                                     const double *fvc, const double *grad_fvc,
                                     const double *grad_fvi, const double *grad_normals,
                                     const int64_t *adj_offsets, const int32_t *adj,
                                     const int32_t *adj_ranges, int64_t num_ranges,
                                     double *grad_vertices, void *stream) {
  return prep_bwd<double>(B, Bv, V, F, faces, camera_proj, camera_transform, fvc, grad_fvc,
                          grad_fvi, grad_normals, adj_offsets, adj, adj_ranges, num_ranges,
                          grad_vertices, stream);
}

int kd_prepare_vertices_backward_vertices_f32(int B, int Bv, int64_t V, int64_t F,
                                              const float *vertices, const int64_t *faces,
                                              const float *camera_proj,
                                              const float *camera_transform,
                                              const float *grad_fvi, const int64_t *adj_offsets,
                                              const int32_t *adj, const int32_t *adj_vertex,
                                              const int32_t *adj_ranges,
                                              int64_t num_ranges, float *grad_vertices,
                                              void *stream) {
  KD_CHECK_ARG(vertices, "vertices is NULL");
  return prep_bwd<float>(B, Bv, V, F, faces, camera_proj, camera_transform, nullptr, nullptr,
                         grad_fvi, nullptr, adj_offsets, adj, adj_ranges, num_ranges,
                         grad_vertices, stream, vertices, adj_vertex);
}
int kd_prepare_vertices_backward_vertices_f64(int B, int Bv, int64_t V, int64_t F,
                                              const double *vertices, const int64_t *faces,
                                              const double *camera_proj,
                                              const double *camera_transform,
                                              const double *grad_fvi, const int64_t *adj_offsets,
                                              const int32_t *adj, const int32_t *adj_vertex,
                                              const int32_t *adj_ranges,
                                              int64_t num_ranges, double *grad_vertices,
                                              void *stream) {
  KD_CHECK_ARG(vertices, "vertices is NULL");
  return prep_bwd<double>(B, Bv, V, F, faces, camera_proj, camera_transform, nullptr, nullptr,
                          grad_fvi, nullptr, adj_offsets, adj, adj_ranges, num_ranges,
                          grad_vertices, stream, vertices, adj_vertex);
}

// Host: workgroup entry ranges of the backward from the CSR offsets (host memory, V + 1 values):
// greedy, whole vertices per range, at most `cap` entries unless one vertex alone has more.
// Writes up to V + 1 range starts plus the end into ranges_out; returns the number of ranges.
int64_t kd_prepare_vertices_ranges(const int64_t *adj_offsets, int64_t V, int32_t cap,
                                   int32_t *ranges_out) {
  if (!adj_offsets || !ranges_out || V < 0 || cap < 1) return -1;
  int64_t n = 0, start = adj_offsets[0];
  for (int64_t v = 0; v < V; ++v) {
    const int64_t end = adj_offsets[v + 1];
    if (end - start > cap && adj_offsets[v] > start) {  // close the range before vertex v
      ranges_out[n++] = (int32_t)start;
      start = adj_offsets[v];
    }
  }
  if (adj_offsets[V] > start) ranges_out[n++] = (int32_t)start;
  ranges_out[n] = (int32_t)adj_offsets[V];
  return n;
}

}  // extern "C"
