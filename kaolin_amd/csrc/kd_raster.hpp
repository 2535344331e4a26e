// kd_raster.hpp -- rasterize forward / backward launch interface shared with the fused DIB-R path
// (kd_dibr.hip).  Kernels: kd_raster.hip.
#pragma once

#include "kd_binning.hpp"

namespace kd {

template <typename T>
struct RasterFwdArgs {
  FaceSet<T> fs;
  BinBuffers bb;       // bins of the valid faces' boxes (bb.cull set: fp32 pair raster)
  const T *fvz;        // depth of corner j of face row i at fvz[i * fvz_fs + j * fvz_cs]
  int64_t fvz_fs, fvz_cs;
  const T *feat;
  int D;
  float eps;
  T *interp;
  int64_t *face_idx;
  T *weights;
};

// The face -> vertex step of the backward fused into the DIB-R backward: a
// face corner's image-space gradient (gx, gy) goes through the projection and the transposed
// camera transform (kaolin/render/camera/legacy.py:120-139, render/mesh/utils.py:164-167; the
// arithmetic of kd_prepare.hip's corner_grad) and is added to its vertex's gradient
// (ops/mesh/mesh.py:24-45: the gather's backward is this scatter).  No (B, F, 3, 2) gradient is
// materialised and no separate face -> vertex kernel runs.
template <typename T>
struct VertexOut {
  T *grad;               // (Bv, V, 3), zeroed by the caller; nullptr: grad_fvi is written instead
  const int64_t *faces;  // (F, 3)
  const T *fvc;          // (B, F, 3, 3) camera-space corners (prepare_vertices' output)
  const T *proj;         // (3)
  const T *tf;           // (B, 4, 3) camera transforms
  int64_t F, V;
  int Bv;                // 1: vertices shared by the views (their gradients summed), else B
};

template <typename T>
__device__ __forceinline__ void vertex_add(const VertexOut<T> &vo, int64_t row, int k, T gx, T gy) {
  if (gx == (T)0 && gy == (T)0) return;
  const int b = (int)(row / vo.F);
  const int64_t f = row - (int64_t)b * vo.F;
  const T *c = vo.fvc + row * 9 + k * 3;
  const T pz = c[2] * vo.proj[2];
  const T x = c[0] * vo.proj[0] / pz, y = c[1] * vo.proj[1] / pz;
  const T g0 = gx * vo.proj[0] / pz, g1 = gy * vo.proj[1] / pz;
  const T g2 = (T)0 - (gx * x + gy * y) / c[2];
  const T *tf = vo.tf + (int64_t)b * 12;
  const int64_t v = vo.faces[f * 3 + k];
  T *out = vo.grad + ((vo.Bv == 1 ? 0 : (int64_t)b * vo.V) + v) * 3;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const T g = tf[q * 3 + 0] * g0 + tf[q * 3 + 1] * g1 + tf[q * 3 + 2] * g2;
    if (g != (T)0) atomicAdd(out + q, g);
  }
}

// fp32 pair raster with edge culling in use (needs BinBuffers::cull)
template <typename T>
bool raster_uses_cull();
// the raster kernel over already built bins
template <typename T>
int raster_launch(RasterFwdArgs<T> &a, hipStream_t stream);
// the backward tile kernel, accumulating into gfvi / gfeat (zeroed by the caller)
template <typename T>
int raster_backward_launch(int B, int H, int W, int64_t F, int D, const T *grad,
                           const int64_t *fidx, const T *weights, const T *fvi, const T *feat,
                           float eps, T *gfvi, T *gfeat, hipStream_t stream);

}  // namespace kd
