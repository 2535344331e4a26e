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
