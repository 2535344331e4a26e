// kd_binning.hpp -- ordered coarse binning of faces into 32x32-pixel (or larger) tiles.
//
// The reference scans every face for every pixel (rasterization_cuda.cu:88-171,
// dibr_soft_mask_cuda.cu:80-172).  Its results depend on face ORDER: the raster keeps the first
// face on a depth tie (strict `z > best`), the soft mask keeps the first K faces by index.  The
// bins therefore hold, for every (view, coarse tile), the faces touching it in ascending index
// order, produced without sorting by a three-pass counting scatter:
//   1. kd_bin_count   one workgroup per (256-face chunk, view): each face computes its exact
//                     pixel span (kd::make_span), stores it, and counts per coarse tile in LDS.
//   2. kd_bin_scan    one workgroup per (coarse tile, view): exclusive scan over the chunks.
//   3. kd_bin_scatter one workgroup per (chunk, view): the rank of a face inside its chunk for a
//                     tile is a popcount over an LDS bitmask of the chunk's faces touching that
//                     tile, so the global position is scan offset + rank: ascending by face.
// Layout in the workspace (N = rows of the face arrays):
//   spans  [N]           Span (8 B)
//   counts [B][nchunk][nct] int32 (turned into exclusive offsets by the scan)
//   totals [B][nct]      int32
//   bins   [nct][N]      int32 local face index; the (b, c) bin starts at c*N + first[b] and has
//                        room for the view's whole face count.
#pragma once

#include "kd_common.hpp"

namespace kd {

struct BinBuffers {
  Span *spans;
  int *counts;
  int *totals;
  int *bins;
  int nchunk;
  BinGeom g;
};

size_t bin_workspace_bytes(int B, int H, int W, int64_t N, int64_t max_per_view);
// Carves the buffers from `ws` starting at *offset (advanced past them).
BinBuffers bin_carve(void *ws, size_t &offset, int B, int H, int W, int64_t N,
                     int64_t max_per_view);

template <typename T>
hipError_t bin_faces(const FaceSet<T> &fs, const BinBuffers &bb, hipStream_t stream);

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

}  // namespace kd
