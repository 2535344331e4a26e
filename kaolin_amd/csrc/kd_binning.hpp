// kd_binning.hpp -- ordered coarse binning of faces into 32x32-pixel (or larger) tiles.
//
// The reference scans every face for every pixel (rasterization_cuda.cu:88-171,
// dibr_soft_mask_cuda.cu:80-172).  Its results depend on face ORDER: the raster keeps the first
// face on a depth tie (strict `z > best`), the soft mask keeps the first K faces by index.  The
// bins therefore hold, for every (view, coarse tile), the faces touching it in ascending index
// order, produced without sorting by a three-pass counting scatter:
//   1. kd_bin_count   one workgroup per (256-face chunk, view): each face computes its exact
//                     pixel span (kd::make_span), stores it, and counts per coarse tile in LDS.
//   2. kd_bin_scan    one wave per (coarse tile, view): exclusive scan over the chunks.
//   3. kd_bin_scatter one workgroup per (chunk, view): the rank of a face inside its chunk for a
//                     tile is a popcount over an LDS bitmask of the chunk's faces touching that
//                     tile, so the global position is scan offset + rank: ascending by face.
//                     Each workgroup scans its view's totals over the coarse tiles to place the
//                     bins in the view's region (CSR; the chunk-0 workgroup stores the bases).
// Layout in the workspace (N = rows of the face arrays):
//   spans  [N]           Span (8 B)
//   counts [B][nct][nchunk] int32, tile-major (read by the scan)
//   offs   [B][nchunk][nct] int32, the scan's exclusive offsets, chunk-major (read by the scatter)
//   totals [B][nct]      int32
//   base   [B][nct]      int32 start of bin (b, c) inside view b's region, -1 = overflowed
//   bins   [xper * N]    int32 local face index; view b owns the region [xper*lo, xper*hi) of
//                        its rows [lo, hi), its bins packed in coarse-tile order (exclusive
//                        scan of the totals, kd_bin_scatter).  A bin that does not fit is marked
//                        overflowed: its tiles walk every face of the view (entry e = face e),
//                        which the exact span filter of the walk turns into the same face list,
//                        so an overflow costs time, never correctness.
//   cull   [N][2]        float4: fp32 raster edge-culling coefficients (raster_cull_coefs), only
//                        written when BinBuffers::cull is set (fp32 rasterization).
//   order  [B * tiles]   int2 (view * tiles + fine tile, coarse bin face count), heaviest
//                        coarse bin first (the count saves the tile kernels a dependent load).
#pragma once

#include "kd_common.hpp"

namespace kd {

// Region entries per face row (xper): 16 covers a face whose box reaches 4 x 4 coarse tiles.
constexpr int kBinEntriesPerFace = 16;

struct BinBuffers {
  Span *spans;
  int *counts;     // [B][nct][nchunk] per-chunk counts, tile-major (kd_bin_count -> kd_bin_scan)
  int *offs;       // [B][nchunk][nct] the chunks' exclusive offsets in each bin, chunk-major
                   // (kd_bin_scan -> kd_bin_scatter: one contiguous row per scatter workgroup)
  int *totals;
  int *base;       // [B][nct]: start of bin (b, c) in view b's region, -1 = overflowed
  int *bins;
  int xper;        // region entries per face row
  float limit;     // usable fraction of each region (kd_set_pool_limits; 1 in production)
  float4 *cull;    // nullptr: not computed
  float cull_eps;  // the raster eps (cull coefficients only)
  int *clear;      // nullable: n_clear ints zeroed by kd_bin_count (counters of later passes)
  int n_clear;
  int *clear_b;    // nullable: a second such range (e.g. the fused mask_iou accumulators)
  int n_clear_b;
  int2 *order;     // [B * fine tiles] (view * tiles + tile, its coarse bin's face count),
                   // heaviest first (tile_order in kd_bin_scatter): the tile kernels' dispatch order
  unsigned short *hist;  // nullable: [B * fine tiles][4] per (tile, part) the previous same-shape
                         // call's duration bucket + 1 (0: none), written by the fused forward and
                         // ordering the tiles instead of the coarse counts (kd_set_tile_history)
  int nchunk;
  int chunk;       // faces per chunk (bin_chunk: 256 or 512)
  BinGeom g;
};

// Edge-culling coefficients of one face in its own frame (column span.x0, row span.y0); see
// kd_cull.hpp.  out: {lo0 P0, lo0 P1, lo1 P0, lo1 P1, hi0 P0, hi0 P1, hi1 P0, hi1 P1}.
template <typename T>
__device__ void raster_cull_coefs(const T v[6], float M, int H, int W, Span sp, float eps,
                                  float out[8]);

// Bin (b, c) of view b (rows [lo, lo + nview)): its ascending local face indices and count, or
// nullptr when the bin overflowed its region -- then the caller walks all nview faces of the
// view (entry e = local face e) and its exact span filter selects the same faces.
__device__ __forceinline__ const int *bin_list(const BinBuffers &bb, int b, int c, int64_t lo,
                                               int nview, int nbin, int &n) {
  const int64_t bc = (int64_t)b * bb.g.nct() + c;
  const int base = bb.base[bc];
  if (base < 0) {
    n = nview;
    return nullptr;
  }
  n = nbin >= 0 ? nbin : bb.totals[bc];
  return bb.bins + (int64_t)bb.xper * lo + base;
}

// Process-wide fractions of the pool capacities usable by a forward (kd_set_pool_limits; a test
// hook that forces the overflow paths).  The workspace layout never depends on them.
float pool_limit_bins();
float pool_limit_pairs();
bool pool_limits_ever_set();  // kd_set_pool_limits has held a pool below 1 in this process

size_t bin_workspace_bytes(int B, int H, int W, int64_t N, int64_t max_per_view,
                           int ct0 = kCoarseTile0);
// Carves the buffers from `ws` starting at *offset (advanced past them).
BinBuffers bin_carve(void *ws, size_t &offset, int B, int H, int W, int64_t N,
                     int64_t max_per_view, int ct0 = kCoarseTile0);

template <typename T>
hipError_t bin_faces(const FaceSet<T> &fs, const BinBuffers &bb, hipStream_t stream);
template <typename T>
struct PrepOut;  // kd_prep.hpp
// Two face sets of the same views and image (e.g. the raster's and the soft mask's boxes) binned
// by the same three launches (blockIdx.z selects the set).  prep (nullable): the corners are
// computed from the vertices by prepare_vertices' arithmetic in the count launch, which also
// writes its outputs (prep->fvc / fvi / nrm; fs*.fvi must point at prep->fvi).
template <typename T>
hipError_t bin_faces2(const FaceSet<T> &fs0, const BinBuffers &bb0, const FaceSet<T> &fs1,
                      const BinBuffers &bb1, hipStream_t stream,
                      const PrepOut<T> *prep = nullptr);

// Zeroes `bytes` (a multiple of 4) at p with a kernel, not a memset node (graph-capture safe).
hipError_t zero_words(void *p, size_t bytes, hipStream_t stream);
// Zeroes n0 elements at p0 and n1 at p1 (either may be null / 0) in one launch.
template <typename T>
int zero_buffers(T *p0, int64_t n0, T *p1, int64_t n1, hipStream_t stream);

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

}  // namespace kd
