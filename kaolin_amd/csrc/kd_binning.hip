// kd_binning.hip -- see kd_binning.hpp for the algorithm.
#include "kd_binning.hpp"

#include "kd_capi.hpp"

namespace kd {

size_t bin_workspace_bytes(int B, int H, int W, int64_t N, int64_t max_per_view) {
  const BinGeom g = bin_geom(H, W);
  const int64_t nchunk = (max_per_view + kChunk - 1) / kChunk;
  size_t s = 0;
  s += align_up(sizeof(Span) * (size_t)N);
  s += align_up(sizeof(int) * (size_t)B * (size_t)(nchunk > 0 ? nchunk : 1) * g.nct());
  s += align_up(sizeof(int) * (size_t)B * g.nct());
  s += align_up(sizeof(int) * (size_t)g.nct() * (size_t)(N > 0 ? N : 1));
  return s;
}

BinBuffers bin_carve(void *ws, size_t &off, int B, int H, int W, int64_t N,
                     int64_t max_per_view) {
  BinBuffers bb;
  bb.g = bin_geom(H, W);
  bb.nchunk = (int)((max_per_view + kChunk - 1) / kChunk);
  char *base = (char *)ws;
  bb.spans = (Span *)(base + off);
  off += align_up(sizeof(Span) * (size_t)N);
  bb.counts = (int *)(base + off);
  off += align_up(sizeof(int) * (size_t)B * (size_t)(bb.nchunk > 0 ? bb.nchunk : 1) * bb.g.nct());
  bb.totals = (int *)(base + off);
  off += align_up(sizeof(int) * (size_t)B * bb.g.nct());
  bb.bins = (int *)(base + off);
  off += align_up(sizeof(int) * (size_t)bb.g.nct() * (size_t)(N > 0 ? N : 1));
  return bb;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_bin_count(FaceSet<T> fs, BinBuffers bb) {
  __shared__ int s_cnt[kMaxCtiles];
  const int b = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int nct = bb.g.nct();
  for (int c = tid; c < nct; c += kBlock) s_cnt[c] = 0;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  const int64_t i = lo + (int64_t)chunk * kChunk + tid;
  __syncthreads();
  if (i < hi) {
    Span s;
    const bool ok = !fs.valid || fs.valid[i];
    if (ok) {
      T v[6], box[4];
      load_corners(fs, i, v);
      face_box(fs, i, v, box);
      s = make_span<T>(box[0], box[1], box[2], box[3], fs.M, fs.H, fs.W);
    } else {
      s.x0 = 1;
      s.x1 = 0;
      s.y0 = 1;
      s.y1 = 0;
    }
    bb.spans[i] = s;
    if (!span_empty(s)) {
      const int cx0 = s.x0 / bb.g.ct, cx1 = s.x1 / bb.g.ct;
      const int cy0 = s.y0 / bb.g.ct, cy1 = s.y1 / bb.g.ct;
      for (int cy = cy0; cy <= cy1; ++cy)
        for (int cx = cx0; cx <= cx1; ++cx) atomicAdd(&s_cnt[cy * bb.g.nctx + cx], 1);
    }
  }
  __syncthreads();
  int *out = bb.counts + ((int64_t)b * bb.nchunk + chunk) * nct;
  for (int c = tid; c < nct; c += kBlock) out[c] = s_cnt[c];
}

// One workgroup per (coarse tile, view): exclusive scan of counts[b][*][c] over the chunks.
__global__ __launch_bounds__(kBlock) void kd_bin_scan(BinBuffers bb, int B) {
  __shared__ int s_sum[kBlock];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int nct = bb.g.nct();
  const int n = bb.nchunk;
  const int per = (n + kBlock - 1) / kBlock;
  int *base = bb.counts + (int64_t)b * n * nct + c;
  int local = 0;
  for (int k = 0; k < per; ++k) {
    const int j = tid * per + k;
    if (j < n) local += base[(int64_t)j * nct];
  }
  s_sum[tid] = local;
  __syncthreads();
  // Hillis-Steele inclusive scan of the 256 thread sums.
  for (int d = 1; d < kBlock; d <<= 1) {
    const int v = tid >= d ? s_sum[tid - d] : 0;
    __syncthreads();
    s_sum[tid] += v;
    __syncthreads();
  }
  int run = s_sum[tid] - local;  // exclusive prefix of this thread's first chunk
  for (int k = 0; k < per; ++k) {
    const int j = tid * per + k;
    if (j < n) {
      const int v = base[(int64_t)j * nct];
      base[(int64_t)j * nct] = run;
      run += v;
    }
  }
  if (tid == kBlock - 1) bb.totals[(int64_t)b * nct + c] = s_sum[kBlock - 1];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_bin_scatter(FaceSet<T> fs, BinBuffers bb) {
  // 256-bit membership mask per coarse tile: bit t set <=> face (chunk*256 + t) touches it.
  extern __shared__ uint32_t s_mask[];  // [nct][8]
  const int b = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int nct = bb.g.nct();
  for (int k = tid; k < nct * 8; k += kBlock) s_mask[k] = 0u;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  const int64_t i = lo + (int64_t)chunk * kChunk + tid;
  Span s;
  s.x0 = 1;
  s.x1 = 0;
  s.y0 = 1;
  s.y1 = 0;
  if (i < hi) s = bb.spans[i];
  const bool has = !span_empty(s);
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (has) {
    cx0 = s.x0 / bb.g.ct;
    cx1 = s.x1 / bb.g.ct;
    cy0 = s.y0 / bb.g.ct;
    cy1 = s.y1 / bb.g.ct;
  }
  __syncthreads();
  const uint32_t bit = 1u << (tid & 31);
  const int word = tid >> 5;
  for (int cy = cy0; cy <= cy1; ++cy)
    for (int cx = cx0; cx <= cx1; ++cx) atomicOr(&s_mask[(cy * bb.g.nctx + cx) * 8 + word], bit);
  __syncthreads();
  if (!has) return;
  const int *offs = bb.counts + ((int64_t)b * bb.nchunk + chunk) * nct;
  const int local = (int)(i - lo);
  for (int cy = cy0; cy <= cy1; ++cy)
    for (int cx = cx0; cx <= cx1; ++cx) {
      const int c = cy * bb.g.nctx + cx;
      const uint32_t *m = s_mask + c * 8;
      int rank = __popc(m[word] & (bit - 1u));
      for (int k = 0; k < word; ++k) rank += __popc(m[k]);
      bb.bins[(int64_t)c * fs.N + lo + offs[c] + rank] = local;
    }
}

template <typename T>
hipError_t bin_faces(const FaceSet<T> &fs, const BinBuffers &bb, hipStream_t stream) {
  if (bb.nchunk <= 0 || fs.B <= 0) {
    // no faces: totals must still read zero
    return hipMemsetAsync(bb.totals, 0, sizeof(int) * (size_t)(fs.B > 0 ? fs.B : 0) * bb.g.nct(),
                          stream);
  }
  const dim3 grid_c(bb.nchunk, fs.B), grid_t(bb.g.nct(), fs.B);
  {
    ProfScope prof(K_BIN_COUNT, stream);
    hipLaunchKernelGGL(kd_bin_count<T>, grid_c, dim3(kBlock), 0, stream, fs, bb);
  }
  {
    ProfScope prof(K_BIN_SCAN, stream);
    hipLaunchKernelGGL(kd_bin_scan, grid_t, dim3(kBlock), 0, stream, bb, fs.B);
  }
  {
    ProfScope prof(K_BIN_SCATTER, stream);
    hipLaunchKernelGGL(kd_bin_scatter<T>, grid_c, dim3(kBlock),
                       sizeof(uint32_t) * 8 * bb.g.nct(), stream, fs, bb);
  }
  return hipGetLastError();
}

template hipError_t bin_faces<float>(const FaceSet<float> &, const BinBuffers &, hipStream_t);
template hipError_t bin_faces<double>(const FaceSet<double> &, const BinBuffers &, hipStream_t);

}  // namespace kd
