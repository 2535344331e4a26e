// kd_binning.hip -- see kd_binning.hpp for the algorithm.
#include "kd_binning.hpp"
#include "kd_cull.hpp"
#include "kd_prep.hpp"
#include "kd_tile.hpp"

#include "kd_capi.hpp"

#include <type_traits>

namespace kd {

static int64_t fine_tiles(int H, int W) {
  return (int64_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
}

size_t bin_workspace_bytes(int B, int H, int W, int64_t N, int64_t max_per_view, int ct0) {
  const BinGeom g = bin_geom(H, W, ct0);
  // sized for the smaller chunk (the most chunks) whatever bin_chunk picks: the diagnostic flag
  // that forces 256-face chunks may change between a size query and a forward
  const int chunk = kChunk / 2;
  const int64_t nchunk = (max_per_view + chunk - 1) / chunk;
  size_t s = 0;
  s += align_up(sizeof(Span) * (size_t)N);
  s += 2 * align_up(sizeof(int) * (size_t)B * (size_t)(nchunk > 0 ? nchunk : 1) * g.nct());
  s += align_up(sizeof(int) * (size_t)B * g.nct());
  s += align_up(sizeof(int) * (size_t)B * g.nct());
  s += align_up(sizeof(int) * (size_t)kBinEntriesPerFace * (size_t)(N > 0 ? N : 1));
  s += align_up(sizeof(float4) * 2 * (size_t)N);
  s += align_up(sizeof(int2) * (size_t)B * fine_tiles(H, W));
  return s;
}

BinBuffers bin_carve(void *ws, size_t &off, int B, int H, int W, int64_t N,
                     int64_t max_per_view, int ct0) {
  BinBuffers bb;
  bb.g = bin_geom(H, W, ct0);
  bb.chunk = bin_chunk(B, max_per_view);
  bb.nchunk = (int)((max_per_view + bb.chunk - 1) / bb.chunk);
  char *base = (char *)ws;
  bb.spans = (Span *)(base + off);
  off += align_up(sizeof(Span) * (size_t)N);
  bb.counts = (int *)(base + off);
  // (sized like bin_workspace_bytes: for the smaller chunk)
  const size_t ncsz = align_up(sizeof(int) * (size_t)B *
                               (size_t)std::max<int64_t>((max_per_view + kChunk / 2 - 1) / (kChunk / 2), 1) *
                               bb.g.nct());
  off += ncsz;
  bb.offs = (int *)(base + off);
  off += ncsz;
  bb.totals = (int *)(base + off);
  off += align_up(sizeof(int) * (size_t)B * bb.g.nct());
  bb.base = (int *)(base + off);
  off += align_up(sizeof(int) * (size_t)B * bb.g.nct());
  bb.bins = (int *)(base + off);
  bb.xper = kBinEntriesPerFace;
  bb.limit = pool_limit_bins();
  off += align_up(sizeof(int) * (size_t)kBinEntriesPerFace * (size_t)(N > 0 ? N : 1));
  bb.cull = (float4 *)(base + off);
  off += align_up(sizeof(float4) * 2 * (size_t)N);
  bb.order = (int2 *)(base + off);
  off += align_up(sizeof(int2) * (size_t)B * fine_tiles(H, W));
  bb.cull_eps = 0.f;
  bb.hist = nullptr;
  bb.clear = nullptr;
  bb.n_clear = 0;
  bb.clear_b = nullptr;
  bb.n_clear_b = 0;
  return bb;
}

// Edge-culling coefficients of one face for the fp32 pair raster: kd_cull.hpp (the rule and its
// proof; host-compilable for tools/cull_check.cpp).
template <typename T>
__device__ void raster_cull_coefs(const T v[6], float M, int H, int W, Span sp, float eps,
                                  float out[8]) {
  raster_cull_coefs_at<T>(v, M, H, W, sp.x0, sp.y0, sp.y1, eps, out);
}

template <typename T>
struct BinJobs {
  FaceSet<T> fs[2];
  BinBuffers bb[2];
  SpanConsts k[2];  // make_span constants of each set (host-computed)
  PrepOut<T> prep;  // prep.a.vertices set: the corners come from prepare_vertices (kd_bin_count PREP)
};

// One face of one set: its exact span (stored), the raster set's cull coefficients, and its
// coarse tiles counted in LDS.  v: the face's scaled corners (loaded once for both sets).
// nzv (PREP): the face's normal z just computed, used instead of reading fs.nz.
template <typename T>
__device__ __forceinline__ void bin_count_face(const FaceSet<T> &fs, const BinBuffers &bb,
                                               const SpanConsts &k, int64_t i, const T v[6],
                                               int *s_cnt, const T *nzv = nullptr) {
  Span s;
  const bool ok = (!fs.valid || fs.valid[i]) &&
                  (!fs.nz || (nzv ? *nzv : fs.nz[i * fs.nz_stride]) >= (T)0);
  if (ok) {
    T box[4];
    face_box(fs, i, v, box);
    s = make_span_k<T>(box[0], box[1], box[2], box[3], k);
    if (bb.cull && !span_empty(s) && !ablate(fs.dbg, 1 << 18)) {  // fp32 and fp64 (kd_cull.hpp)
      float cc[8];
      raster_cull_coefs<T>(v, fs.M, fs.H, fs.W, s, bb.cull_eps, cc);
      bb.cull[2 * i] = make_float4(cc[0], cc[1], cc[2], cc[3]);
      bb.cull[2 * i + 1] = make_float4(cc[4], cc[5], cc[6], cc[7]);
    }
  } else {
    s.x0 = 1;
    s.x1 = 0;
    s.y0 = 1;
    s.y1 = 0;
  }
  bb.spans[i] = s;
  if (!span_empty(s) && !ablate(fs.dbg, 1 << 19)) {
    const int cx0 = s.x0 >> bb.g.sh, cx1 = s.x1 >> bb.g.sh;
    const int cy0 = s.y0 >> bb.g.sh, cy1 = s.y1 >> bb.g.sh;
    for (int cy = cy0; cy <= cy1; ++cy)
      for (int cx = cx0; cx <= cx1; ++cx) atomicAdd(&s_cnt[cy * bb.g.nctx + cx], 1);
  }
}

// One workgroup per (chunk, view): the chunk's faces in the NS sets (NS = 2: the raster's and
// the soft mask's boxes of the same corners, which are loaded once), their counts per coarse
// tile written tile-major (counts[b][c][chunk]: the scan reads each tile's chunks contiguously).
//
// PREP (dibr_rasterization from vertices): the corners come from prepare_vertices' arithmetic
// (kd_prep.hpp) on the vertices, and the raster set's workgroups (blockIdx.z 0; NS = 2: every
// workgroup) also write its outputs (fvc, fvi, normals; rows staged in LDS, coalesced) -- no
// kd_prepare_fwd launch, no reading the corners back.
template <typename T, int PER, int NS, bool PREP = false>  // PER = chunk / 256 faces per thread
__global__ __launch_bounds__(kBlock) void kd_bin_count(BinJobs<T> jobs) {
  __shared__ int s_cnt[NS][kMaxCtiles];
  __shared__ __align__(16) T s_pc[PREP ? kBlock * 9 : 1];
  __shared__ __align__(16) T s_pi[PREP ? kBlock * 6 : 1];
  __shared__ __align__(16) T s_pn[PREP ? kBlock * 3 : 1];
  const int b = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int z0 = NS == 2 ? 0 : blockIdx.z;  // NS = 1: blockIdx.z selects the set
  const int nct = jobs.bb[z0].g.nct();
#pragma unroll
  for (int z = 0; z < NS; ++z)
    for (int c = tid; c < nct; c += kBlock) s_cnt[z][c] = 0;
  if (b == 0 && chunk == 0) {
#pragma unroll
    for (int z = 0; z < NS; ++z) {
      const BinBuffers &bb = jobs.bb[z0 + z];
      if (bb.clear)
        for (int i = tid; i < bb.n_clear; i += kBlock) bb.clear[i] = 0;
      for (int i = tid; i < bb.n_clear_b; i += kBlock) bb.clear_b[i] = 0;
    }
  }
  int64_t lo, hi;
  view_range(jobs.fs[z0], b, lo, hi);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int64_t i0 = lo + (int64_t)chunk * (PER * kBlock) + u * kBlock;
    const int64_t i = i0 + tid;
    if constexpr (PREP) {
      const FaceSet<T> &fs = jobs.fs[z0];
      if (i < hi) {
        T c[3][3], fi[6], n[3], v[6];
        prep_face_bf<T>(jobs.prep.a, b, i - lo, c, fi, n);  // (row i = view b's face i - lo)
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] = fi[k] * fs.scale;  // load_corners' product
        if (z0 == 0) prep_stage<T>(c, fi, n, s_pc, s_pi, s_pn);
#pragma unroll
        for (int z = 0; z < NS; ++z)
          bin_count_face<T>(jobs.fs[z0 + z], jobs.bb[z0 + z], jobs.k[z0 + z], i, v, s_cnt[z],
                            &n[2]);
      }
      if (z0 == 0 && i0 < hi && !ablate(fs.dbg, 1 << 30)) {  // (workgroup-uniform; diagnostics:
                                                              // 1 << 30 skips the outputs)
        const int rows = (int)min((int64_t)kBlock, hi - i0);
        __syncthreads();
        lds_to_global<T>(jobs.prep.fvc + i0 * 9, s_pc, rows * 9);
        lds_to_global<T>(jobs.prep.fvi + i0 * 6, s_pi, rows * 6);
        lds_to_global<T>(jobs.prep.nrm + i0 * 3, s_pn, rows * 3);
        __syncthreads();
      }
    } else if (i < hi) {
      T v[6];
      load_corners(jobs.fs[z0], i, v);
#pragma unroll
      for (int z = 0; z < NS; ++z)
        bin_count_face<T>(jobs.fs[z0 + z], jobs.bb[z0 + z], jobs.k[z0 + z], i, v, s_cnt[z]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int z = 0; z < NS; ++z) {
    const BinBuffers &bb = jobs.bb[z0 + z];
    int *out = bb.counts + (int64_t)b * nct * bb.nchunk + chunk;
    for (int c = tid; c < nct; c += kBlock) out[(int64_t)c * bb.nchunk] = s_cnt[z][c];
  }
}

// One wave per (coarse tile, view, set), four per workgroup: exclusive scan of counts[b][c][*]
// over the chunks (contiguous: tile-major), written to offs[b][*][c].  Lane l owns the contiguous run of chunks
// [l*per, l*per + per), held in registers; the run sums are scanned with DPP (wave_incl_scan).
// No LDS, no barriers: every wave's loads are in flight at once and the grid is one round on the
// chip.
// (up to 16 waves per workgroup: the chunk-major offsets of 16 consecutive tiles are 64
// contiguous bytes per chunk row -- at 8 views 7.8 -> 7.0 us; small batches keep 4 waves, 16
// would leave too few workgroups: 1 view 6.7 -> 8.0 us)
constexpr int kScanWaves = 16;
template <typename T>
__global__ __launch_bounds__(kScanWaves * kWave) void kd_bin_scan(BinJobs<T> jobs) {
  const BinBuffers &bb = jobs.bb[blockIdx.z];
  const int nct = bb.g.nct();
  const int wv = threadIdx.x >> 6;
  const int c = blockIdx.x * (int)(blockDim.x >> 6) + wv;
  const int b = blockIdx.y, lane = threadIdx.x & (kWave - 1);
  const int n = bb.nchunk;
  const int per = (n + kWave - 1) / kWave;
  const int *base = bb.counts + ((int64_t)b * nct + c) * n;
  // the offsets go out chunk-major (offs[b][j][c]): the four waves of a workgroup write 16
  // contiguous bytes per chunk, and every scatter workgroup then reads one contiguous row
  int *outp = bb.offs + (int64_t)b * n * nct + c;
  constexpr int kMaxPer = 16;  // register-held run (n <= 1024 chunks = 262k faces per view)
  int v[kMaxPer];
  int local = 0;
  const bool live = c < nct;
  if (live && per <= kMaxPer) {
#pragma unroll
    for (int k = 0; k < kMaxPer; ++k) {
      const int j = lane * per + k;
      v[k] = (k < per && j < n) ? base[j] : 0;
      local += v[k];
    }
  } else if (live) {
    for (int k = 0; k < per; ++k) {
      const int j = lane * per + k;
      if (j < n) local += base[j];
    }
  }
  const int incl = wave_incl_scan(local);
  int run = incl - local;  // exclusive prefix of this lane's run
  const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
  if (live && per <= kMaxPer) {
#pragma unroll
    for (int k = 0; k < kMaxPer; ++k) {
      const int j = lane * per + k;
      if (k < per && j < n) {
        outp[(int64_t)j * nct] = run;
        run += v[k];
      }
    }
  } else if (live) {
    for (int k = 0; k < per; ++k) {
      const int j = lane * per + k;
      if (j < n) {
        const int x = base[j];
        outp[(int64_t)j * nct] = run;
        run += x;
      }
    }
  }
  if (live && lane == 0) bb.totals[(int64_t)b * nct + c] = total;
}

template <typename T, int PER>  // PER = chunk / 256 faces per thread
__global__ __launch_bounds__(kBlock, 7) void kd_bin_scatter(BinJobs<T> jobs) {
  const FaceSet<T> &fs = jobs.fs[blockIdx.z];
  const BinBuffers &bb = jobs.bb[blockIdx.z];
  if (blockIdx.x == gridDim.x - 1) {  // the extra column: the set's tile dispatch order
    if (blockIdx.y == 0)
      tile_order(bb, fs.B, (fs.W + kTile - 1) / kTile, (fs.H + kTile - 1) / kTile);
    return;
  }
  // chunk-bit membership mask per coarse tile: bit t set <=> face (chunk * chunk size + t) touches
  // it; each thread holds faces tid (and tid + 256).
  // (rows padded to an odd stride: lanes reading one word of different tiles' masks hit
  // different banks)
  constexpr int kWords = PER * kBlock / 32, kStride = kWords + 1, kPerT = PER;
  extern __shared__ uint32_t s_mask[];  // [nct][kStride]
  __shared__ int s_bbase[kMaxCtiles], s_offs[kMaxCtiles], s_scan[kBlock / kWave];
  const int b = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int nct = bb.g.nct();
  for (int k = tid; k < nct * kStride; k += kBlock) s_mask[k] = 0u;
  // this chunk's exclusive offsets in every tile's bin (kd_bin_scan's chunk-major row), the
  // chunk's spans and (below) the view's totals: all loaded before any of them is waited for
  // (one round trip; staging the offsets into LDS first made it two)
  constexpr int kOffPer = kMaxCtiles / kBlock;
  int ofv[kOffPer];
  {
    const int *offs = bb.offs + ((int64_t)b * bb.nchunk + chunk) * nct;
#pragma unroll
    for (int k = 0; k < kOffPer; ++k) {
      const int c = k * kBlock + tid;
      ofv[k] = c < nct ? offs[c] : 0;
    }
  }
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  Span sp[kPerT];
#pragma unroll
  for (int u = 0; u < kPerT; ++u) {
    const int64_t i = lo + (int64_t)chunk * (PER * kBlock) + u * kBlock + tid;
    sp[u] = Span{1, 0, 1, 0};
    if (i < hi) sp[u] = bb.spans[i];
  }
  {
    // the view's bins in its region [xper*lo, xper*hi): exclusive scan of the totals over the
    // coarse tiles (every workgroup of the view computes the same bases; chunk 0 stores them
    // for the tile kernels); a bin past the usable end of the region overflows (base -1)
    constexpr int kPer = kMaxCtiles / kBlock;
    const int *tot = bb.totals + (int64_t)b * nct;
    int v[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int c = tid * kPer + k;
      v[k] = c < nct ? tot[c] : 0;
      sum += v[k];
    }
#pragma unroll
    for (int k = 0; k < kOffPer; ++k) {
      const int c = k * kBlock + tid;
      if (c < nct) s_offs[c] = ofv[k];
    }
    int all;
    int run = wg_exclusive_scan(sum, s_scan, all);
    const int64_t room = (int64_t)((double)bb.limit * (double)bb.xper * (double)(hi - lo));
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int c = tid * kPer + k;
      if (c < nct) {
        const int bc = (int64_t)run + v[k] <= room ? run : -1;
        s_bbase[c] = bc;
        if (chunk == 0) bb.base[(int64_t)b * nct + c] = bc;
      }
      run += v[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPerT; ++u) {
    if (span_empty(sp[u])) continue;
    const int t = u * kBlock + tid;
    const uint32_t bit = 1u << (t & 31);
    const int word = t >> 5;
    for (int cy = sp[u].y0 >> bb.g.sh; cy <= sp[u].y1 >> bb.g.sh; ++cy)
      for (int cx = sp[u].x0 >> bb.g.sh; cx <= sp[u].x1 >> bb.g.sh; ++cx)
        atomicOr(&s_mask[(cy * bb.g.nctx + cx) * kStride + word], bit);
  }
  __syncthreads();
  const int *offs = s_offs;  // (staged above: counts are tile-major)
  const int *bbase = s_bbase;
  int *bins = bb.bins + (int64_t)bb.xper * lo;
#pragma unroll
  for (int u = 0; u < kPerT; ++u) {
    if (span_empty(sp[u])) continue;
    const int t = u * kBlock + tid;
    const uint32_t bit = 1u << (t & 31);
    const int word = t >> 5;
    const int local = chunk * (PER * kBlock) + t;
    for (int cy = sp[u].y0 >> bb.g.sh; cy <= sp[u].y1 >> bb.g.sh; ++cy)
      for (int cx = sp[u].x0 >> bb.g.sh; cx <= sp[u].x1 >> bb.g.sh; ++cx) {
        const int c = cy * bb.g.nctx + cx;
        const int bc = bbase[c];
        if (bc < 0) continue;  // overflowed: its tiles walk all faces of the view
        const uint32_t *m = s_mask + c * kStride;
        int rank = __popc(m[word] & (bit - 1u));
        for (int k = 0; k < word; ++k) rank += __popc(m[k]);
        bins[bc + offs[c] + rank] = local;
      }
  }
}

// Dispatch order of the tile kernels: (view, fine tile) by descending bit length of its coarse
// bin's face count (a proxy for its work), so the heaviest tiles start first and the grid's
// tail is short.  With a tile history (bb.hist: the fused forward's measured duration buckets of
// the previous same-shape call, per (fine tile, part)), a coarse tile's key is instead the
// largest bucket of its fine tiles' parts (quarter octaves of the duration) -- the soft-mask
// work of a silhouette tile does not show in its bin counts.  Run by one extra 256-thread workgroup of kd_bin_scatter per face set (it only
// needs the scan's totals, so it overlaps the scatter instead of taking a launch of its own):
// one coarse tile (and its <= (ct/16)^2 fine tiles) per thread and pass, histograms and cursors
// per wave.  Order within a bucket follows the (view, coarse tile) index; results never depend
// on the order.  Each entry also carries the coarse bin's face count.
__device__ void tile_order(const BinBuffers &bb, int B, int ntx, int nty) {
  constexpr int kNB = 64, kWaves = kBlock / kWave, kPer = 8;  // buckets: one per lane
  __shared__ int s_cnt[kWaves][kNB];
  __shared__ int s_base, s_next;
  const int tid = threadIdx.x, w = tid >> 6;
  const int nct = bb.g.nct(), n = B * nct;
  const int per = bb.g.ct / kTile;  // fine tiles per coarse tile side
  auto fine_count = [&](int v) {    // fine tiles of (view, coarse tile) v inside the image
    const int c = v % nct;
    const int cx = c % bb.g.nctx, cy = c / bb.g.nctx;
    return (min(cx * per + per, ntx) - cx * per) * (min(cy * per + per, nty) - cy * per);
  };
  if (tid == 0) s_base = 0;
  for (int v0 = 0; v0 < n; v0 += kBlock * kPer) {
    for (int i = tid; i < kWaves * kNB; i += kBlock) (&s_cnt[0][0])[i] = 0;
    __syncthreads();
    int bk[kPer], nf[kPer], tot[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {  // coalesced: consecutive threads, consecutive bins
      const int v = v0 + k * kBlock + tid;
      tot[k] = v < n ? bb.totals[v] : 0;
      bk[k] = v < n ? 32 - __clz((unsigned)tot[k]) : -1;
      nf[k] = v < n ? fine_count(v) : 0;
      if (bb.hist && v < n) {  // the history's bucket when there is one (max over fine tiles)
        const int b = v / nct, c = v - b * nct;
        const int cx = c % bb.g.nctx, cy = c / bb.g.nctx;
        int h = 0;
        for (int ty = cy * per; ty < min(cy * per + per, nty); ++ty)
          for (int tx = cx * per; tx < min(cx * per + per, ntx); ++tx) {
            const uint2 e = *reinterpret_cast<const uint2 *>(
                bb.hist + 4 * ((int64_t)(b * nty + ty) * ntx + tx));  // 4 parts, 8 B aligned
            h = max(h, (int)max(max(e.x & 0xffffu, e.x >> 16), max(e.y & 0xffffu, e.y >> 16)));
          }
        if (h > 0) bk[k] = min(h - 1, kNB - 1);
      }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (bk[k] >= 0) atomicAdd(&s_cnt[w][bk[k]], nf[k]);
    __syncthreads();
    if (w == 0) {  // exclusive offsets, buckets heaviest first then waves: lane = bucket
      const int lane = tid & 63;
      const int kb = kNB - 1 - lane;  // lane 0 = heaviest bucket
      int c[kWaves];
      int t = 0;
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) {
        c[ww] = kb >= 0 ? s_cnt[ww][kb] : 0;
        t += c[ww];
      }
      int run = s_base + wave_incl_scan(t) - t;
      if (kb >= 0) {
#pragma unroll
        for (int ww = 0; ww < kWaves; ++ww) {
          s_cnt[ww][kb] = run;
          run += c[ww];
        }
      }
      const int all = __builtin_amdgcn_readlane(wave_incl_scan(t), 63);
      if (lane == 0) s_next = s_base + all;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (bk[k] < 0) continue;
      const int v = v0 + k * kBlock + tid;
      const int b = v / nct, c = v - b * nct;
      const int cx = c % bb.g.nctx, cy = c / bb.g.nctx;
      int pos = atomicAdd(&s_cnt[w][bk[k]], nf[k]);
      for (int ty = cy * per; ty < min(cy * per + per, nty); ++ty)
        for (int tx = cx * per; tx < min(cx * per + per, ntx); ++tx)
          bb.order[pos++] = make_int2((b * nty + ty) * ntx + tx, tot[k]);
    }
    __syncthreads();
    if (tid == 0) s_base = s_next;
  }
}

template <typename T>
static hipError_t bin_jobs(const BinJobs<T> &jobs_in, int njobs, hipStream_t stream) {
  BinJobs<T> jobs = jobs_in;
  jobs.fs[0].dbg = jobs.fs[1].dbg = debug_flags();  // (diagnostic ablations 1 << 18, 1 << 19)
  const FaceSet<T> &fs = jobs.fs[0];
  const BinBuffers &bb = jobs.bb[0];
  if (bb.nchunk <= 0 || fs.B <= 0) {
    // no faces: totals (and the counters kd_bin_count would clear) must still read zero
    for (int j = 0; j < njobs; ++j) {
      const BinBuffers &b = jobs.bb[j];
      if (b.clear && b.n_clear > 0) {
        const hipError_t e = zero_words(b.clear, sizeof(int) * b.n_clear, stream);
        if (e != hipSuccess) return e;
      }
      if (b.clear_b && b.n_clear_b > 0) {
        const hipError_t e = zero_words(b.clear_b, sizeof(int) * b.n_clear_b, stream);
        if (e != hipSuccess) return e;
      }
      hipError_t e =
          zero_words(b.totals, sizeof(int) * (size_t)(fs.B > 0 ? fs.B : 0) * b.g.nct(), stream);
      if (e != hipSuccess) return e;
      e = zero_words(b.base, sizeof(int) * (size_t)(fs.B > 0 ? fs.B : 0) * b.g.nct(), stream);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const dim3 grid_c(bb.nchunk, fs.B, njobs);
  const int scan_waves = fs.B >= 4 ? kScanWaves : kBlock / kWave;
  const dim3 grid_t((bb.g.nct() + scan_waves - 1) / scan_waves, fs.B, njobs);
  const bool two = bb.chunk == 2 * kBlock;
  // both sets in one workgroup when they share the corners (dibr_rasterization's raster and soft
  // boxes), the corners loaded once: measured slower at C3 (24.6 vs 19.8 us at 8 views, 11.7 vs
  // 7.2 at 1: twice the work per wave at 93 VGPRs), so only on request (debug flag 1 << 21)
  // (not with PREP: that count variant writes prepare_vertices' outputs, this one does not)
  const bool shared = (debug_flags() & (1 << 21)) && njobs == 2 && !jobs.prep.a.vertices &&
                      jobs.fs[0].fvi == jobs.fs[1].fvi &&
                      jobs.fs[0].scale == jobs.fs[1].scale && jobs.fs[0].F == jobs.fs[1].F &&
                      jobs.fs[0].first_idx == jobs.fs[1].first_idx;
  {
    ProfScope prof(K_BIN_COUNT, stream);
    const dim3 grid_s(bb.nchunk, fs.B, 1);
    bool done = false;
    if constexpr (KD_DIAG) {
      if (shared && two)
        hipLaunchKernelGGL((kd_bin_count<T, 2, 2>), grid_s, dim3(kBlock), 0, stream, jobs);
      else if (shared)
        hipLaunchKernelGGL((kd_bin_count<T, 1, 2>), grid_s, dim3(kBlock), 0, stream, jobs);
      done = shared;
    }
    const bool prep = jobs.prep.a.vertices != nullptr;
    if (done) {
    } else if (prep && two)
      hipLaunchKernelGGL((kd_bin_count<T, 2, 1, true>), grid_c, dim3(kBlock), 0, stream, jobs);
    else if (prep)
      hipLaunchKernelGGL((kd_bin_count<T, 1, 1, true>), grid_c, dim3(kBlock), 0, stream, jobs);
    else if (two)
      hipLaunchKernelGGL((kd_bin_count<T, 2, 1>), grid_c, dim3(kBlock), 0, stream, jobs);
    else
      hipLaunchKernelGGL((kd_bin_count<T, 1, 1>), grid_c, dim3(kBlock), 0, stream, jobs);
  }
  {
    ProfScope prof(K_BIN_SCAN, stream);
    hipLaunchKernelGGL(kd_bin_scan<T>, grid_t, dim3(scan_waves * kWave), 0, stream, jobs);
  }
  {  // + one column of workgroups for the tile order (kd_bin_scatter, tile_order)
    // chunk-bit masks per coarse tile: up to 64 KB of dynamic LDS at 1024 coarse tiles (a
    // gfx950 workgroup may hold up to 160 KB; past 64 KB it has to be asked for)
    const size_t dyn = sizeof(uint32_t) * (bb.chunk / 32 + 1) * (size_t)bb.g.nct();
    const void *fn = two ? (const void *)kd_bin_scatter<T, 2> : (const void *)kd_bin_scatter<T, 1>;
    if (dyn > 48 * 1024) {
      const hipError_t ea =
          hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
      if (ea != hipSuccess) return ea;
    }
    ProfScope prof(K_BIN_SCATTER, stream);
    if (two)
      hipLaunchKernelGGL((kd_bin_scatter<T, 2>), dim3(bb.nchunk + 1, fs.B, njobs), dim3(kBlock),
                         dyn, stream, jobs);
    else
      hipLaunchKernelGGL((kd_bin_scatter<T, 1>), dim3(bb.nchunk + 1, fs.B, njobs), dim3(kBlock),
                         dyn, stream, jobs);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t bin_faces(const FaceSet<T> &fs, const BinBuffers &bb, hipStream_t stream) {
  BinJobs<T> jobs{};
  jobs.fs[0] = jobs.fs[1] = fs;
  jobs.bb[0] = jobs.bb[1] = bb;
  jobs.k[0] = jobs.k[1] = span_consts(fs.M, fs.H, fs.W);
  return bin_jobs<T>(jobs, 1, stream);
}

template <typename T>
hipError_t bin_faces2(const FaceSet<T> &fs0, const BinBuffers &bb0, const FaceSet<T> &fs1,
                      const BinBuffers &bb1, hipStream_t stream, const PrepOut<T> *prep) {
  // both sets must describe the same views, faces and image (same chunking and tile grid)
  if (fs0.B != fs1.B || fs0.N != fs1.N || fs0.H != fs1.H || fs0.W != fs1.W ||
      bb0.nchunk != bb1.nchunk || bb0.g.nct() != bb1.g.nct())
    return hipErrorInvalidValue;
  // the projecting count takes view b's rows as [b F, (b + 1) F) (kd_bin_count PREP)
  if (prep && prep->a.vertices && (fs0.first_idx || fs1.first_idx || fs0.F != prep->a.F))
    return hipErrorInvalidValue;
  BinJobs<T> jobs{};
  if (prep) jobs.prep = *prep;
  jobs.fs[0] = fs0;
  jobs.fs[1] = fs1;
  jobs.bb[0] = bb0;
  jobs.bb[1] = bb1;
  jobs.k[0] = span_consts(fs0.M, fs0.H, fs0.W);
  jobs.k[1] = span_consts(fs1.M, fs1.H, fs1.W);
  return bin_jobs<T>(jobs, 2, stream);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_zero2(T *p0, int64_t n0, T *p1, int64_t n1) {
  const int64_t n = n0 + n1;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    if (i < n0)
      p0[i] = (T)0;
    else
      p1[i - n0] = (T)0;
  }
}

template <typename T>
int zero_buffers(T *p0, int64_t n0, T *p1, int64_t n1, hipStream_t stream) {
  if (!p0) n0 = 0;
  if (!p1) n1 = 0;
  const int64_t n = n0 + n1;
  if (n == 0) return KD_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 2048);
  {
    ProfScope prof(K_ZERO, stream);
    hipLaunchKernelGGL(kd_zero2<T>, dim3(blocks), dim3(kBlock), 0, stream, p0, n0, p1, n1);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "zero: %s", hipGetErrorString(e));
  return KD_OK;
}

// Zeroes `bytes` (a multiple of 4) at p with a kernel.  Used instead of hipMemsetAsync wherever a
// call can be captured in a HIP graph: replays of captured memset nodes were measured to leave
// stale data on this stack (tools/dbg_lists_graph.py: the second replay of the close-list soft
// backward summed into an unzeroed gradient), while kernel nodes replay in stream order.
hipError_t zero_words(void *p, size_t bytes, hipStream_t stream) {
  if (!p || bytes == 0) return hipSuccess;
  if (bytes % 4) return hipErrorInvalidValue;
  const int64_t n = (int64_t)(bytes / 4);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 2048);
  {
    ProfScope prof(K_ZERO, stream);
    hipLaunchKernelGGL(kd_zero2<float>, dim3(blocks), dim3(kBlock), 0, stream, (float *)p, n,
                       (float *)nullptr, (int64_t)0);
  }
  return hipGetLastError();
}

template hipError_t bin_faces2<float>(const FaceSet<float> &, const BinBuffers &,
                                      const FaceSet<float> &, const BinBuffers &, hipStream_t,
                                      const PrepOut<float> *);
template hipError_t bin_faces2<double>(const FaceSet<double> &, const BinBuffers &,
                                       const FaceSet<double> &, const BinBuffers &, hipStream_t,
                                       const PrepOut<double> *);
template int zero_buffers<float>(float *, int64_t, float *, int64_t, hipStream_t);
template int zero_buffers<double>(double *, int64_t, double *, int64_t, hipStream_t);
template hipError_t bin_faces<float>(const FaceSet<float> &, const BinBuffers &, hipStream_t);
template hipError_t bin_faces<double>(const FaceSet<double> &, const BinBuffers &, hipStream_t);

}  // namespace kd
