// kd_softpair.hip -- the autograd path of dibr_soft_mask (dibr.py:27-73) as a pair pipeline.
//
// The reference's per-pixel loop (dibr_soft_mask_cuda.cu:27-184) spends its time in two places:
// finding each uncovered pixel's first K close faces, and the distance / probability math of
// those (pixel, face) pairs.  Only pixels near the silhouette have pairs (~8 % of the pixels,
// ~16 pairs each at C3).
//   kd_soft_pairs<FUSED>  one workgroup per 16x16 tile: walks the tile's ordered bin
//                      (kd_tile.hpp); pass A picks each uncovered pixel's first K close faces by
//                      face index and writes (pixel, slot, face) records into the tile's room
//                      of the record pool (SoftPairBuf, kd_soft.hpp), stopping once every
//                      uncovered pixel holds K.
//                      FUSED (knum <= 32, no close lists): the same workgroup then does the pair
//                      math over its records (distance type and probability, bit-identical to
//                      the reference) and the ordered product soft = 1 - prod(1 - p)
//                      (dibr_soft_mask_cuda.cu:174-181, double-promoted) -- the whole soft mask
//                      in one launch.
//   kd_soft_pair_math, kd_soft_reduce   the same math and product as separate launches, for
//                      the op form with the reference's close-face lists (and knum > 32).
//   kd_soft_bwd_items  the backward, flat over (tile, 256-record) items.
//   kd_soft_ovf_fwd / kd_soft_ovf_bwd   the tiles whose room did not fit the pool.
//   kd_dibr_fwd_tiles  dibr_rasterization's forward: per tile, the raster pair pipeline
//                      (kd_raster_pairs.hpp) and then the FUSED soft mask of the same tile.
//   kd_dibr_bwd        dibr_rasterization's backward: the raster backward's tiles
//                      (kd_raster_bwd.hpp) and the soft items in one grid.
// Pool overflow (tiles reserving more than the pool's min(knum, 32) records per pixel, or
// kd_set_pool_limits): the tile writes no records; kd_soft_ovf_fwd runs its walk again, each
// pixel lane computing its pairs' probabilities in slot order and the product directly
// ("streaming": the reference's per-pixel loop over the tile's face list), so the soft mask is
// bit-identical; kd_soft_ovf_bwd walks it again for the backward.
// Backward factorisation: the reference's per-pair gradient (dibr_soft_mask_cuda.cu:281-348) is
//   dLdz * f_j / M  with  dLdz = -sigmainv * dLdp * (1 - soft) / (1 - p + 1e-7) * p
// and f_j the geometric factors of the distance type (2(x1 - x0) ... for a vertex, the four
// dzdA / dzdB / dzdC combinations for an edge).  Only s_p = -sigmainv * dLdp * (1 - soft)
// depends on the incoming gradient: the backward computes h_j = p / (1 - p + 1e-7) * f_j / M from
// the record (face corners, distance type, the forward's probability) and adds s_p * h_j per
// coordinate (same value up to rounding order, like the reference's own atomics).  The close
// lists are never needed.
#include "kd_raster_bwd.hpp"
#include "kd_raster_pairs.hpp"
#include "kd_soft.hpp"

namespace kd {

constexpr unsigned kMathBlocks = 8192;  // pair-math / backward-item grid

// Records of the pool: min(knum, kPoolPairsPerPixel) per tile pixel (every tile fits when
// knum <= 32).
static int64_t pool_records(int B, int H, int W, int K) {
  const int64_t ntiles = (int64_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
  return (int64_t)B * ntiles * kBlock * std::min(K, kPoolPairsPerPixel);
}

size_t soft_pair_workspace_bytes(int B, int H, int W, int64_t N, int64_t F, int K, int esize,
                                 int ct0) {
  const int64_t ntiles = (int64_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
  const int64_t tiles = (int64_t)B * ntiles, P = (int64_t)B * H * W;
  const int64_t recs = pool_records(B, H, W, K);
  size_t s = bin_workspace_bytes(B, H, W, N, F, ct0);
  s += align_up(sizeof(SoftPairRec) * (size_t)recs);
  s += align_up((size_t)esize * (size_t)recs);
  s += align_up(sizeof(int64_t) * (size_t)tiles);
  s += align_up(sizeof(int32_t) * (size_t)P);
  s += align_up(sizeof(int32_t) * (size_t)tiles);
  // items: a tile's n records take ceil(n / 256) items.  Overflow entries: up to one per tile.
  s += align_up(sizeof(PairItem) * (size_t)(recs / kBlock + tiles));
  s += align_up(sizeof(int32_t) * (size_t)tiles);
  s += align_up(sizeof(int32_t) * (size_t)tiles);
  s += align_up(sizeof(int32_t) * kPairClear);  // counters and the record cursor
  return s;
}

template <typename T>
SoftPairBuf<T> soft_pair_carve(void *ws, size_t &off, int B, int H, int W, int K) {
  SoftPairBuf<T> pb;
  pb.ntx = (W + kTile - 1) / kTile;
  pb.ntiles = (int64_t)pb.ntx * ((H + kTile - 1) / kTile);
  pb.cap = pool_records(B, H, W, K);
  pb.lim = (int64_t)((double)pool_limit_pairs() * (double)pb.cap);
  pb.fixed = K <= kPoolPairsPerPixel && pb.lim >= pb.cap;
  const int64_t tiles = (int64_t)B * pb.ntiles, P = (int64_t)B * H * W;
  pb.npixels = P;
  char *base = (char *)ws;
  pb.rec = (SoftPairRec *)(base + off);
  off += align_up(sizeof(SoftPairRec) * (size_t)pb.cap);
  pb.sprob = (T *)(base + off);
  off += align_up(sizeof(T) * (size_t)pb.cap);
  pb.tbase = (int64_t *)(base + off);
  off += align_up(sizeof(int64_t) * (size_t)tiles);
  pb.npix = (int32_t *)(base + off);
  off += align_up(sizeof(int32_t) * (size_t)P);
  pb.ntile = (int32_t *)(base + off);
  off += align_up(sizeof(int32_t) * (size_t)tiles);
  pb.items = (PairItem *)(base + off);
  pb.icap = pb.cap / kBlock + tiles;
  off += align_up(sizeof(PairItem) * (size_t)pb.icap);
  pb.tiles = (int32_t *)(base + off);
  off += align_up(sizeof(int32_t) * (size_t)tiles);
  pb.ovf = (int32_t *)(base + off);
  off += align_up(sizeof(int32_t) * (size_t)tiles);
  pb.counters = (int32_t *)(base + off);
  pb.cursor = (unsigned long long *)(pb.counters + 4);
  off += align_up(sizeof(int32_t) * kPairClear);
  return pb;
}

// pixel of tile-local thread index q (kd_tile.hpp tile_geom layout)
__device__ __forceinline__ void tile_pixel(int tx, int ty, int q, int &px, int &py) {
  const int w = q >> 6, l = q & 63;
  px = tx * kTile + (w & 1) * 8 + (l & 7);
  py = ty * kTile + (w >> 1) * 8 + (l >> 3);
}

// ------------------------------------------------------------------------------------------
// pass A: (pixel, slot, face) records per tile
// ------------------------------------------------------------------------------------------
// Lowest `need` set bits of m (0 <= need < popc(m)): binary search for the need-th set bit.
__device__ __forceinline__ uint64_t lowest_bits(uint64_t m, int need) {
  if (need <= 0) return 0ull;
  int pos = 0, left = need;  // find the bit position of the need-th set bit (1-based)
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t lowmask = (w == 64) ? ~0ull : ((1ull << w) - 1ull);
    const int c = __popcll((m >> pos) & lowmask);
    if (c < left) {
      left -= c;
      pos += w;
    }
  }
  // bit `pos` is the need-th set bit: keep bits 0..pos
  return m & ((pos >= 63) ? ~0ull : ((2ull << pos) - 1ull));
}

// The faces of one 64-face chunk of a wave's sub-list (lane j = chunk entry j) this pixel lane
// takes: the first K - kid whose exact enlarged span holds its centre (ascending face index =
// ascending entry, dibr_soft_mask_cuda.cu:95 and :165-171).
// The faces of chunk c of sub-list s (lane j = entry c*64 + j) whose exact enlarged span holds
// this pixel lane's centre (pixel (ox + (lane & 7), oy + (lane >> 3))).  Every lane of the wave
// must call it (its ballots gather the chunk's faces from all lanes).
__device__ __forceinline__ uint64_t chunk_hits(const TileLists &L, int s, int nsub, int c, int ox,
                                               int oy) {
  const int lane = threadIdx.x & 63;
  const int qx = lane & 7, qy = lane >> 3;
  const int j = c * kWave + lane;
  const bool has = j < nsub;
  const int k = has ? L.sub[s][j] : 0;
  const Span sp = has ? L.span[k] : Span{1, -1, 1, -1};
  const int x0 = sp.x0 - ox, x1 = sp.x1 - ox, y0 = sp.y0 - oy, y1 = sp.y1 - oy;
  uint64_t mc = 0ull, mr = 0ull;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t bc = __ballot(x0 <= i && i <= x1);
    const uint64_t br = __ballot(y0 <= i && i <= y1);
    mc = (qx == i) ? bc : mc;
    mr = (qy == i) ? br : mr;
  }
  return mc & mr;
}

__device__ __forceinline__ uint64_t chunk_select(const TileLists &L, int nsub, int c, bool unc,
                                                 int K, const TileGeom &t, int kid) {
  const int w = threadIdx.x >> 6;
  uint64_t sel = chunk_hits(L, w, nsub, c, t.WX0, t.WY0);
  sel = (unc && kid < K) ? sel : 0ull;
  if (__popcll(sel) > K - kid) sel = lowest_bits(sel, K - kid);
  return sel;
}

// One 64-face chunk of a wave's sub-list: each uncovered pixel lane takes its chunk_select faces.
// Records are placed face-major (face j's pixels contiguous, pixels ascending): the transposed
// selections give each face its record count and offset; each pixel lane then writes its own
// records (slot = its running close-face count) at offset[j] + rank of the pixel in face j.
// The record writes of one chunk for a selection `sel` (pixel lane: its faces of the chunk),
// slots from my_kid on (advanced).  tile_q: the pixel's thread index in the 16x16 tile frame (the
// record's q); ridx_q: its column of the (slot, pixel) record table.
// The face lanes' pixel masks, first records and face rows reach the pixel lanes through lane
// permutes (ds_bpermute: no LDS allocation -- 4 KB less per workgroup than staging them, which
// lets a seventh workgroup onto a CU); the permute loop runs wave-uniform, so every source lane
// is active.
__device__ __forceinline__ void soft_chunk_write(const TileLists &L, int ls, uint64_t sel, int c,
                                                 int64_t lo, int &my_kid, int *s_nrec,
                                                 SoftPairRec *rec,
                                                 unsigned short (*s_ridx)[kBlock], int tile_q,
                                                 int ridx_q) {
  const int lane = threadIdx.x & 63;
  // face lanes: pixel masks, record counts and offsets
  const uint64_t pm = wave_transpose64(sel);
  const int cnt = __popcll(pm);
  const int incl = wave_incl_scan(cnt);
  const int tot = __builtin_amdgcn_readlane(incl, 63);
  if (tot == 0) return;
  int base = 0;
  if (lane == 0) base = atomicAdd(s_nrec, tot);
  // the face lane's row (its entry of the chunk) and first record
  const int row = cnt ? (int)(lo + L.f[L.sub[ls][c * kWave + lane]]) : 0;
  base = __builtin_amdgcn_readfirstlane(base);
  const int first = base + incl - cnt;
  const int pml = (int)(uint32_t)pm, pmh = (int)(uint32_t)(pm >> 32);
  // pixel lanes: write own records, slots ascending with the face index, two selected faces per
  // step with every permute issued before the first store; a record is one 8-byte store
  const uint64_t below = (1ull << lane) - 1ull;
  unsigned long long *rec8 = reinterpret_cast<unsigned long long *>(rec);
  const unsigned long long qbits = (unsigned long long)(uint8_t)tile_q << 48;
  int slot = my_kid;
  for (uint64_t m = sel; __ballot(m != 0ull);) {
    constexpr int U = 2;
    int jj[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      jj[u] = m ? (int)__builtin_ctzll(m) : -1;
      m &= m - 1ull;  // (0 stays 0)
    }
    int off[U], rw[U];
    uint64_t pmu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int a = (jj[u] < 0 ? 0 : jj[u]) << 2;  // (byte address of the source lane)
      off[u] = __builtin_amdgcn_ds_bpermute(a, first);
      rw[u] = __builtin_amdgcn_ds_bpermute(a, row);
      pmu[u] = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(a, pml) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(a, pmh) << 32);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (jj[u] >= 0) {
        const int ri = off[u] + __popcll(pmu[u] & below);
        // SoftPairRec {row, slot, q, type = 0} as one little-endian 64-bit word
        rec8[ri] = (unsigned long long)(uint32_t)rw[u] |
                   ((unsigned long long)(uint16_t)(slot + u) << 32) | qbits;
        if (s_ridx) s_ridx[slot + u][ridx_q] = (unsigned short)ri;  // (slot, pixel) -> record
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) slot += jj[u] >= 0;
  }
  my_kid = slot;
  wave_lds_sync();
}

__device__ __forceinline__ void soft_chunk_records(const TileLists &L, int nsub, int c, bool unc,
                                                   int K, const TileGeom &t, int64_t lo,
                                                   int &my_kid, int *s_nrec, SoftPairRec *rec,
                                                   unsigned short (*s_ridx)[kBlock] = nullptr) {
  const int tile_q = threadIdx.x;
  const uint64_t sel = chunk_select(L, nsub, c, unc, K, t, my_kid);
  soft_chunk_write(L, threadIdx.x >> 6, sel, c, lo, my_kid, s_nrec, rec, s_ridx, tile_q, tile_q);
}

// The streaming form of one chunk (a tile without records): the pixel lane visits the same
// faces in slot order and hands each (face row, slot) to fn.
template <typename PairFn>
__device__ __forceinline__ void soft_chunk_stream(const TileLists &L, int nsub, int c, bool unc,
                                                  int K, const TileGeom &t, int64_t lo,
                                                  int &my_kid, PairFn fn) {
  const int w = threadIdx.x >> 6;
  for (uint64_t sel = chunk_select(L, nsub, c, unc, K, t, my_kid); sel; sel &= sel - 1ull) {
    const int kk = L.sub[w][c * kWave + __builtin_ctzll(sel)];
    fn(lo + L.f[kk], my_kid++);
  }
}

// The soft mask of the tiles whose pass A found the pool exhausted (kd_soft_pairs dropped
// their records): each uncovered pixel lane walks its first K close faces in slot order and
// multiplies their probabilities into its product -- the reference's per-pixel loop over the
// tile list, bit-identical to the pair pipeline; the split pipeline also gets its lists here.
// One workgroup per such tile; a grid that finds none exits at once.
template <typename T, bool FUSED>
__global__ __launch_bounds__(kBlock) void kd_soft_ovf_fwd(SoftArgs<T> a, SoftPairBuf<T> pb) {
  __shared__ TileLists L;
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const float M = fs.M;
  const int novf = pb.counters[2];
  for (int i = blockIdx.x; i < novf; i += gridDim.x) {
    const int64_t tile = pb.ovf[i];
    const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
    int64_t lo, hi;
    view_range(fs, b, lo, hi);
    const TileGeom t = tile_geom(H, W, tl);
    const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
    const bool unc = t.inimg && a.face_idx[p] < 0;
    const bool wave_unc = __ballot(unc) != 0ull;
    const T x0 = (T)px_cx(M, W, t.px), y0 = (T)px_cy(M, H, t.py);
    int my_kid = 0;
    T prod = (T)1.0;
    auto stage = [&](int, int64_t) {};
    auto round = [&](int nsub, int) {
      if (wave_unc)
        for (int c = 0; c * kWave < nsub; ++c)
          soft_chunk_stream(L, nsub, c, unc, K, t, lo, my_kid, [&](int64_t row, int slot) {
            T v[6];
            load_corners(fs, row, v);
            int et = 0;
            T prob = (T)0;
            soft_face_dist<T>(x0, y0, v, M, a.sigmainv, et, prob);
            prod = (T)((double)prod * (1.0 - (double)prob));
            if (!FUSED) {
              if (a.prob) {
                a.prob[p * K + slot] = prob;
                a.cidx[p * K + slot] = row - lo;
                a.ctype[p * K + slot] = (uint8_t)(et + 1);
              }
              if (a.last && slot == K - 1) a.last[p] = (int32_t)(row - lo);
            }
          });
    };
    auto done = [&]() { return __syncthreads_and(!unc || my_kid >= K) != 0; };
    if (__syncthreads_or(unc))
      tile_rounds(L, a.bb, (int)(hi - lo), b, lo, t, stage, round, fs.dbg, done);
    if (unc && my_kid > 0 && a.soft) a.soft[p] = (T)(1.0 - (double)prod);
    if (!FUSED && a.prob && t.inimg) pb.npix[p] = my_kid;  // (the lists' row lengths)
    if (!FUSED && a.prob && t.inimg)
      for (int s = my_kid; s < K; ++s) {  // the -1 / 0 / 0 padding (kd_soft_lists skips the tile)
        a.prob[p * K + s] = (T)0;
        a.cidx[p * K + s] = -1;
        a.ctype[p * K + s] = 0;
      }
    __syncthreads();
  }
}

// Records of one tile's pixel set (pass A).  FUSED (knum <= kFuseSlots, no close-face lists):
// the same workgroup then runs the pair math over its own records and the ordered product of
// each pixel's slots -- the whole soft mask in one launch.  Pass A notes each (slot, pixel)'s
// record in LDS, so the product reads the probabilities in slot order.
// mask_iou fused into the soft mask (SoftArgs::iou_gt): this tile's share of its view's
// U_b = sum(s g) and D_b = sum(s + g - s g), the per-pixel terms in T as kaolin/metrics/
// render.py:35-38 forms them (kd_metrics.hip iou_terms), summed in fp64 over the tile and added
// to one of the view's kIouParts accumulator pairs with one fp64 atomic each.  s_red: 8 doubles
// of LDS.
template <typename T>
__device__ __forceinline__ void iou_tile_terms(const SoftArgs<T> &a, int b, int tl, int64_t p,
                                               bool in, T s, double *s_red) {
  if (!a.iou_gt) return;
  double u = 0.0, d = 0.0;
  if (in) {
    const T g = a.iou_gt[p];
    const T mul = s * g, add = s + g;
    u = (double)mul;
    d = (double)(add - mul);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    u += __shfl_xor(u, o);
    d += __shfl_xor(d, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[w] = u;
    s_red[4 + w] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // partials spread the atomics of a view's tiles over 32 lines
    double *acc = a.iou_acc + 2 * ((int64_t)b * kIouParts + (tl & (kIouParts - 1)));
    atomicAdd(acc, s_red[0] + s_red[1] + s_red[2] + s_red[3]);
    atomicAdd(acc + 1, s_red[4] + s_red[5] + s_red[6] + s_red[7]);
  }
}

// Side job of the fused forward launches: the backward's gradient buffers, zeroed grid-stride
// (coalesced) by every workgroup of the grid -- also by those without a tile.
// (16-byte stores where the buffer is 16-byte aligned, element stores for the rest)
template <typename T>
__device__ __forceinline__ void zero_range(T *p, int64_t n, int64_t gtid, int64_t gstride) {
  if (!p || n <= 0) return;
  int64_t done = 0;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    constexpr int E = 16 / (int)sizeof(T);
    const int64_t nv = n / E;
    float4 *q = reinterpret_cast<float4 *>(p);
    for (int64_t i = gtid; i < nv; i += gstride) q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    done = nv * E;
  }
  for (int64_t i = done + gtid; i < n; i += gstride) p[i] = (T)0;
}
template <typename T>
__device__ __forceinline__ void zero_side_job(const SoftArgs<T> &a) {
  const int64_t gstride = (int64_t)gridDim.x * gridDim.y * kBlock;
  const int64_t gtid = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kBlock + threadIdx.x;
  zero_range<T>(a.zero0, a.nzero0, gtid, gstride);
  zero_range<T>(a.zero1, a.nzero1, gtid, gstride);
}

template <bool FUSED>
struct SoftPairsLDS {
  unsigned short ridx[FUSED ? kFuseSlots : 1][kBlock];
  TileLists L;
  int64_t base;
  int nrec, ibase, box[4];
  double iou[8];  // iou_tile_terms
  int wbox[4][4];   // per wave: the box of its pixels that can still take a face (walk filter)
  unsigned char gcnt[2][4][kWave];  // split tiles: per wave, each pixel's hits of its chunk
};

// Tile tl of view b (nbin: faces of its soft coarse bin, or -1).  Each thread owns pixel
// (t.px, t.py) of tile_geom(H, W, tl); a.face_idx of that pixel is read by the same thread (the
// fused forward wrote it in the same workgroup, same thread).
//
// The pair math of records [i0, i1) of the tile whose records start at `base` (tile column tx,
// row ty): distance type and probability, bit-identical to the reference (kd_softdist.hpp).
//
// pt (nullable; split tiles): the part's LDS probability table [slot][q - q0] (row stride ptw),
// so that the product reads each pixel's probabilities in slot order from LDS.
// R records per thread and pass, their record and corner loads issued together (R = 2 for the
// split tiles of small batches, whose heavy tiles run alone at the end of the launch: the loop is
// bound by its two dependent loads per record there; at 8 views it is VALU-bound and R = 1).
template <typename T, int R = 1>
__device__ __forceinline__ void pair_math_range(const SoftArgs<T> &a, const SoftPairBuf<T> &pb,
                                                int64_t base, int tx, int ty, int i0, int i1,
                                                T *pt = nullptr, int q0 = 0, int ptw = 0) {
  const FaceSet<T> &fs = a.fs;
  const float M = fs.M;
  const SoftPairRec *rec = pb.rec + base;
  T *sp = pb.sprob + base;
  for (int i = i0 + (int)threadIdx.x; i < i1 && !ablate(fs.dbg, 32); i += R * kBlock) {
    SoftPairRec r[R];
    bool ok[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      ok[u] = u == 0 || i + u * kBlock < i1;
      r[u] = rec[ok[u] ? i + u * kBlock : i];
    }
    T v[R][6];
#pragma unroll
    for (int u = 0; u < R; ++u) load_corners(fs, (int64_t)r[u].row, v[u]);
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (!ok[u]) break;
      int px, py;
      tile_pixel(tx, ty, r[u].q, px, py);
      const T x0 = (T)px_cx(M, fs.W, px), y0 = (T)px_cy(M, fs.H, py);
      int et = 0;
      T prob = (T)0;
      soft_face_dist<T>(x0, y0, v[u], M, a.sigmainv, et, prob);
      const int ii = i + u * kBlock;
      sp[ii] = prob;
      pb.rec[base + ii].type = (uint8_t)et;
      if (pt) pt[(int)r[u].slot * ptw + ((int)r[u].q - q0)] = prob;
      // (no backward coefficients here: kd_soft_bwd_items computes them from the record)
    }
  }
}

// SPLIT > 1 (FUSED, fixed pool only; kd_tile.hpp tile_geom_part): the workgroup is part `part`
// of the tile, with its own room of the tile's records (the part's pixels x K) and its own work
// items; records keep the tile frame's pixel index q.  Pass A takes a sub-tile's chunks in groups
// of SPLIT, chunk g * SPLIT + r by role r: each role counts its pixels' hits, and after one barrier
// every role knows the hits of the roles before it, so a pixel's slots stay in face order (its
// first K).  Role 0 forms the product and writes the pixel outputs.  uncm (nullptr: read
// face_idx): per sub-tile, the mask of uncovered in-image pixels (the fused raster phase's).
// CLK (diagnostics, kd_dibr_fwd_tiles<true>): wave 0's pass-A cycle counts into clk[(i) * slots
// + slot]: [0] round (hits, selection, record writes) [1] record writes [2] done() [3] batches
// [4] chunks [5] faces through the filter [6] records of the workgroup [7] pass A
template <typename T, bool FUSED, int SPLIT = 1, bool CLK = false>
__device__ __forceinline__ void soft_pairs_tile(const SoftArgs<T> &a, const SoftPairBuf<T> &pb,
                                                int b, int tl, int nbin, SoftPairsLDS<FUSED> &S,
                                                int part = 0, const uint64_t *uncm = nullptr,
                                                long long *clk = nullptr,
                                                int bbase = kNoBinBase) {
  static_assert(SPLIT == 1 || FUSED, "split tiles: the fused soft mask only");
  TileLists &L = S.L;
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  const int nview = (int)(hi - lo);
  TileGeom t = SPLIT == 1 ? tile_geom(H, W, tl) : tile_geom_part<SPLIT>(H, W, tl, part);
  t.nbin = nbin;
  t.bbase = bbase;
  const int tile_q = t.sub * kWave + lane;  // the pixel's index in the 16x16 tile frame
  if (KD_DIAG && fs.tbuf && tid == 0 && nbin >= 0)  // diagnostics: (view, tile, bin) of the slot
    fs.tbuf[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] =
        ((long long)nbin << 32) | (long long)(b * pb.ntiles + tl);
  const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
  const bool unc = t.inimg && (uncm ? ((uncm[t.sub] >> lane) & 1ull) != 0ull : a.face_idx[p] < 0);
  const bool wave_unc = __ballot(unc) != 0ull;
  const bool owner = t.role == 0;  // this lane writes the pixel's outputs
  const int64_t tile = (int64_t)b * pb.ntiles + tl;
  int my_kid = 0;

  // faces matter only where they reach an uncovered pixel: the filter boxes of tile_rounds
  // shrink to the uncovered pixels' bounding boxes (exact: a record needs the pixel centre
  // inside the face's enlarged span)
  int *s_box = S.box;
  if (tid == 0) {
    s_box[0] = s_box[2] = 1 << 30;
    s_box[1] = s_box[3] = -1;
    S.nrec = 0;
    S.base = -1;
  }
  {
    const uint64_t um = __ballot(unc);
    t.wave_live = t.wave_live && um != 0ull;
    if (um) {
      uint32_t cols = 0u;
#pragma unroll
      for (int r = 0; r < 8; ++r) cols |= (uint32_t)(um >> (8 * r)) & 0xffu;
      t.SX0 = t.WX0 + __builtin_ctz(cols);
      t.SX1 = t.WX0 + 31 - __builtin_clz(cols);
      t.SY0 = t.WY0 + __builtin_ctzll(um) / 8;
      t.SY1 = t.WY0 + (63 - __builtin_clzll(um)) / 8;
    }
  }
  __syncthreads();
  if (t.wave_live && lane == 0) {
    atomicMin(&s_box[0], t.SX0);
    atomicMax(&s_box[1], t.SX1);
    atomicMin(&s_box[2], t.SY0);
    atomicMax(&s_box[3], t.SY1);
  }
  const int U = __syncthreads_count(unc);
  bool ovf = false;
  if (U > 0) {
    // the tile's room in the pool: its own 256 K records (`fixed`), or, reserved with one device
    // atomic, min(K, faces of the tile's soft coarse bin) per uncovered pixel; the atomic's
    // latency overlaps the walk's first loads (records are written after a barrier of
    // tile_rounds)
    if (pb.fixed) {
      if (tid == 0) S.base = tile * kBlock * K + (int64_t)part * (kBlock / SPLIT) * K;
    } else if (tid == 0) {
      const BinGeom &g = a.bb.g;
      const int ct = (t.Y0 >> g.sh) * g.nctx + (t.X0 >> g.sh);
      int nb;
      bin_list(a.bb, b, ct, lo, nview, nbin, nb);
      const int64_t room = (int64_t)U * (int64_t)min(K, nb);
      if (room > 0) {
        const int64_t b0 = (int64_t)atomicAdd(pb.cursor, (unsigned long long)room);
        S.base = b0 + room <= pb.lim ? b0 : -2;  // -2: the pool is exhausted
      }
    }
    t.FX0 = s_box[0];
    t.FX1 = s_box[1];
    t.FY0 = s_box[2];
    t.FY1 = s_box[3];
    auto stage = [&](int, int64_t) {};  // pass A needs the spans only
    long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto now_clk = [&]() -> long long {
      return CLK ? (long long)__builtin_readcyclecounter() : 0ll;
    };
    const long long pa0 = now_clk();
    auto round = [&](int nsub, int ncnt) {
      const long long r0 = now_clk();
      if (CLK) {
        cyc[3] += 1;
        cyc[5] += ncnt;
      }
      if constexpr (SPLIT == 1) {
        if (wave_unc && !ablate(fs.dbg, 1024)) {
          for (int c = 0; c * kWave < nsub; ++c) {
            if constexpr (CLK) {
              cyc[4] += 1;
              const uint64_t sel = chunk_select(L, nsub, c, unc, K, t, my_kid);
              const long long w0 = now_clk();
              soft_chunk_write(L, w, sel, c, lo, my_kid, &S.nrec, pb.rec + S.base,
                               FUSED ? S.ridx : nullptr, tid, tid);
              cyc[1] += now_clk() - w0;
            } else {
              soft_chunk_records(L, nsub, c, unc, K, t, lo, my_kid, &S.nrec, pb.rec + S.base,
                                 FUSED ? S.ridx : nullptr);
            }
          }
        }
        if (CLK) cyc[0] += now_clk() - r0;
      } else {
        // groups of SPLIT chunks (a workgroup-uniform count: every wave meets the barriers)
        const int nmax = max(max(L.nsub[0], L.nsub[1]), max(L.nsub[2], L.nsub[3]));
        constexpr int NS = 4 / SPLIT;
        for (int g = 0; g * SPLIT * kWave < nmax; ++g) {
          const int c = g * SPLIT + t.role;
          const bool mine = wave_unc && c * kWave < nsub;  // (wave-uniform)
          uint64_t hits = mine ? chunk_hits(L, w, nsub, c, t.WX0, t.WY0) : 0ull;
          hits = (unc && my_kid < K) ? hits : 0ull;
          const int cnt = __popcll(hits);
          S.gcnt[g & 1][w][lane] = (unsigned char)cnt;
          __syncthreads();
          int before = 0, all = 0;
#pragma unroll
          for (int r = 0; r < SPLIT; ++r) {
            const int x = S.gcnt[g & 1][r * NS + w % NS][lane];
            before += r < t.role ? x : 0;
            all += x;
          }
          int slot = my_kid + before;
          const int take = min(cnt, max(K - slot, 0));
          const uint64_t sel = take < cnt ? lowest_bits(hits, take) : hits;
          const long long w0 = now_clk();
          if (mine)  // (split tiles: no record table -- the pair math fills a probability table)
            soft_chunk_write(L, w, sel, c, lo, slot, &S.nrec, pb.rec + S.base, nullptr, tile_q,
                             tile_q);
          if (CLK) {
            cyc[1] += now_clk() - w0;
            cyc[4] += mine ? 1 : 0;
          }
          my_kid = min(K, my_kid + all);
        }
        if (CLK) cyc[0] += now_clk() - r0;
      }
    };
    // once every uncovered pixel holds K close faces, later faces cannot enter; a tile without
    // room in the pool stops at the first barrier.  Otherwise the walk's filter boxes shrink to
    // the pixels that can still take a face (uncovered, fewer than K so far): a later face whose
    // enlarged span reaches none of them cannot enter any list, so the next batches' tile list
    // and sub-lists hold only faces that can (exact, like the first filter)
    auto done = [&]() {
      const long long d0 = now_clk();
      struct Acc {
        long long &c, t0;
        bool on;
        __device__ ~Acc() {
          if (on) c += (long long)__builtin_readcyclecounter() - t0;
        }
      } acc{cyc[2], d0, CLK};
      const bool open = unc && my_kid < K;
      const uint64_t om = __ballot(open);
      int bx0 = 1 << 30, bx1 = -1, by0 = 1 << 30, by1 = -1;
      if (om) {
        uint32_t cols = 0u;
#pragma unroll
        for (int r = 0; r < 8; ++r) cols |= (uint32_t)(om >> (8 * r)) & 0xffu;
        bx0 = t.WX0 + __builtin_ctz(cols);
        bx1 = t.WX0 + 31 - __builtin_clz(cols);
        by0 = t.WY0 + __builtin_ctzll(om) / 8;
        by1 = t.WY0 + (63 - __builtin_clzll(om)) / 8;
      }
      if (lane == 0) {
        S.wbox[w][0] = bx0;
        S.wbox[w][1] = bx1;
        S.wbox[w][2] = by0;
        S.wbox[w][3] = by1;
      }
      const bool all = __syncthreads_and(!open) != 0 || S.base == -2;
      if (!all) {
        t.wave_live = om != 0ull;
        t.SX0 = bx0;
        t.SX1 = bx1;
        t.SY0 = by0;
        t.SY1 = by1;
        int fx0 = S.wbox[0][0], fx1 = S.wbox[0][1], fy0 = S.wbox[0][2], fy1 = S.wbox[0][3];
#pragma unroll
        for (int v = 1; v < 4; ++v) {
          fx0 = min(fx0, S.wbox[v][0]);
          fx1 = max(fx1, S.wbox[v][1]);
          fy0 = min(fy0, S.wbox[v][2]);
          fy1 = max(fy1, S.wbox[v][3]);
        }
        t.FX0 = fx0;
        t.FX1 = fx1;
        t.FY0 = fy0;
        t.FY1 = fy1;
      }
      return all;
    };
    // (S.base == -2 is visible from tile_rounds' first barrier on, before any record is written)
    auto round_checked = [&](int nsub, int cnt) {
      if (S.base >= 0) round(nsub, cnt);
    };
    tile_rounds(L, a.bb, nview, b, lo, t, stage, round_checked, fs.dbg, done);
    __syncthreads();
    ovf = S.base == -2;
    if (CLK && KD_DIAG && clk && tid == 0) {
      const int64_t nb = (int64_t)gridDim.x * gridDim.y,
                    slot = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
      cyc[6] = S.nrec;
      cyc[7] = now_clk() - pa0;
#pragma unroll
      for (int i = 0; i < 8; ++i) clk[i * nb + slot] = cyc[i];
    }
    if (KD_DIAG && fs.tbuf && tid == 0 && FUSED)  // diagnostics: end of pass A
      fs.tbuf[5ll * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] =
          wall_clock64();
  }
  if (ovf) {  // no records: kd_soft_ovf_fwd computes the tile's soft mask, kd_soft_ovf_bwd its
              // backward
    my_kid = 0;
    if (tid == 0) {
      pb.ovf[atomicAdd(&pb.counters[2], 1)] = (int32_t)tile;
      S.nrec = 0;
    }
  }
  T sval = unc ? (T)0.0 : (T)1.0;  // this pixel's soft value (FUSED: the product below)
  if (t.inimg && owner) {
    // the split pipeline's reduce / the close-list writer (kd_soft_lists, also after FUSED)
    if (!FUSED || a.prob) pb.npix[p] = my_kid;
    if (a.soft && !unc) a.soft[p] = (T)1.0;  // dibr_soft_mask_cuda.cu:69
    else if (a.soft && my_kid == 0) a.soft[p] = (T)0.0;
    if (a.last && my_kid < K) a.last[p] = -1;
    // (the close lists, values and -1 / 0 / 0 padding alike, are written row-coalesced by
    // kd_soft_lists)
  }
  __syncthreads();
  const int n = S.nrec;
  const int64_t base = S.base;
  if (tid == 0) {
    pb.ntile[tile] = ovf ? -1 : n;  // -1: kd_soft_ovf_fwd streams the tile (lists included)
    pb.tbase[tile] = n > 0 ? base : 0;
  }
  // work items of the math and backward passes: nch items reserved with one device atomic.
  // FUSED: the reservation's latency overlaps the pair math (thread 0 keeps the returned base in
  // a register; the items are written after the product)
  const int nch = (n + kBlock - 1) / kBlock;
  int ibase = 0;
  if (n > 0 && tid == 0) ibase = atomicAdd(&pb.counters[0], nch);
  auto write_items = [&]() {
    if (n <= 0) return;
    if (tid == 0) S.ibase = ibase;
    __syncthreads();
    for (int c = tid; c < nch; c += kBlock)
      pb.items[S.ibase + c] =
          PairItem{base + (int64_t)c * kBlock, (int32_t)tile, min(kBlock, n - c * kBlock)};
  };
  if constexpr (!FUSED) {
    if (n > 0 && tid == 0) pb.tiles[atomicAdd(&pb.counters[1], 1)] = (int32_t)tile;
    write_items();
  }
  if constexpr (FUSED) {
    zero_side_job(a);
    if (n == 0) {
      iou_tile_terms<T>(a, b, tl, p, t.inimg && owner, sval, S.iou);
      return;
    }
    // pair math over this tile's records (record order: coalesced reads; diag 32: none)
    const int tx = tl % pb.ntx, ty = tl / pb.ntx;
    const T *sp = pb.sprob + base;
    // split tiles (a part owns kBlock / SPLIT pixels): the record table's LDS holds the part's
    // probabilities by (slot, pixel) instead -- the product then needs no global reads
    constexpr int kPtw = kBlock / SPLIT;
    static_assert(SPLIT == 1 || sizeof(T) * kFuseSlots * kPtw <= sizeof(S.ridx),
                  "split tiles: the probability table must fit the record table's LDS");
    T *pt = SPLIT > 1 ? reinterpret_cast<T *>(&S.ridx[0][0]) : nullptr;
    const int q0 = part * kPtw;
    pair_math_range<T, SPLIT == 1 ? 1 : 2>(a, pb, base, tx, ty, 0, n, pt, q0, kPtw);
    __syncthreads();  // the workgroup's probabilities are visible to it
    if (KD_DIAG && fs.tbuf && tid == 0)  // diagnostics: end of the pair math
      fs.tbuf[6ll * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] =
          wall_clock64();
    // soft = 1 - prod(1 - p) in slot order (dibr_soft_mask_cuda.cu:174-181, double-promoted)
    if (unc && owner && my_kid > 0) {
      constexpr int U8 = 8;
      const int rq = tile_q;  // the pixel's column of the record table
      T prod = (T)1.0;
      for (int s0 = 0; s0 < my_kid; s0 += U8) {
        T pv[U8];
#pragma unroll
        for (int u = 0; u < U8; ++u)
          pv[u] = s0 + u < my_kid ? (SPLIT > 1 ? pt[(s0 + u) * kPtw + (rq - q0)]
                                               : sp[S.ridx[s0 + u][rq]])
                                  : (T)0;
#pragma unroll
        for (int u = 0; u < U8; ++u)
          if (s0 + u < my_kid) prod = (T)((double)prod * (1.0 - (double)pv[u]));
      }
      sval = (T)(1.0 - (double)prod);
      a.soft[p] = sval;
    }
    write_items();
    iou_tile_terms<T>(a, b, tl, p, t.inimg && owner, sval, S.iou);
  }
}

template <typename T, bool FUSED, int OCC = 8>
__global__ __launch_bounds__(kBlock, OCC) void kd_soft_pairs(SoftArgs<T> a, SoftPairBuf<T> pb) {
  __shared__ SoftPairsLDS<FUSED> S;
  TileClock clk(a.fs.tbuf, 1);
  clk.start_to(2);
  if (ablate(a.fs.dbg, 16384)) return;  // diagnostics: dispatch cost only
  int b, tl, nbin;
  tile_of_block(a.bb, a.fs.H, a.fs.W, b, tl, nbin, a.fs.dbg);
  soft_pairs_tile<T, FUSED>(a, pb, b, tl, nbin, S);
}

// The DIB-R forward's per-tile work in one launch: a workgroup rasterizes its tile (the pair
// pipeline, kd_raster_pairs.hpp) and then runs the fused soft mask on the same tile; each thread
// owns the same pixel in both, so the soft phase reads the face_idx its own thread just wrote.
// No launch boundary between the two, and a tile's raster and soft work (heavy in different
// tiles: interior vs silhouette) share one workgroup slot.  The two phases' LDS is a union.
template <typename T>
union DibrTileLDS {
  RasterPairsLDS<T> r;
  SoftPairsLDS<true> s;
};

// DIAG (debug flag 64 with a debug buffer): per dispatch slot the tile, its bin counts, start,
// duration and raster-phase end (tools/soft_timeline.py).  A separate instantiation: the clock's
// live registers alone make the kernel spill.
//
// SPLIT (1, 2, 4; kd_tile.hpp tile_geom_part): each tile as SPLIT workgroups over a (tiles *
// SPLIT, views) grid, for batches too small to fill the chip with whole tiles: a heavy tile's
// raster chunks, pass A chunks and pair math spread over SPLIT CUs.  The raster phase hands the
// soft phase its uncovered pixels through `uncm` (the soft phase's waves need not own them).
// 7 workgroups per CU (21.5 KB of LDS, <= 72 VGPRs: four of the values the raster walk keeps in
// flight spill to 20 bytes of scratch; at 6 per CU, 78 VGPRs, the launch measured 124.7 against
// 119.5 us at 8 views).
template <bool DIAG, int SPLIT>
__global__ __launch_bounds__(kBlock, 7) void kd_dibr_fwd_tiles(RasterFwdArgs<float> ra,
                                                              SoftArgs<float> a,
                                                              SoftPairBuf<float> pb) {
  __shared__ DibrTileLDS<float> U;
  __shared__ uint64_t uncm[4];
  __shared__ long long s_t0;  // tile history: the workgroup's start and finished waves
  __shared__ int s_done;
  TileClock clk(DIAG ? a.fs.tbuf : nullptr, 1);
  if (DIAG) clk.start_to(2);
  if (ra.bb.hist && threadIdx.x == 0) {  // (the walk's barriers order these before any read)
    s_t0 = (long long)wall_clock64();
    s_done = 0;
  }
  int b, tl, nbin, part;
  tile_of_block_split<SPLIT>(ra.bb, ra.fs.H, ra.fs.W, b, tl, part, nbin, ra.fs.dbg);
  // split tiles (small batches, where the heavy tiles' chain of round trips is the launch's
  // length): the soft mask's coarse bin (same geometry as the raster's) -- its base and face
  // count loaded now, in flight during the raster phase, instead of as the soft walk's first
  // round trip (1 view 41.7 -> 41.4 us, 2 views 56.5 -> 55.8; whole tiles: +0.4 us, not used)
  int s_nb = -1, s_base = kNoBinBase;
  if constexpr (SPLIT > 1) {
    const BinGeom &g = a.bb.g;
    const int ntx = (a.fs.W + kTile - 1) / kTile;
    const int ct = (((tl / ntx) * kTile) >> g.sh) * g.nctx + (((tl % ntx) * kTile) >> g.sh);
    const int64_t bc = (int64_t)b * g.nct() + ct;
    s_base = a.bb.base[bc];
    s_nb = a.bb.totals[bc];
  }
  if (DIAG && a.fs.tbuf && threadIdx.x == 0) {
    const int64_t nb = (int64_t)gridDim.x * gridDim.y, slot = blockIdx.y * gridDim.x + blockIdx.x;
    a.fs.tbuf[slot] = ((long long)nbin << 32) | (long long)(b * pb.ntiles + tl);
    const BinGeom &g = a.bb.g;  // the soft coarse bin's face count
    const int tx = tl % pb.ntx, ty = tl / pb.ntx;
    const int ct = (ty * kTile / g.ct) * g.nctx + (tx * kTile / g.ct);
    a.fs.tbuf[4 * nb + slot] = a.bb.totals[(int64_t)b * g.nct() + ct];
  }
  raster_pairs_tile<float, DIAG, SPLIT>(
      ra, b, tl, nbin, U.r, DIAG && a.fs.tbuf ? a.fs.tbuf + 7ll * gridDim.x * gridDim.y : nullptr,
      part, uncm);
  __syncthreads();  // the raster phase is done with the LDS
  if (DIAG && a.fs.tbuf && threadIdx.x == 0)
    a.fs.tbuf[3ll * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] =
        wall_clock64();
  if (!ablate(a.fs.dbg, 1 << 24))  // diagnostics: the raster phase alone (instruction counts)
    soft_pairs_tile<float, true, SPLIT, DIAG>(
        a, pb, b, tl, s_nb, U.s, part, uncm,
        DIAG && a.fs.tbuf ? a.fs.tbuf + 16ll * gridDim.x * gridDim.y : nullptr, s_base);
  // tile history (kd_set_tile_history): the last wave to finish stores the workgroup's duration
  // as a quarter-octave bucket (1..63; 0 = none) for the next same-shape call's dispatch order
  if (ra.bb.hist && (threadIdx.x & (kWave - 1)) == 0 &&
      atomicAdd(&s_done, 1) == kBlock / kWave - 1) {
    const long long dt = (long long)wall_clock64() - s_t0;  // 100 MHz ticks
    const unsigned t = (unsigned)min(max(dt, 1ll), 0x7fffffffll);
    const int bl = 32 - __clz(t);
    const int q = bl >= 3 ? 4 * bl + (int)((t >> (bl - 3)) & 3u) : bl;
    ra.bb.hist[4 * ((int64_t)b * pb.ntiles + tl) + part] = (unsigned short)(min(max(q - 16, 0), 62) + 1);
  }
}

// The fp64 DIB-R forward in one launch: the pair raster (fp64 test, fp64-culled candidates, the
// exact-depth winner of RasterPairsLDS<double>) and the fused soft mask per tile, as
// kd_dibr_fwd_tiles does for fp32 (the culling data read from global memory in pass A: 29 KB of
// LDS, five workgroups per CU).
__global__ __launch_bounds__(kBlock, 5) void kd_dibr_fwd_tiles_f64(RasterFwdArgs<double> ra,
                                                                 SoftArgs<double> a,
                                                                 SoftPairBuf<double> pb) {
  __shared__ DibrTileLDS<double> U;
  int b, tl, nbin;
  tile_of_block(ra.bb, ra.fs.H, ra.fs.W, b, tl, nbin, ra.fs.dbg);
  raster_pairs_tile<double>(ra, b, tl, nbin, U.r);
  __syncthreads();  // the raster phase is done with the LDS
  soft_pairs_tile<double, true>(a, pb, b, tl, -1, U.s);
}

// ------------------------------------------------------------------------------------------
// the split pipeline: pair math and product as their own launches
// ------------------------------------------------------------------------------------------
// soft = 1 - prod(1 - p) over the close faces of the 256 pixels of one tile, in slot order
// (dibr_soft_mask_cuda.cu:174-181, double-promoted product).  kReduceSlots slots at a time of
// the tile's records are placed into an LDS table by
// (slot, pixel) and each pixel lane multiplies its slots in order.  Pixels without close faces
// (and the tiles that streamed) were written by kd_soft_pairs.
constexpr int kReduceSlots = 32;

template <typename T>
__device__ __forceinline__ void soft_reduce_tile(const SoftArgs<T> &a, const SoftPairBuf<T> &pb,
                                                 int64_t tile, T (*s_p)[kBlock]) {
  const int K = a.K, H = a.fs.H, W = a.fs.W;
  const int tid = threadIdx.x;
  const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
  const int n = pb.ntile[tile];
  const int64_t base = pb.tbase[tile];
  int px, py;
  tile_pixel(tl % pb.ntx, tl / pb.ntx, tid, px, py);
  const bool in = px < W && py < H;
  const int64_t p = ((int64_t)b * H + py) * W + px;
  const int np = in ? pb.npix[p] : 0;
  T prod = (T)1.0;
  for (int s0 = 0; s0 < K; s0 += kReduceSlots) {
    __syncthreads();  // the previous pass is done with s_p
    for (int i = tid; i < n; i += kBlock) {
      const int64_t ri = base + i;
      const uint32_t sq = ((const uint32_t *)(pb.rec + ri))[1];  // slot | q << 16
      const int s = (int)(sq & 0xffffu) - s0;
      if (s >= 0 && s < kReduceSlots) s_p[s][(sq >> 16) & 0xffu] = pb.sprob[ri];
    }
    __syncthreads();
    const int e = min(np - s0, kReduceSlots);
    for (int s = 0; s < e; ++s) prod = (T)((double)prod * (1.0 - (double)s_p[s][tid]));
    if (__syncthreads_and(np <= s0 + kReduceSlots)) break;
  }
  if (np > 0) a.soft[p] = (T)(1.0 - (double)prod);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_soft_reduce(SoftArgs<T> a, SoftPairBuf<T> pb) {
  __shared__ T s_p[kReduceSlots][kBlock];
  const int64_t nz = a.nzero0 + a.nzero1;  // side job: zero fills (grid-stride, coalesced)
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nz;
       i += (int64_t)gridDim.x * kBlock) {
    if (i < a.nzero0)
      a.zero0[i] = (T)0;
    else
      a.zero1[i - a.nzero0] = (T)0;
  }
  const int ntl = pb.counters[1];
  for (int ti = blockIdx.x; ti < ntl; ti += gridDim.x) soft_reduce_tile<T>(a, pb, pb.tiles[ti], s_p);
}

// The split pipeline's soft mask and close-face lists, one workgroup per tile (grid-stride over
// every tile: the lists of a tile without records are all padding): kReduceSlots slots at a time,
// the tile's records put their values -- probability, face, type -- into LDS (slot, pixel)
// tables (coalesced record reads); each pixel multiplies its slots in order
// (dibr_soft_mask_cuda.cu:174-181, double-promoted), and the lists -- values (:165-171) and the
// -1 / 0 / 0 padding of the unused slots (dibr_soft_mask.cpp:86-97) -- are written in memory
// order from LDS alone: consecutive threads take consecutive elements (slot pairs: 8 / 16 /
// 2-byte stores with an even knum) of each tile row's contiguous (16 pixels x K) block, so the
// 13 K bytes per pixel go out as whole lines (the per-pixel rows of K elements written by one
// lane each were a 17x slower store shape; gathering each element's record from L2 inside the
// store loop left the loop latency-bound).  Half tiles of 8 rows (8192 -> 16384 work units, the
// tables halved: 4 workgroups per CU instead of 2).  Dynamic LDS: T val[128][33],
// int face_type[128][33], int np[128].
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_soft_lists(SoftArgs<T> a, SoftPairBuf<T> pb) {
  extern __shared__ unsigned char s_raw[];
  // [pixel][slot] with an odd row stride: the store loop's lanes read consecutive slots of one
  // pixel, the product's lanes one slot of consecutive pixels -- both bank-conflict free
  constexpr int R = kReduceSlots + 1, HP = kBlock / 2;
  T(*s_val)[R] = (T(*)[R])s_raw;
  int(*s_ft)[R] = (int(*)[R])(s_raw + sizeof(T) * R * HP);
  int *s_np = (int *)(s_raw + (sizeof(T) + sizeof(int)) * R * HP);
  const int K = a.K, H = a.fs.H, W = a.fs.W;
  const int tid = threadIdx.x;
  zero_side_job(a);  // side job: the backward's zero fills
  // half tiles: rows 0-7 (tile pixels q < 128) and rows 8-15 of a tile, so that the tables are
  // half the size and twice the workgroups fit a CU (the loop is store / load latency bound)
  const int64_t nht = 2 * (int64_t)a.fs.B * pb.ntiles;
  for (int64_t ht = blockIdx.x; ht < nht; ht += gridDim.x) {
    const int64_t tile = ht >> 1;
    const int half = (int)(ht & 1), q0 = half * HP;
    const int n = pb.ntile[tile];
    if (n < 0) continue;  // overflowed: kd_soft_ovf_fwd wrote its soft mask and lists
    const int64_t base = pb.tbase[tile];
    const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
    const int X0 = (tl % pb.ntx) * kTile, Y0 = (tl / pb.ntx) * kTile + half * (kTile / 2);
    const int nx = min(kTile, W - X0), ny = max(0, min(kTile / 2, H - Y0));
    int64_t lo, hi;
    view_range(a.fs, b, lo, hi);
    int px = W, py = H;
    if (tid < HP) tile_pixel(tl % pb.ntx, tl / pb.ntx, q0 + tid, px, py);
    const bool in = px < W && py < H;
    const int64_t p = ((int64_t)b * H + py) * W + px;
    const int np = in ? pb.npix[p] : 0;
    lds_barrier();  // the previous tile is done with the tables
    if (tid < HP) s_np[tid] = np;
    T prod = (T)1.0;
    for (int s0 = 0; s0 < K; s0 += kReduceSlots) {
      const int S = min(kReduceSlots, K - s0);
      lds_barrier();  // the previous pass is done with the tables (and s_np is written)
      // four records per thread in flight (the pass is load-latency bound otherwise)
      for (int i0 = tid; i0 < n; i0 += 4 * kBlock) {
        SoftPairRec rr[4];
        T pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = min(i0 + u * kBlock, n - 1);
          rr[u] = pb.rec[base + i];
          pv[u] = pb.sprob[base + i];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int s = (int)rr[u].slot - s0, q = (int)rr[u].q - q0;
          if (i0 + u * kBlock < n && s >= 0 && s < S && q >= 0 && q < HP) {
            s_val[q][s] = pv[u];
            s_ft[q][s] = (int)(((int64_t)rr[u].row - lo) << 3) | (rr[u].type + 1);
          }
        }
      }
      lds_barrier();
      const int e_hi = a.soft ? min(np - s0, S) : 0;  // (no soft: the one launch wrote it)
      for (int s = 0; s < e_hi; ++s) prod = (T)((double)prod * (1.0 - (double)s_val[tid][s]));
      // the pass's slots of the half tile's rows, in memory order
      auto value = [&](int q, int s, T &pv, int64_t &cv, uint8_t &tv) {
        if (s0 + s < s_np[q]) {
          const int ft = s_ft[q][s];
          pv = s_val[q][s];
          cv = (int64_t)(ft >> 3);
          tv = (uint8_t)(ft & 7);
        } else {
          pv = (T)0;
          cv = -1;
          tv = 0;
        }
      };
      if (ablate(a.fs.dbg, 1 << 16)) continue;  // diagnostics: no list stores
      // pixel (r, i) of the half tile -> its table row (tile_geom's q minus q0)
      auto hq = [](int r, int i) { return ((i >> 3) * kWave) + (r & 7) * 8 + (i & 7); };
      if ((K & 1) == 0) {  // slot pairs: every pair starts at an even element
        // a row's nx x S2 slot pairs (<= 16 x 16 = 256) are one pass of the workgroup: thread
        // tid takes pixel i, pair s of every row (no divisions in the loop)
        const int S2 = S >> 1, per_row = nx * S2;
        const int i = tid / S2, s = 2 * (tid - i * S2);
        for (int r = 0; tid < per_row && r < ny; ++r) {
          const int q = hq(r, i);
          const int64_t o = (((int64_t)b * H + Y0 + r) * W + X0 + i) * K + s0 + s;
          T p0, p1;
          int64_t c0, c1;
          uint8_t t0, t1;
          value(q, s, p0, c0, t0);
          value(q, s + 1, p1, c1, t1);
          if constexpr (sizeof(T) == 4) {
            *(float2 *)(a.prob + o) = make_float2(p0, p1);
          } else {
            *(double2 *)(a.prob + o) = make_double2(p0, p1);
          }
          if (ablate(a.fs.dbg, 1 << 23)) continue;  // diagnostics: probabilities only
          *(longlong2 *)(a.cidx + o) = make_longlong2(c0, c1);
          *(uint16_t *)(a.ctype + o) = (uint16_t)(t0 | (t1 << 8));
        }
      } else {
        const int per_row = nx * S;
        for (int e = tid; e < ny * per_row; e += kBlock) {
          const int r = e / per_row, rem = e - r * per_row;
          const int i = rem / S, s = rem - i * S;
          const int64_t o = (((int64_t)b * H + Y0 + r) * W + X0 + i) * K + s0 + s;
          value(hq(r, i), s, a.prob[o], a.cidx[o], a.ctype[o]);
        }
      }
    }
    if (np > 0 && a.soft) a.soft[p] = (T)(1.0 - (double)prod);
  }
}

// Flat over the (tile, 256-record) items: each record's distance type and probability
// (bit-identical to the reference) and optionally the close lists.
template <typename T, bool LISTS>
__global__ __launch_bounds__(kBlock) void kd_soft_pair_math(SoftArgs<T> a, SoftPairBuf<T> pb) {
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const float M = fs.M;
  const int nitems = pb.counters[0];
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const PairItem item = pb.items[it];
    if ((int)threadIdx.x >= item.n) continue;
    const int64_t i = item.start + threadIdx.x;
    const SoftPairRec r = pb.rec[i];
    T v[6];
    load_corners(fs, (int64_t)r.row, v);
    const int64_t tile = item.tile;
    const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
    int px, py;
    tile_pixel(tl % pb.ntx, tl / pb.ntx, r.q, px, py);
    const T x0 = (T)px_cx(M, W, px), y0 = (T)px_cy(M, H, py);
    int et = 0;
    T prob = (T)0;
    soft_face_dist<T>(x0, y0, v, M, a.sigmainv, et, prob);
    pb.sprob[i] = prob;
    pb.rec[i].type = (uint8_t)et;
    // (LISTS: kd_soft_lists writes the close lists from the records, row-coalesced)
    if (a.last && r.slot == K - 1) {
      const int64_t gp = ((int64_t)b * H + py) * W + px;
      int64_t lo, hi;
      view_range(fs, b, lo, hi);
      a.last[gp] = (int32_t)((int64_t)r.row - lo);
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// Flat over the (tile, 256-record chunk) items, one record per thread: s_p * h_j expanded to
// the face's 6 corner coordinates, summed over the record's run of equal faces inside its wave
// by a segmented inclusive scan (records are face-major runs; no LDS), and the run's last lane
// adds the nonzero sums with float atomics.  Every
// record costs the same, so the grid is balanced however the records fall on the tiles.
// One step of a segmented inclusive wave scan with DPP (no LDS): lanes add the DPP source lane's
// six sums when it belongs to the same segment (invalid sources read segment -1).
// The DPP reads are pinned with an empty asm where the whole wave is active: left inside the
// select, the compiler may issue them under the `take` lanes only, and a source lane outside
// EXEC reads the `old` operand (0).
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_scan_dpp(int seg, float g[6]) {
  int os = __builtin_amdgcn_update_dpp(-1, seg, CTRL, ROWS, 0xf, false);
  asm volatile("" : "+v"(os));
  const bool take = os == seg;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    float o = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(g[q]), CTRL, ROWS, 0xf, false));
    asm volatile("" : "+v"(o));
    g[q] += take ? o : 0.f;
  }
}

// fp64 form: the two 32-bit halves of each sum move by DPP (no LDS permutes)
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_scan_dpp(int seg, double g[6]) {
  int os = __builtin_amdgcn_update_dpp(-1, seg, CTRL, ROWS, 0xf, false);
  asm volatile("" : "+v"(os));
  const bool take = os == seg;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const long long x = __double_as_longlong(g[q]);
    int lo = __builtin_amdgcn_update_dpp(0, (int)(x & 0xffffffffll), CTRL, ROWS, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, ROWS, 0xf, false);
    asm volatile("" : "+v"(lo), "+v"(hi));
    const double o = __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
    g[q] += take ? o : 0.0;
  }
}

template <typename T>
__device__ __forceinline__ void seg_scan_shfl(int seg, int lane, T g[6]) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int o_seg = __shfl_up(seg, d);
    const bool take = lane >= d && o_seg == seg;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const T o = __shfl_up(g[q], d);
      g[q] += take ? o : (T)0;
    }
  }
}

// Flat over the (tile, 256-record) items, one record per thread: the coefficients are computed
// from the record's face corners, distance type and forward probability (soft_pair_coef: the
// forward's critical path skips them; this kernel, bound by its load chains and atomics, absorbs
// the arithmetic), s_p * h_j is expanded to the face's 6 corner coordinates, summed over the
// record's run of equal faces inside its wave by a segmented inclusive scan (records are
// face-major runs; no LDS), and the run's last lane adds the nonzero sums with float atomics.
// Every record costs the same, so the grid is balanced however the records fall on the tiles.
template <typename T, int R, bool VTX = false>
__device__ __forceinline__ void soft_bwd_items_body(const SoftArgs<T> &a, const SoftPairBuf<T> &pb,
                                                    int blk, int nblk) {
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W;
  const int lane = threadIdx.x & (kWave - 1);
  // the first pass's items are loaded with the item count, not after it (entries past the count
  // are stale and dropped; the grid covers the items in about one pass)
  PairItem first[R];
#pragma unroll
  for (int u = 0; u < R; ++u)
    first[u] = blk * R + u < pb.icap ? pb.items[blk * R + u] : PairItem{0, 0, 0};
  const int nitems = pb.counters[0];
  // R items per workgroup pass; their load chains (item -> record -> the pixel's gradient and
  // soft value, the face's corners) are issued together
  for (int it0 = blk * R; it0 < nitems; it0 += nblk * R) {
    bool ok[R];
    SoftPairRec r[R];
    SoftCoef<T> c[R];
    T gs[R], so[R];
    int et[R];
    PairItem item[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      item[u] = it0 + u < nitems ? (it0 == blk * R ? first[u] : pb.items[it0 + u])
                                 : PairItem{0, 0, 0};
      ok[u] = (int)threadIdx.x < item[u].n;
      if (ok[u]) r[u] = pb.rec[item[u].start + threadIdx.x];
    }
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (ok[u]) {
        const int64_t ri = item[u].start + threadIdx.x;
        const int64_t tile = item[u].tile;
        const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
        int px, py;
        tile_pixel(tl % pb.ntx, tl / pb.ntx, r[u].q, px, py);
        const int64_t gp = ((int64_t)b * H + py) * W + px;
        gs[u] = soft_grad_at<T>(a, b, gp);
        so[u] = a.soft_in[gp];
        T v[6];
        load_corners(fs, (int64_t)r[u].row, v);
        const float M = fs.M;
        et[u] = r[u].type;
        soft_pair_coef<T>((T)px_cx(M, W, px), (T)px_cy(M, H, py), v, et[u], pb.sprob[ri], M,
                          c[u].h);
      }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      int key = -1;
      T g[6] = {0, 0, 0, 0, 0, 0};
      if (ok[u]) {
        const double sp = -(double)a.sigmainv * (double)gs[u] * (1.0 - (double)so[u]);
        soft_add_pair<T>(g, et[u], sp, c[u]);
        key = r[u].row;
      }
      // segmented inclusive scan over the wave's lanes; segments are the runs of equal key (a
      // face may have several runs: one per wave sub-list chunk), numbered by the count of run
      // heads up to the lane
      const int prev_key = __shfl_up(key, 1);
      const uint64_t heads = __ballot(lane == 0 || prev_key != key);
      const int seg = __popcll(heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)));
      seg_scan_dpp<0x111, 0xf>(seg, g);  // row_shr:1
      seg_scan_dpp<0x112, 0xf>(seg, g);  // row_shr:2
      seg_scan_dpp<0x114, 0xf>(seg, g);  // row_shr:4
      seg_scan_dpp<0x118, 0xf>(seg, g);  // row_shr:8
      seg_scan_dpp<0x142, 0xa>(seg, g);  // row_bcast:15 -> rows 1, 3
      seg_scan_dpp<0x143, 0xc>(seg, g);  // row_bcast:31 -> rows 2, 3
      const int next_key = __shfl_down(key, 1);
      const bool tail = key >= 0 && (lane == kWave - 1 || next_key != key);
      if constexpr (!VTX && sizeof(T) == 4) {
        // the run sums leave as whole face rows: tail r's term q goes to lane 6 r + q of a pass,
        // so one atomic instruction adds ~10 faces' consecutive 24-byte rows.  Float atomics
        // execute at the memory side, one request per 64-byte segment an instruction touches
        // (MI355X_MICROARCH.md, Global float atomics): six one-term instructions made one
        // request per tail and term.  (diagnostics 4096: no atomics)
        const uint64_t tm = __ballot(tail);
        const int nt = __popcll(tm);
        const int rank = __popcll(tm & ((1ull << lane) - 1ull));
        // lane r < nt learns the lane of the r-th tail (a push; the other lanes push to lane 63,
        // which is a tail's destination only when every lane is a tail)
        const int tail_lane = __builtin_amdgcn_ds_permute((tail ? rank : 63) << 2, lane);
        for (int v0 = 0; v0 < 6 * nt && !ablate(fs.dbg, 4096); v0 += kWave) {
          const int v = v0 + lane;
          const int r = v / 6, q = v - 6 * r;
          const int src = __builtin_amdgcn_ds_bpermute(min(r, kWave - 1) << 2, tail_lane) << 2;
          const int kk = __builtin_amdgcn_ds_bpermute(src, key);
          float x = 0.f;
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            const float gj = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(g[j])));
            x = q == j ? gj : x;
          }
          if (v < 6 * nt && x != 0.f) atomicAdd(a.grad_fvi + (int64_t)kk * 6 + q, x);
        }
      } else if (tail && !ablate(fs.dbg, 4096)) {  // (diagnostics 4096: no atomics)
        if constexpr (VTX) {
#pragma unroll
          for (int k = 0; k < 3; ++k) vertex_add(a.vo, (int64_t)key, k, g[2 * k], g[2 * k + 1]);
        } else {
#pragma unroll
          for (int q = 0; q < 6; ++q)
            if (g[q] != (T)0) atomicAdd(a.grad_fvi + (int64_t)key * 6 + q, g[q]);
        }
      }
    }
  }
}

// The backward of the tiles that streamed their soft mask (pool exhausted): the same walk again,
// each pixel lane recomputing its pairs (bit-identical probabilities and types) and adding their
// terms with float atomics.  One workgroup per such tile; a grid that finds none exits at once.
template <typename T, bool VTX>
__global__ __launch_bounds__(kBlock) void kd_soft_ovf_bwd(SoftArgs<T> a, SoftPairBuf<T> pb) {
  __shared__ TileLists L;
  const int blk = blockIdx.x, nblk = gridDim.x;
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const float M = fs.M;
  const int novf = pb.counters[2];
  for (int i = blk; i < novf; i += nblk) {
    const int64_t tile = pb.ovf[i];
    const int b = (int)(tile / pb.ntiles), tl = (int)(tile - (int64_t)b * pb.ntiles);
    int64_t lo, hi;
    view_range(fs, b, lo, hi);
    const TileGeom t = tile_geom(H, W, tl);
    const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
    const bool unc = t.inimg && a.face_idx[p] < 0;
    const bool wave_unc = __ballot(unc) != 0ull;
    const double sp =
        unc ? -(double)a.sigmainv * (double)soft_grad_at<T>(a, b, p) * (1.0 - (double)a.soft_in[p])
            : 0.0;
    const T x0 = (T)px_cx(M, W, t.px), y0 = (T)px_cy(M, H, t.py);
    int my_kid = 0;
    auto stage = [&](int, int64_t) {};
    auto round = [&](int nsub, int) {
      if (wave_unc)
        for (int c = 0; c * kWave < nsub; ++c)
          soft_chunk_stream(L, nsub, c, unc, K, t, lo, my_kid, [&](int64_t row, int) {
            T v[6];
            load_corners(fs, row, v);
            int et = 0;
            T prob = (T)0;
            soft_face_dist<T>(x0, y0, v, M, a.sigmainv, et, prob);
            SoftCoef<T> cf;
            soft_pair_coef<T>(x0, y0, v, et, prob, M, cf.h);
            T g[6] = {0, 0, 0, 0, 0, 0};
            soft_add_pair<T>(g, et, sp, cf);
            if constexpr (VTX) {
#pragma unroll
              for (int k = 0; k < 3; ++k) vertex_add(a.vo, row, k, g[2 * k], g[2 * k + 1]);
            } else {
#pragma unroll
              for (int q = 0; q < 6; ++q)
                if (g[q] != (T)0) atomicAdd(a.grad_fvi + row * 6 + q, g[q]);
            }
          });
    };
    auto done = [&]() { return __syncthreads_and(!unc || my_kid >= K) != 0; };
    if (__syncthreads_or(unc)) tile_rounds(L, a.bb, (int)(hi - lo), b, lo, t, stage, round, fs.dbg, done);
    __syncthreads();
  }
}

template <typename T, int R>
__global__ __launch_bounds__(kBlock) void kd_soft_bwd_items(SoftArgs<T> a, SoftPairBuf<T> pb) {
  soft_bwd_items_body<T, R>(a, pb, blockIdx.x, gridDim.x);
}

// The DIB-R backward in one launch: the raster backward's tiles and the soft mask's items are
// independent (both only add into grad_fvi), so one grid holds both, the raster tiles first
// (their XCD band mapping keeps its block ids), and the soft items fill the raster's tail:
// 72 us against 38 + 41 for the two launches at C3 (alternating runs of 8: 74 us).
template <typename T, bool VTX>
__global__ __launch_bounds__(kBlock) void kd_dibr_bwd(SoftArgs<T> a, SoftPairBuf<T> pb,
                                                      RasterBwdArgs<T> ra, int nr, int ns,
                                                      int ntl) {
  const int blk = blockIdx.x;
  if (blk < nr)
    raster_bwd_tile_body<T, 3, VTX>(ra, blk, nr, ntl);
  else
    soft_bwd_items_body<T, 2, VTX>(a, pb, blk - nr, ns);
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
constexpr unsigned kOvfBlocks = 256;  // grid of the overflow kernels (exit at once when unused)

// Whether a tile can find the pool exhausted: never with knum <= 32 (the pool holds 32 records
// per pixel) unless a test limits the pool; the overflow kernels are launched only then.  Once a
// limit has been set in this process (pool_limits_ever_set, the test hook), they are launched
// for every later call too -- they exit at once when no tile overflowed -- so a backward that
// runs after the limits were restored (a retained graph) still sees its forward's overflows.
static bool pool_may_overflow(int K) {
  return K > kPoolPairsPerPixel || pool_limit_pairs() < 1.f || pool_limits_ever_set();
}

template <typename T, bool FUSED>
static void ovf_fwd_launch(const SoftArgs<T> &a, const SoftPairBuf<T> &pb, hipStream_t stream) {
  ProfScope prof(K_SOFT_OVF_FWD, stream);
  hipLaunchKernelGGL((kd_soft_ovf_fwd<T, FUSED>), dim3(kOvfBlocks), dim3(kBlock), 0, stream, a,
                     pb);
}

template <typename T>
static void ovf_bwd_launch(const SoftArgs<T> &a, const SoftPairBuf<T> &pb, hipStream_t stream) {
  ProfScope prof(K_SOFT_OVF_BWD, stream);
  if (a.vo.grad)
    hipLaunchKernelGGL((kd_soft_ovf_bwd<T, true>), dim3(kOvfBlocks), dim3(kBlock), 0, stream, a,
                       pb);
  else
    hipLaunchKernelGGL((kd_soft_ovf_bwd<T, false>), dim3(kOvfBlocks), dim3(kBlock), 0, stream, a,
                       pb);
}

// The close-face lists after a one-launch soft mask (kd_soft_pairs FUSED or kd_dibr_fwd_tiles,
// which leave every record's probability and distance type): an overflowed tile's soft mask and
// lists from the streaming walk (the split form), then the lists writer over the records.
template <typename T>
static int lists_after_one_launch(const SoftArgs<T> &a, SoftPairBuf<T> &pb, hipStream_t stream) {
  // (F < 2^28 was checked before the first launch: dibr_fwd, soft_pairs_launch)
  if (pool_may_overflow(a.K)) ovf_fwd_launch<T, false>(a, pb, stream);
  SoftArgs<T> al = a;  // (the backward's zero fills were the one launch's side job)
  al.nzero0 = al.nzero1 = 0;
  al.soft = nullptr;  // (and the soft mask)
  const size_t dyn = ((sizeof(T) + sizeof(int)) * (kReduceSlots + 1) + sizeof(int)) * kBlock / 2;
  ProfScope prof(K_SOFT_REDUCE, stream);
  hipLaunchKernelGGL(kd_soft_lists<T>, dim3(8192), dim3(kBlock), dyn, stream, al, pb);
  return KD_OK;
}

template <typename T>
int soft_pairs_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, bool grad, bool reduce,
                      hipStream_t stream) {
  const FaceSet<T> &fs = a.fs;
  // the close lists pack (face << 3 | type) into an int: checked before any launch, so a refused
  // call writes no output
  KD_CHECK_ARG(!a.prob || fs.F < (1ll << 28), "close lists: more than 2^28 faces per view");
  a.fs.dbg = debug_flags();
  a.fs.tbuf = debug_tile_buffer();
  // one launch for the whole soft mask (knum <= 32); with the close-face lists (the op form,
  // dibr.py's SAVE_CLOSE_LISTS) the lists writer follows it, reading the records, types and
  // probabilities the one launch left (no separate pair-math launch)
  const bool fused = reduce && a.soft && !a.last && a.K <= kFuseSlots &&
                     !(test_forms() & KD_FORM_SOFT_SPLIT);
  if (fused) {
    {
      ProfScope prof(K_SOFT_PAIRS, stream);
      // 6 workgroups per CU (the 16 KB record-index table); 4 and 8 measured no faster
      hipLaunchKernelGGL((kd_soft_pairs<T, true, 6>), dim3((unsigned)pb.ntiles, fs.B),
                         dim3(kBlock), 0, stream, a, pb);
    }
    if (a.prob) {
      const int rc = lists_after_one_launch<T>(a, pb, stream);
      if (rc != KD_OK) return rc;
    } else if (pool_may_overflow(a.K)) {
      ovf_fwd_launch<T, true>(a, pb, stream);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft mask: %s", hipGetErrorString(e));
    return KD_OK;
  }
  {
    ProfScope prof(K_SOFT_PAIRS, stream);
    hipLaunchKernelGGL((kd_soft_pairs<T, false>), dim3((unsigned)pb.ntiles, fs.B), dim3(kBlock),
                       0, stream, a, pb);
  }
  if (pool_may_overflow(a.K)) ovf_fwd_launch<T, false>(a, pb, stream);
  {
    ProfScope prof(K_SOFT_MATH, stream);
    const dim3 grid(kMathBlocks);
    if (a.prob)
      hipLaunchKernelGGL((kd_soft_pair_math<T, true>), grid, dim3(kBlock), 0, stream, a, pb);
    else
      hipLaunchKernelGGL((kd_soft_pair_math<T, false>), grid, dim3(kBlock), 0, stream, a, pb);
  }
  if (reduce && a.soft) {
    ProfScope prof(K_SOFT_REDUCE, stream);
    if (a.prob) {  // soft mask + the close lists, row-coalesced (dynamic LDS past 64 KB)
      const size_t dyn = ((sizeof(T) + sizeof(int)) * (kReduceSlots + 1) + sizeof(int)) * kBlock / 2;
      if (dyn > 64 * 1024) {  // (34 KB fp32, 51 KB fp64: within the default limit)
        const hipError_t ea = hipFuncSetAttribute((const void *)kd_soft_lists<T>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  (int)dyn);
        if (ea != hipSuccess)
          return set_error(KD_ERR_LAUNCH, "soft lists: %s", hipGetErrorString(ea));
      }
      if (ablate(debug_flags(), (1 << 16) | (1 << 23)))  // diagnostics: the skipped index stores
        (void)hipMemsetAsync(a.cidx, 0xFF, sizeof(int64_t) * fs.B * fs.H * fs.W * a.K, stream);  // -1
      hipLaunchKernelGGL(kd_soft_lists<T>, dim3(8192), dim3(kBlock), dyn, stream, a, pb);
    } else
      hipLaunchKernelGGL(kd_soft_reduce<T>, dim3(8192), dim3(kBlock), 0, stream, a, pb);
  } else if (a.prob) {
    return set_error(KD_ERR_INVALID_ARGUMENT, "close lists need the soft mask");
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft mask: %s", hipGetErrorString(e));
  return KD_OK;
}

bool dibr_fwd_fusable(const RasterFwdArgs<double> &ra, const SoftArgs<double> &a) {
  return ra.bb.cull && a.soft && !a.last && a.K <= kFuseSlots &&
         !(test_forms() & (KD_FORM_SPLIT_FWD | KD_FORM_SOFT_SPLIT));
}

int dibr_fwd_fused_launch(RasterFwdArgs<double> &ra, SoftArgs<double> &a,
                          SoftPairBuf<double> &pb, hipStream_t stream) {
  ra.fs.dbg = a.fs.dbg = debug_flags();
  ra.fs.tbuf = nullptr;
  a.fs.tbuf = nullptr;
  {
    ProfScope prof(K_DIBR_FWD, stream);
    hipLaunchKernelGGL(kd_dibr_fwd_tiles_f64, dim3((unsigned)pb.ntiles, ra.fs.B), dim3(kBlock), 0,
                       stream, ra, a, pb);
  }
  if (a.prob) {  // the close-face lists (dibr_rasterization inside close_lists())
    const int rc = lists_after_one_launch<double>(a, pb, stream);
    if (rc != KD_OK) return rc;
  } else if (pool_may_overflow(a.K)) {
    ovf_fwd_launch<double, true>(a, pb, stream);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "dibr fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

// Workgroups per tile of the fused fp32 forward (kd_dibr_fwd_tiles SPLIT): the tile split hook
// (kd_set_tile_split) when set, else by the batch's tile count against the chip's workgroup
// slots.  Split tiles need the fixed record pool (every part owns its pixels' K records).
// history: the dispatch follows the tile history (kd_set_tile_history).
int fwd_tile_split(int64_t tiles, bool fixed_pool, bool history, hipStream_t stream) {
  if (!fixed_pool) return 1;
  const int forced = tile_split();
  if (forced > 0) return forced;
  const int cus = device_cus(stream);
  // measured at C3 (bench.py --tile-split, same box): 1 view (1024 tiles) 0.1177 / 0.1076 /
  // 0.1170 ms per step at 1 / 2 / 4 workgroups per tile; 2 views (2048) 0.1388 / 0.1463 / 0.1624;
  // 8 views 0.310 / 0.352.  A part repeats the tile's raster walk (~10 us of dependent loads at
  // one wave per SIMD), so splitting pays only while the whole tiles fit one round of slots.
  // With the tile history the silhouette parts no longer wait for a second round, and 2 views
  // split pay too (profiles/r04/ab_split_history.txt: 1 view 0.1142 / 0.0992 / 0.1012 (4), 2
  // views 0.1298 / 0.1221, 4 views 0.1667 / 0.1903, 8 views 0.2692 / 0.3289 ms).
  const int64_t slots = (int64_t)cus * (history ? 8 : 6);  // (6 workgroups per CU)
  return tiles <= slots ? 2 : 1;
}

int dibr_fwd_split(const SoftPairBuf<float> &pb, int K, int B, bool history, hipStream_t stream) {
  return fwd_tile_split((int64_t)B * pb.ntiles, pb.fixed && !pool_may_overflow(K), history,
                        stream);
}

bool dibr_fwd_fusable(const RasterFwdArgs<float> &ra, const SoftArgs<float> &a) {
  return ra.bb.cull && a.soft && !a.last && a.K <= kFuseSlots &&
         !(test_forms() & (KD_FORM_SPLIT_FWD | KD_FORM_SOFT_SPLIT));
}

int dibr_fwd_fused_launch(RasterFwdArgs<float> &ra, SoftArgs<float> &a, SoftPairBuf<float> &pb,
                          hipStream_t stream) {
  ra.fs.dbg = a.fs.dbg = debug_flags();
  ra.fs.tbuf = nullptr;
  a.fs.tbuf = debug_tile_buffer();
  {
    ProfScope prof(K_DIBR_FWD, stream);
    // (the lists writer reads each tile's records as one run: whole tiles)
    const int split = a.prob ? 1 : dibr_fwd_split(pb, a.K, ra.fs.B, ra.bb.hist != nullptr, stream);
    const dim3 grid((unsigned)pb.ntiles * split, ra.fs.B);
    const bool diag = KD_DIAG && a.fs.tbuf;
#define KD_FWD_TILES(S)                                                                         \
  do {                                                                                        \
    if (diag)                                                                                 \
      hipLaunchKernelGGL((kd_dibr_fwd_tiles<KD_DIAG != 0, S>), grid, dim3(kBlock), 0, stream, \
                         ra, a, pb);                                                          \
    else                                                                                      \
      hipLaunchKernelGGL((kd_dibr_fwd_tiles<false, S>), grid, dim3(kBlock), 0, stream, ra, a,  \
                         pb);                                                                 \
  } while (0)
    if (split == 4)
      KD_FWD_TILES(4);
    else if (split == 2)
      KD_FWD_TILES(2);
    else
      KD_FWD_TILES(1);
#undef KD_FWD_TILES
  }
  if (a.prob) {  // the close-face lists (dibr_rasterization inside close_lists())
    const int rc = lists_after_one_launch<float>(a, pb, stream);
    if (rc != KD_OK) return rc;
  } else if (pool_may_overflow(a.K)) {
    ovf_fwd_launch<float, true>(a, pb, stream);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "dibr fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int soft_pairs_forward(SoftArgs<T> &a, void *ws, size_t ws_bytes, bool grad, bool reduce,
                       hipStream_t stream) {
  const FaceSet<T> &fs = a.fs;
  const size_t need = soft_pair_workspace_bytes(fs.B, fs.H, fs.W, fs.N, fs.F, a.K, sizeof(T));
  if (ws_bytes < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  if (fs.B == 0 || fs.H == 0 || fs.W == 0) return KD_OK;
  size_t off = 0;
  a.bb = bin_carve(ws, off, fs.B, fs.H, fs.W, fs.N, fs.F);
  a.bb.cull = nullptr;
  SoftPairBuf<T> pb = soft_pair_carve<T>(ws, off, fs.B, fs.H, fs.W, a.K);
  a.bb.clear = pb.counters;
  a.bb.n_clear = kPairClear;
  hipError_t e = bin_faces<T>(fs, a.bb, stream);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "binning: %s", hipGetErrorString(e));
  return soft_pairs_launch<T>(a, pb, grad, reduce, stream);
}

template <typename T>
int soft_pairs_backward_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, hipStream_t stream) {
  a.fs.dbg = debug_flags();
  a.fs.tbuf = debug_tile_buffer();
  {
    ProfScope prof(K_SOFT_BWD_PAIRS, stream);
    hipLaunchKernelGGL((kd_soft_bwd_items<T, 1>), dim3(kMathBlocks), dim3(kBlock), 0, stream, a,
                       pb);
  }
  if (pool_may_overflow(a.K)) ovf_bwd_launch<T>(a, pb, stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int dibr_backward_merged_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, const RasterBwdArgs<T> &ra,
                                hipStream_t stream) {
  KD_CHECK_ARG(ra.D <= 3, "merged backward: D > 3");
  const int ntl = (int)pb.ntiles;
  const int64_t nr64 = ra.grad ? (int64_t)ra.B * ntl : 0;  // raster tiles (grad_interp given)
  KD_CHECK_ARG(nr64 + kMathBlocks < (1ll << 31), "merged backward: too many tiles");
  const int nr = (int)nr64, ns = (a.grad_soft || a.iou_gt) ? (int)kMathBlocks : 0;
  a.fs.dbg = debug_flags();
  a.fs.tbuf = debug_tile_buffer();
  if (nr + ns > 0) {
    ProfScope prof(K_DIBR_BWD, stream);
    if (a.vo.grad)  // the face -> vertex step fused (VertexOut)
      hipLaunchKernelGGL((kd_dibr_bwd<T, true>), dim3((unsigned)(nr + ns)), dim3(kBlock), 0,
                         stream, a, pb, ra, nr, ns, ntl);
    else
      hipLaunchKernelGGL((kd_dibr_bwd<T, false>), dim3((unsigned)(nr + ns)), dim3(kBlock), 0,
                         stream, a, pb, ra, nr, ns, ntl);
  }
  if ((a.grad_soft || a.iou_gt) && pool_may_overflow(a.K)) ovf_bwd_launch<T>(a, pb, stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "dibr bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int soft_pairs_backward(SoftArgs<T> &a, void *ws, size_t ws_bytes, hipStream_t stream) {
  const FaceSet<T> &fs = a.fs;
  const size_t need = soft_pair_workspace_bytes(fs.B, fs.H, fs.W, fs.N, fs.F, a.K, sizeof(T));
  if (ws_bytes < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  if (fs.B == 0 || fs.H == 0 || fs.W == 0) return KD_OK;
  size_t off = 0;
  a.bb = bin_carve(ws, off, fs.B, fs.H, fs.W, fs.N, fs.F);
  SoftPairBuf<T> pb = soft_pair_carve<T>(ws, off, fs.B, fs.H, fs.W, a.K);
  return soft_pairs_backward_launch<T>(a, pb, stream);
}

template SoftPairBuf<float> soft_pair_carve<float>(void *, size_t &, int, int, int, int);
template SoftPairBuf<double> soft_pair_carve<double>(void *, size_t &, int, int, int, int);
template int soft_pairs_launch<float>(SoftArgs<float> &, SoftPairBuf<float> &, bool, bool,
                                      hipStream_t);
template int soft_pairs_launch<double>(SoftArgs<double> &, SoftPairBuf<double> &, bool, bool,
                                       hipStream_t);
template int soft_pairs_backward_launch<float>(SoftArgs<float> &, SoftPairBuf<float> &,
                                               hipStream_t);
template int dibr_backward_merged_launch<float>(SoftArgs<float> &, SoftPairBuf<float> &,
                                                const RasterBwdArgs<float> &, hipStream_t);
template int dibr_backward_merged_launch<double>(SoftArgs<double> &, SoftPairBuf<double> &,
                                                 const RasterBwdArgs<double> &, hipStream_t);
template int soft_pairs_backward_launch<double>(SoftArgs<double> &, SoftPairBuf<double> &,
                                                hipStream_t);
template int soft_pairs_forward<float>(SoftArgs<float> &, void *, size_t, bool, bool,
                                       hipStream_t);
template int soft_pairs_forward<double>(SoftArgs<double> &, void *, size_t, bool, bool,
                                        hipStream_t);
template int soft_pairs_backward<float>(SoftArgs<float> &, void *, size_t, hipStream_t);
template int soft_pairs_backward<double>(SoftArgs<double> &, void *, size_t, hipStream_t);

}  // namespace kd
