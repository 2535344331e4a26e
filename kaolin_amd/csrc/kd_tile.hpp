// kd_tile.hpp -- the per-tile face-list machinery shared by the raster and soft-mask kernels.
//
// A 256-thread workgroup owns a 16x16 pixel tile of one view; wave w owns the 8x8 sub-tile
// (w & 1, w >> 1).  tile_rounds() walks the tile's ordered coarse bin, keeps the faces whose exact
// pixel span touches the tile (ballot compaction keeps ascending face order), lets the caller
// stage their data in LDS (stage(k, row)), builds per-wave sub-lists of the faces touching each
// 8x8 sub-tile, and calls round(nsub, cnt) once per batch of at most kCap faces.  Across batches
// the faces keep ascending order, so a caller that processes batches in sequence sees the faces
// in exactly the order the reference loop does (minus faces whose box misses the pixel).
// A caller whose result depends only on a prefix of the faces (the soft mask's first K) stops
// the walk early through `done`.
//
// The box test itself is done on the exact integer pixel spans (kd_common.hpp make_span): pixel
// (x, y) passes the reference's half-open float box test iff x0 <= x <= x1 and y0 <= y <= y1.
// SubSpans keeps a wave's sub-list (<= kCap = 4 x 64 entries) in registers: lane l holds entry
// c*64 + l of chunk c, so per-pixel hit masks are 4 compares and a ballot, no LDS traffic.
#pragma once

#include "kd_binning.hpp"

namespace kd {

constexpr int kCap = 256;     // faces per batch (LDS list)
constexpr int kPrefetch = 4;  // bin chunks loaded ahead by tile_rounds

struct TileGeom {
  int X0, X1, Y0, Y1;      // tile pixel rect (inclusive)
  int WX0, WX1, WY0, WY1;  // this wave's 8x8 sub-tile
  int px, py;              // this lane's pixel
  bool inimg, wave_live;
  int nbin;                // faces in the tile's coarse bin when known (tile order), else -1
  // face filter boxes of tile_rounds (default: the tile and the wave's sub-tile); a caller whose
  // pixels do not all need faces may shrink them to the pixels that do (wave_live = false when
  // the wave has none)
  int FX0, FX1, FY0, FY1;      // tile filter
  int SX0, SX1, SY0, SY1;      // this wave's sub-list filter
  int sub;                     // this wave's 8x8 sub-tile in the 16x16 tile frame (0..3)
  int role;                    // split tiles: which of the sub-tile's waves this is (0 owns pixels)
  int bbase;                   // the coarse bin's base when already loaded (with nbin), else
                               // kNoBinBase: tile_rounds loads it
};
constexpr int kNoBinBase = INT_MIN;

// (view, fine tile) of dispatch slot d of n tile slots: the bins' heaviest-first order
// (tile_order) when the bins were built, else slot order.
__device__ __forceinline__ void tile_of_slot(const BinBuffers &bb, int H, int W, int d, int n,
                                             int &b, int &tile, int &nbin, int dbg = 0) {
  if (bb.order && bb.nchunk > 0) {
    const int ntiles = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    // XCD-aware: workgroups are dealt to the 8 XCDs round-robin (d % 8), and the order holds a
    // coarse tile's fine tiles consecutively; within each group of 32 workgroups fine tile j of
    // coarse tile g runs at d = 8 j + g, so the tiles sharing a coarse bin share one L2.
    if ((d | 31) < n && !ablate(dbg, (1 << 17))) d = (d & ~31) | ((d & 7) << 2) | ((d >> 3) & 3);
    const int2 v = bb.order[d];
    b = v.x / ntiles;
    tile = v.x - b * ntiles;
    nbin = v.y;
  } else {
    const int ntiles = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    b = d / ntiles;
    tile = d - b * ntiles;
    nbin = -1;
  }
}
// ... of this workgroup of a (tiles, views) grid
__device__ __forceinline__ void tile_of_block(const BinBuffers &bb, int H, int W, int &b,
                                              int &tile, int &nbin, int dbg = 0) {
  if (bb.order && bb.nchunk > 0) {
    tile_of_slot(bb, H, W, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, b, tile,
                 nbin, dbg);
  } else {
    b = blockIdx.y;
    tile = blockIdx.x;
    nbin = -1;
  }
}

__device__ __forceinline__ TileGeom tile_geom(int H, int W, int tile) {
  const int ntx = (W + kTile - 1) / kTile;
  const int tx = tile % ntx, ty = tile / ntx;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  TileGeom t;
  t.X0 = tx * kTile;
  t.Y0 = ty * kTile;
  t.X1 = min(t.X0 + kTile - 1, W - 1);
  t.Y1 = min(t.Y0 + kTile - 1, H - 1);
  t.WX0 = t.X0 + (w & 1) * 8;
  t.WY0 = t.Y0 + (w >> 1) * 8;
  t.WX1 = min(t.WX0 + 7, W - 1);
  t.WY1 = min(t.WY0 + 7, H - 1);
  t.px = t.WX0 + (lane & 7);
  t.py = t.WY0 + (lane >> 3);
  t.inimg = t.px < W && t.py < H;
  t.wave_live = t.WX0 < W && t.WY0 < H;
  t.nbin = -1;
  t.FX0 = t.X0;
  t.FX1 = t.X1;
  t.FY0 = t.Y0;
  t.FY1 = t.Y1;
  t.SX0 = t.WX0;
  t.SX1 = t.WX1;
  t.SY0 = t.WY0;
  t.SY1 = t.WY1;
  t.sub = w;
  t.role = 0;
  t.bbase = kNoBinBase;
  return t;
}
__device__ __forceinline__ TileGeom tile_geom(int H, int W) { return tile_geom(H, W, blockIdx.x); }

// Split tiles (few views: more workgroups than tiles fill the chip).  Part `part` of SPLIT (1, 2
// or 4) of a 16x16 tile is a 256-thread workgroup over 4 / SPLIT of its 8x8 sub-tiles (SPLIT 2:
// the upper or lower 16x8 half; SPLIT 4: one sub-tile), with SPLIT waves per sub-tile: wave w
// takes sub-tile part * (4 / SPLIT) + w % (4 / SPLIT) in role w / (4 / SPLIT).  Every wave of a
// sub-tile maps its lanes to the sub-tile's pixels; role 0 owns them (writes the outputs), the
// other roles share the sub-tile's face chunks.  The workgroup's filter box is its part.
template <int SPLIT>
__device__ __forceinline__ TileGeom tile_geom_part(int H, int W, int tile, int part) {
  static_assert(SPLIT == 1 || SPLIT == 2 || SPLIT == 4, "SPLIT in {1, 2, 4}");
  constexpr int NS = 4 / SPLIT;  // sub-tiles per part
  const int ntx = (W + kTile - 1) / kTile;
  const int tx = tile % ntx, ty = tile / ntx;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = part * NS + w % NS;
  TileGeom t;
  // the part's pixel rect: the union of its sub-tiles (s0 .. s0 + NS - 1)
  const int s0 = part * NS;
  t.X0 = tx * kTile + (NS == 1 ? (s0 & 1) * 8 : 0);
  t.Y0 = ty * kTile + (s0 >> 1) * 8;
  t.X1 = min(t.X0 + (NS == 1 ? 7 : kTile - 1), W - 1);
  t.Y1 = min(t.Y0 + (NS == 4 ? kTile - 1 : 7), H - 1);
  t.WX0 = tx * kTile + (s & 1) * 8;
  t.WY0 = ty * kTile + (s >> 1) * 8;
  t.WX1 = min(t.WX0 + 7, W - 1);
  t.WY1 = min(t.WY0 + 7, H - 1);
  t.px = t.WX0 + (lane & 7);
  t.py = t.WY0 + (lane >> 3);
  t.inimg = t.px < W && t.py < H;
  t.wave_live = t.WX0 < W && t.WY0 < H;
  t.nbin = -1;
  t.FX0 = t.X0;
  t.FX1 = t.X1;
  t.FY0 = t.Y0;
  t.FY1 = t.Y1;
  t.SX0 = t.WX0;
  t.SX1 = t.WX1;
  t.SY0 = t.WY0;
  t.SY1 = t.WY1;
  t.sub = s;
  t.role = w / NS;
  t.bbase = kNoBinBase;
  return t;
}

// (view, fine tile, part) of this workgroup of a (tiles * SPLIT, views) grid: dispatch slot d
// is part d % SPLIT of tile slot d / SPLIT (heaviest-first order when the bins were built), after
// the XCD-aware regrouping of tile_of_slot applied to the parts' slots (the parts of a tile and
// their coarse-bin siblings share an XCD's L2).
template <int SPLIT>
__device__ __forceinline__ void tile_of_block_split(const BinBuffers &bb, int H, int W, int &b,
                                                    int &tile, int &part, int &nbin,
                                                    int dbg = 0) {
  if (SPLIT == 1) {
    part = 0;
    tile_of_block(bb, H, W, b, tile, nbin, dbg);
    return;
  }
  const int n = gridDim.x * gridDim.y;
  int d = blockIdx.y * gridDim.x + blockIdx.x;
  if ((d | 31) < n && !ablate(dbg, (1 << 17))) d = (d & ~31) | ((d & 7) << 2) | ((d >> 3) & 3);
  part = d % SPLIT;
  const int ts = d / SPLIT;
  const int ntiles = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
  if (bb.order && bb.nchunk > 0) {
    const int2 v = bb.order[ts];
    b = v.x / ntiles;
    tile = v.x - b * ntiles;
    nbin = v.y;
  } else {
    b = ts / ntiles;
    tile = ts - b * ntiles;
    nbin = -1;
  }
}

struct TileLists {
  int f[kCap];                   // local face index (ascending)
  Span span[kCap];
  unsigned char sub[4][kCap];    // per-wave sub-list: indices into f[]
  int cnt[4];
  int nsub[4];                   // the sub-lists' lengths of the current batch
};

// Packed span: lo = x0 | x1 << 16, hi = y0 | y1 << 16 (int16 fields, sign-extended on unpack).
struct PSpan {
  uint32_t lo, hi;
};
__device__ __forceinline__ PSpan pack_span(Span s) {
  PSpan p;
  p.lo = (uint32_t)(uint16_t)s.x0 | ((uint32_t)(uint16_t)s.x1 << 16);
  p.hi = (uint32_t)(uint16_t)s.y0 | ((uint32_t)(uint16_t)s.y1 << 16);
  return p;
}
__device__ __forceinline__ bool pspan_has(PSpan p, int x, int y) {
  const int x0 = (int)(int16_t)(p.lo & 0xffff), x1 = (int)(int16_t)(p.lo >> 16);
  const int y0 = (int)(int16_t)(p.hi & 0xffff), y1 = (int)(int16_t)(p.hi >> 16);
  return x >= x0 && x <= x1 && y >= y0 && y <= y1;
}

struct SubSpans {
  PSpan s[4];        // chunk c, lane l -> sub-list entry c*64 + l
  int k[4];          // its index into the tile list
};

__device__ __forceinline__ SubSpans load_subspans(const TileLists &L, int nsub) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  SubSpans r;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j = c * kWave + lane;
    if (j < nsub) {
      r.k[c] = L.sub[w][j];
      r.s[c] = pack_span(L.span[r.k[c]]);
    } else {
      r.k[c] = 0;
      r.s[c].lo = 0xffff0001u;  // empty: x0 = 1 > x1 = -1
      r.s[c].hi = 0xffff0001u;
    }
  }
  return r;
}

struct NeverDone {
  __device__ bool operator()() const { return false; }
};
struct NoPrefetch {
  __device__ void operator()(int) const {}
};

// `done()` (evaluated by every thread; must return a workgroup-uniform value, e.g. through
// __syncthreads_and) lets a caller stop the walk once later faces cannot matter any more.
// `pre(nsub)` (per wave, before the batch's face data is staged): the wave's sub-list of the
// batch is in L.sub[w] / L.nsub[w] (written by the wave itself), so a caller can issue the loads
// its round needs per sub-list entry here, in flight together with the stage's loads.
// nview: faces of view b (rows [lo, lo + nview)), walked in full when the bin overflowed.
template <typename Stage, typename Round, typename Done = NeverDone, typename Pre = NoPrefetch>
__device__ __forceinline__ void tile_rounds(TileLists &L, const BinBuffers &bb, int nview, int b,
                                            int64_t lo, const TileGeom &t, Stage stage,
                                            Round round, int dbg = 0, Done done = Done(),
                                            Pre pre = Pre()) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const BinGeom &g = bb.g;
  const int ct = (t.Y0 >> g.sh) * g.nctx + (t.X0 >> g.sh);
  int n;
  const int *bin;
  if (t.nbin == 0) {  // an empty bin never overflows: no header load
    n = 0;
    bin = nullptr;
  } else if (t.bbase != kNoBinBase && t.nbin >= 0) {  // (bin_list with its loads done by the caller)
    n = t.bbase < 0 ? nview : t.nbin;
    bin = t.bbase < 0 ? nullptr : bb.bins + (int64_t)bb.xper * lo + t.bbase;
  } else {
    bin = bin_list(bb, b, ct, lo, nview, t.nbin, n);
  }
  // one batch of cnt faces in L.f / L.span: sub-lists, the caller's prefetch, staging, its round
  auto flush = [&](int cnt) {
    __syncthreads();
    int nsub = 0;
    for (int k0 = 0; k0 < cnt; k0 += kWave) {
      const int k = k0 + lane;
      const bool ok =
          t.wave_live && k < cnt && span_overlaps(L.span[k], t.SX0, t.SX1, t.SY0, t.SY1);
      const uint64_t m = __ballot(ok);
      if (ok) L.sub[w][nsub + mbcnt(m)] = (unsigned char)k;
      nsub += __popcll(m);
    }
    if (lane == 0) L.nsub[w] = nsub;
    pre(nsub);
    if (!ablate(dbg, 2))
      for (int k = tid; k < cnt; k += kBlock) stage(k, lo + L.f[k]);
    __syncthreads();
    if (!ablate(dbg, 4)) round(nsub, cnt);
    __syncthreads();
  };
  int cnt = 0;
  // kPrefetch chunks of bin entries and their spans are loaded up front (two dependent
  // round trips per kPrefetch * 256 entries instead of per 256)
  for (int base0 = 0; base0 < n; base0 += kBlock * kPrefetch) {
    int fr[kPrefetch];
    Span spr[kPrefetch];
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
      const int e = base0 + u * kBlock + tid;
      fr[u] = e < n ? (bin ? bin[e] : e) : 0;
    }
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
      const int e = base0 + u * kBlock + tid;
      if (e < n) spr[u] = bb.spans[lo + fr[u]];
    }
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
      if (base0 + u * kBlock >= n) break;
      const int e = base0 + u * kBlock + tid;
      const int f = fr[u];
      const Span sp = spr[u];
      const bool ov = e < n && span_overlaps(sp, t.FX0, t.FX1, t.FY0, t.FY1);
      int tot;
      const int pos = wg_compact(ov, L.cnt, tot);
      // a batch holds at most kCap faces: flush first if this chunk would overflow it
      if (cnt + tot > kCap) {
        flush(cnt);
        cnt = 0;
        if (done()) return;
      }
      if (ov) {
        L.f[cnt + pos] = f;
        L.span[cnt + pos] = sp;
      }
      cnt += tot;
    }
  }
  if (cnt > 0) flush(cnt);
}

// Orders LDS traffic between lanes of one wave (LDS ops of a wave complete in order; this keeps
// the compiler from moving them across the phase boundary).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP: row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast 15 / 31 carry the row totals across rows.  No LDS traffic.
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// x of lane (lane ^ SH), for the whole wave without the LDS crossbar (ds_bpermute): gfx950's
// permlane swaps for 32 / 16, DPP for 8 / 4 / 2 / 1.  Both candidates are materialised before the
// select (empty asm), so the cross-lane reads run with every lane active (a DPP or permlane read
// issued under a partial EXEC would see `old` for the inactive source lanes).
template <int SH>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
  const int lane = threadIdx.x & 63;
  uint32_t a, b;
  bool hi;
  if constexpr (SH == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    a = r[1];  // lanes 0..31: the upper half's values
    b = r[0];  // lanes 32..63: the lower half's values
    hi = lane >= 32;
  } else if constexpr (SH == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    a = r[1];  // even rows: the odd rows' values
    b = r[0];  // odd rows: the even rows' values
    hi = (lane & 16) != 0;
  } else if constexpr (SH == 8) {  // (every source lane exists: bound_ctrl, no `old` to set up)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, true);  // row_ror:8
  } else if constexpr (SH == 4) {
    // banks 0 and 2 of each row (lanes with bit 2 clear) read row_shl:4, banks 1 and 3 row_shr:4
    // into the same register (bank_mask): no select
    const int t = __builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xf, 0x5, false);  // row_shl:4
    return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)x, 0x114, 0xf, 0xa, false);  // row_shr:4
  } else if constexpr (SH == 2) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, true);  // [2,3,0,1]
  } else {
    static_assert(SH == 1, "lane_xor: SH in {1, 2, 4, 8, 16, 32}");
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, true);  // [1,0,3,2]
  }
  asm volatile("" : "+v"(a), "+v"(b));
  return hi ? b : a;
}

// One block-swap stage of the transpose in the form of the reference text (a lane-dependent
// branch per stage: both sides run under partial EXEC); wave_transpose64_blocks keeps it as the
// check of wave_transpose64 (tools/micro/transpose_check.hip).
template <int SH>
__device__ __forceinline__ uint64_t transpose_step(uint64_t x, uint64_t mlo) {
  const int lane = threadIdx.x & 63;
  const uint32_t ylo = lane_xor<SH>((uint32_t)x);
  const uint32_t yhi = lane_xor<SH>((uint32_t)(x >> 32));
  const uint64_t y = ((uint64_t)yhi << 32) | ylo;
  return (lane & SH) ? ((x & ~mlo) | ((y & ~mlo) >> SH)) : ((x & mlo) | ((y & mlo) << SH));
}

__device__ __forceinline__ uint64_t wave_transpose64_blocks(uint64_t x) {
  x = transpose_step<32>(x, 0x00000000ffffffffull);
  x = transpose_step<16>(x, 0x0000ffff0000ffffull);
  x = transpose_step<8>(x, 0x00ff00ff00ff00ffull);
  x = transpose_step<4>(x, 0x0f0f0f0f0f0f0f0full);
  x = transpose_step<2>(x, 0x3333333333333333ull);
  x = transpose_step<1>(x, 0x5555555555555555ull);
  return x;
}

// Stage SH <= 8 without a branch, on each 32-bit half: a lane with bit SH clear keeps its low
// SH-bit parts (m) and takes its partner's low parts moved up; a lane with the bit set keeps the
// high parts and takes the partner's high parts moved down.  So every lane SENDS its half rotated
// by its own parity (clear: right by SH, its high parts land on the low places; set: left by SH)
// and merges the received word under its keep mask with one bit-field insert.
template <int SH>
__device__ __forceinline__ uint32_t transpose_half(uint32_t h, uint32_t keep, uint32_t rot) {
  const uint32_t s = __builtin_amdgcn_alignbit(h, h, rot);  // rotate right
  return (h & keep) | (lane_xor<SH>(s) & ~keep);  // v_bfi_b32
}

// lane: the lane id, opaque to the compiler (wave_transpose64), so that the per-lane masks are
// recomputed at each use (three instructions a stage) rather than hoisted into eight VGPRs
template <int SH>
__device__ __forceinline__ uint64_t transpose_step_rot(uint64_t x, uint32_t m, uint32_t lane) {
  const uint32_t neg = (uint32_t)((int)(lane << (31 - __builtin_ctz(SH))) >> 31);  // 0 / ~0
  const uint32_t keep = m ^ neg;
  const uint32_t rot = (neg & (uint32_t)(32 - SH)) | (~neg & (uint32_t)SH);
  const uint32_t lo = transpose_half<SH>((uint32_t)x, keep, rot);
  const uint32_t hi = transpose_half<SH>((uint32_t)(x >> 32), keep, rot);
  return ((uint64_t)hi << 32) | lo;
}

// 64x64 bit-matrix transpose across a wave: lane l bit j -> lane j bit l.  Every lane of the
// wave must be active.  The stages are the block swaps of wave_transpose64_blocks, written for
// gfx950's lane movers so that no stage branches:
//   32: one v_permlane32_swap of the two halves (the low half's upper lanes <-> the high half's
//       lower lanes is exactly the 32-bit block swap);
//   16: the two 16-bit parts each lane keeps / sends packed into one word each (v_perm), one
//       v_permlane16_swap of the packed words, unpacked by v_perm -- the same two selectors for
//       every lane;
//   8, 4, 2, 1: transpose_step_rot (rotate, DPP exchange, bit-field insert).
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x) {
  {
    const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)x, (uint32_t)(x >> 32), false, false);
    x = ((uint64_t)r[1] << 32) | r[0];
  }
  {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t a = __builtin_amdgcn_perm(hi, lo, 0x05040100u);  // low 16-bit parts
    const uint32_t b = __builtin_amdgcn_perm(hi, lo, 0x07060302u);  // high 16-bit parts
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    // even rows: a' = own low parts, b' = the partner's low parts; odd rows: a' = the partner's
    // high parts, b' = own high parts -- both unpack as (a' part, b' part)
    const uint32_t nlo = __builtin_amdgcn_perm(r[1], r[0], 0x05040100u);
    const uint32_t nhi = __builtin_amdgcn_perm(r[1], r[0], 0x07060302u);
    x = ((uint64_t)nhi << 32) | nlo;
  }
  uint32_t lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  x = transpose_step_rot<8>(x, 0x00ff00ffu, lane);
  x = transpose_step_rot<4>(x, 0x0f0f0f0fu, lane);
  x = transpose_step_rot<2>(x, 0x33333333u, lane);
  x = transpose_step_rot<1>(x, 0x55555555u, lane);
  return x;
}

// Exclusive prefix sum over the 256 threads of the workgroup; total returned in `total`.
// scratch: 4 ints of LDS.
__device__ __forceinline__ int wg_exclusive_scan(int v, int *scratch, int &total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = wave_incl_scan(v);
  if (lane == kWave - 1) scratch[w] = x;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / kWave; ++k) {
    const int c = scratch[k];
    off += (k < w) ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + x - v;
}

}  // namespace kd
