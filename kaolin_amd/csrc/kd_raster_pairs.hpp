// kd_raster_pairs.hpp -- the reference's per-face raster test and the fp32 pair pipeline's tile
// body (kd_raster_fwd_pairs), shared with the fused DIB-R forward (kd_dibr_fwd_tiles in
// kd_softpair.hip).
#pragma once

#include "kd_binning.hpp"
#include "kd_raster.hpp"
#include "kd_tile.hpp"

namespace kd {

template <typename T>
struct ScaleUp {  // 2^(-min normal exponent): |w| * value >= |norm| => |w / norm| >= min normal
  static constexpr T value = 0x1p126f;
};
template <>
struct ScaleUp<double> {
  static constexpr double value = 0x1p1022;
};

// The reference per-face test (rasterization_cuda.cu:131-159) for one pixel whose centre passed
// the box test: edge functions, eps-normalised barycentrics (division before the sign test,
// exactly as the reference), depth.  EarlyReject adds an exact shortcut for pixels outside.
template <typename T, bool EarlyReject = true>
__device__ __forceinline__ bool raster_face_test(T x0, T y0, T ax, T ay, T bx, T by, T cx, T cy,
                                                 T az, T bz, T cz, float eps, T &w0, T &w1,
                                                 T &w2, T &z0) {
  const T a_edge_x = ax - x0, a_edge_y = ay - y0;
  const T b_edge_x = bx - x0, b_edge_y = by - y0;
  const T c_edge_x = cx - x0, c_edge_y = cy - y0;
  w0 = b_edge_x * c_edge_y - b_edge_y * c_edge_x;
  w1 = c_edge_x * a_edge_y - c_edge_y * a_edge_x;
  w2 = a_edge_x * b_edge_y - a_edge_y * b_edge_x;
  T norm = w0 + w1 + w2;
  norm = (T)((double)norm + copysign((double)eps, (double)norm));
  // Exact early rejection: with a finite nonzero norm, a nonzero non-NaN w of the opposite sign
  // whose quotient cannot round to -0 (|w| >= |norm| * 2^-(min normal exponent)) makes the
  // reference's `w / norm < 0` true.  Anything else takes the reference path below.
  if (EarlyReject && isfinite(norm) && norm != (T)0) {
    const bool nneg = norm < (T)0;
    const T big = ScaleUp<T>::value;
    const T an = fabs(norm);
    if (((w0 < (T)0) != nneg && w0 != (T)0 && !isnan(w0) && fabs(w0) * big >= an) ||
        ((w1 < (T)0) != nneg && w1 != (T)0 && !isnan(w1) && fabs(w1) * big >= an) ||
        ((w2 < (T)0) != nneg && w2 != (T)0 && !isnan(w2) && fabs(w2) * big >= an))
      return false;
  }
  w0 /= norm;
  w1 /= norm;
  w2 /= norm;
  if (w0 < (T)0. || w1 < (T)0. || w2 < (T)0.) return false;
  z0 = w0 * az + w1 * bz + w2 * cz;
  return true;
}

// ------------------------------------------------------------------------------------------
// fp32 forward as a (pixel, face) pair pipeline.  The lane-per-pixel loop above runs every face
// of the wave's sub-list on every lane, although a pixel centre is inside only ~1/5 of the boxes
// that hold it on this workload; here the full test runs once per (pixel, candidate face) pair
// with every lane busy, and the candidates are culled per pixel row by the triangle's edges:
//   stage  lane = face (once per tile): the keep-interval of every edge as an affine function of
//          the row, in tile-local pixel units, with a rigorous error margin (raster_cull_coefs);
//   A  lane = face: per row of the 8x8 sub-tile, [ceil(max lo - d), floor(min hi + d)] clipped
//      to the exact box span -> a 64-bit pixel mask; a 64x64 bit transpose across the wave gives
//      each pixel lane its candidate mask over the chunk; a DPP scan places the (pixel, face)
//      pairs in a per-wave list;
//   B  lane = pair: the reference's edge functions, eps-norm, divisions, inside test and depth;
//      an inside face posts key = (order-preserving bits of z, ~face index) with a 64-bit LDS
//      atomicMax per pixel.
//   The winner is the face with the largest z and, among equal z, the lowest index -- exactly
//   what the reference's ascending scan with strict `z > best` keeps (rasterization_cuda.cu:162),
//   provided no depth is NaN (-0 is folded to +0 first; -inf never wins there); a pixel that
//   meets a NaN depth replays the reference's sequential loop over its coarse bin instead.
//   The winner's weights are recomputed with the identical expression for the outputs.
// ------------------------------------------------------------------------------------------
constexpr int kRasterPairCap = 256;

__device__ __forceinline__ uint32_t ordered_f32(float z) {
  const uint32_t u = __float_as_uint(z + 0.0f);  // -0 -> +0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ unsigned long long ordered_f64(double z) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(z + 0.0);  // -0 -> +0
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// LDS of one tile of the pair pipeline.  fp64: the 64-bit winner key holds the depth rounded
// down to fp32 (monotone: the deepest face keeps the largest key) and the exact maximum depth is
// kept beside it (zx): the key's face is the reference's winner when its own depth is that
// maximum -- else (two faces within one fp32 step of depth, the lower index the shallower) the
// pixel replays the reference's loop.
template <typename T>
struct RasterPairsLDS {
  TileLists L;
  T geo[9][kCap];        // ax ay bx by cx cy (scaled), az bz cz
  // raster_cull_coefs (kd_binning), face frame: read from global memory in pass A (fp64 since
  // round 3: five workgroups per CU instead of four; fp32 since round 6 -- with the soft phase's
  // lane permutes, 8 KB less LDS makes the fused forward's 7 workgroups per CU instead of 6)
  float4 cull[2][1];
  unsigned short pair[4][kRasterPairCap];  // (q << 8) | sub-list entry
  unsigned long long key[4][64];
  unsigned long long zx[sizeof(T) == 8 ? 4 : 1][64];  // fp64: ordered exact maximum depth
  unsigned long long nan[4];
};

// Tile tl of view b (nbin: faces of its coarse bin, or -1).  Each thread owns pixel
// (t.px, t.py) of tile_geom(H, W, tl) and writes its outputs; wave w tests its own sub-tile's
// 64-face chunks.
// CLK (diagnostics, kd_dibr_fwd_tiles<true>): the wall clock at the end of the walk and tests
// (before the epilogue) into clk[slot].
// SPLIT > 1 (kd_tile.hpp tile_geom_part): the workgroup is part `part` of the tile; the waves of
// one sub-tile take its face chunks in turn (chunk c by role c % SPLIT) and post into the
// sub-tile's key row, whose maximum does not depend on the order; role 0 writes the outputs.
// uncm (nullptr: none): receives per sub-tile the mask of its uncovered in-image pixels.
template <typename T, bool CLK = false, int SPLIT = 1>
__device__ __forceinline__ void raster_pairs_tile(const RasterFwdArgs<T> &a, int b, int tl,
                                                  int nbin, RasterPairsLDS<T> &S,
                                                  long long *clk = nullptr, int part = 0,
                                                  uint64_t *uncm = nullptr) {
  constexpr bool kF64 = sizeof(T) == 8;
  TileLists &L = S.L;
  auto &s_geo = S.geo;
  auto &s_pair = S.pair;
  auto &s_key = S.key;
  auto &s_nan = S.nan;
  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W;
  const float M = fs.M;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  TileGeom t = SPLIT == 1 ? tile_geom(H, W, tl) : tile_geom_part<SPLIT>(H, W, tl, part);
  t.nbin = nbin;
  const int kw = t.sub;  // LDS key row of this wave's pixels
  const float sx = M / (float)W, sy = M / (float)H;  // px_cx / px_cy, first factor
  {  // (the walk's first barrier orders these before any pass B)
    s_key[kw][lane] = 0ull;
    if (kF64) S.zx[kF64 ? kw : 0][lane] = 0ull;
    if (lane == 0) s_nan[kw] = 0ull;
    if (uncm && lane == 0 && t.role == 0) uncm[t.sub] = 0ull;
  }
  // this wave's first row centre (pass A: row r's centre relative to it)
  const float ysub = px_cy(M, H, t.WY0);
  constexpr float kSlack = 1.f / 64.f;

  auto stage = [&](int k, int64_t fi) {
    T v[6];
    load_corners(fs, fi, v);
#pragma unroll
    for (int q = 0; q < 6; ++q) s_geo[q][k] = v[q];
    const T *zz = a.fvz + fi * a.fvz_fs;
    s_geo[6][k] = zz[0];
    s_geo[7][k] = zz[a.fvz_cs];
    s_geo[8][k] = zz[2 * a.fvz_cs];
  };
  // CLK: per-wave cycle counts of the phases (wave 0's are written out): [0] pass A row
  // intervals + transpose + scan, [1] pair placement, [2] pass B, [4] chunks, [5] candidate
  // pairs, [7] batches
  long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto now_clk = [&]() -> long long {
    return CLK ? (long long)__builtin_readcyclecounter() : 0ll;
  };
  // B: the reference's per-pixel test (rasterization_cuda.cu:131-162) over the current batch
  auto test_batch = [&](int total) {
    const long long tb0 = now_clk();
    struct Acc {
      long long &c, t0;
      bool on;
      __device__ ~Acc() {
        if (on) c += (long long)__builtin_readcyclecounter() - t0;
      }
    } acc{cyc[2], tb0, CLK};
    if (ablate(fs.dbg, 16)) return;
    wave_lds_sync();
    // branch-free (all three quotients, every load issued up front, selects), so the LDS reads
    // and the three division chains interleave: one wave per SIMD (small batches) would
    // otherwise wait out each dependent step
    struct PairIn {
      int q, f;
      T g[9];
      bool valid;
    };
    auto pair_load = [&](int e, PairIn &P) {
      P.valid = e < total;
      const int pr = s_pair[w][P.valid ? e : 0];  // pair: (pixel << 8) | entry
      P.q = (pr >> 8) & 63;
      const int k = L.sub[w][pr & 255];
#pragma unroll
      for (int i = 0; i < 9; ++i) P.g[i] = s_geo[i][k];
      P.f = L.f[k];
    };
    auto pair_key = [&](const PairIn &P, unsigned long long &key, bool &nan_hit, T &zout) {
      const float x0 = sx * (float)(2 * (t.WX0 + (P.q & 7)) + 1 - W);
      const float y0 = sy * (float)(H - 2 * (t.WY0 + (P.q >> 3)) - 1);
      const T a_edge_x = P.g[0] - (T)x0, a_edge_y = P.g[1] - (T)y0;
      const T b_edge_x = P.g[2] - (T)x0, b_edge_y = P.g[3] - (T)y0;
      const T c_edge_x = P.g[4] - (T)x0, c_edge_y = P.g[5] - (T)y0;
      const T w0 = b_edge_x * c_edge_y - b_edge_y * c_edge_x;
      const T w1 = c_edge_x * a_edge_y - c_edge_y * a_edge_x;
      const T w2 = a_edge_x * b_edge_y - a_edge_y * b_edge_x;
      T norm = w0 + w1 + w2;
      // (an exact fp32 shortcut for |norm| > |eps| 2^25 -- the double add then rounds back to
      // norm -- on a real branch measured slower: 128.1 -> 133.0 us at 8 views)
      norm = (T)((double)norm + copysign((double)a.eps, (double)norm));
      // rasterization_cuda.cu:131-162 (raster_face_test's sequence, without its branches)
      const T q0 = w0 / norm, q1 = w1 / norm, q2 = w2 / norm;
      const bool in = P.valid && !(q0 < (T)0. || q1 < (T)0. || q2 < (T)0.);
      const T z0 = q0 * P.g[6] + q1 * P.g[7] + q2 * P.g[8];
      nan_hit = in && isnan(z0);
      const bool ok = in && !isnan(z0) && z0 != (T)-INFINITY;
      float zk;  // fp64: the depth rounded down to fp32 in the key, the exact one in zx
      if constexpr (kF64)
        zk = __double2float_rd((double)z0);
      else
        zk = (float)z0;
      const unsigned long long packed = ((unsigned long long)ordered_f32(zk) << 32) |
                                        (unsigned long long)(0xffffffffu - (uint32_t)P.f);
      key = packed & (0ull - (unsigned long long)ok);
      zout = z0;
    };
    for (int e0 = 0; e0 < total; e0 += kWave) {
      PairIn pa;
      pair_load(e0 + lane, pa);
      unsigned long long ka;
      bool na;
      T za;
      pair_key(pa, ka, na, za);
      if (ka) {
        atomicMax(&s_key[kw][pa.q], ka);
        if constexpr (kF64) atomicMax(&S.zx[kw][pa.q], ordered_f64((double)za));
      }
      if (__ballot(na)) {  // (rare) a NaN depth: the pixel replays the reference loop
        if (na) atomicOr(&s_nan[kw], 1ull << pa.q);
      }
    }
    wave_lds_sync();
  };
  // pass A's culling coefficients of the wave's first chunk of the batch, loaded as soon as the
  // wave's sub-list is known (tile_rounds `pre`): their round trip overlaps the stage's instead
  // of following the barrier
  float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f, p4 = 0.f, p5 = 0.f, p6 = 0.f, p7 = 0.f;
  auto pre = [&](int nsub) {
    const int j = t.role * kWave + lane;
    wave_lds_sync();  // this wave's own sub-list stores
    // (only entries of the sub-list: past nsub -- e.g. an empty sub-list -- L.sub holds stale
    // or never-written bytes)
    float4 cl = make_float4(0.f, 0.f, 0.f, 0.f), ch = cl;
    if (j < nsub) {
      const int64_t r = lo + L.f[L.sub[w][j]];
      cl = a.bb.cull[2 * r];
      ch = a.bb.cull[2 * r + 1];
    }
    p0 = cl.x; p1 = cl.y; p2 = cl.z; p3 = cl.w;
    p4 = ch.x; p5 = ch.y; p6 = ch.z; p7 = ch.w;
  };
  auto round = [&](int nsub, int) {
    if (ablate(fs.dbg, 1)) return;
    if (nsub == 0) return;
    int total = 0;
    if (CLK) cyc[7] += 1;
#pragma unroll 1
    for (int c = t.role; c < 4; c += SPLIT) {
      if (c * kWave >= nsub) break;
      long long tc0 = now_clk();
      if (CLK) cyc[4] += 1;
      const int ls = w;
      const int ns = nsub;
      const int ox = t.WX0, oy = t.WY0;
      const float ysb = ysub;
      // A: lane = face (chunk entry c*64 + lane): culled row intervals -> 64-bit pixel mask
      const int j = c * kWave + lane;
      uint64_t fm = 0ull;
      if (j < ns) {
        const int k = L.sub[ls][j];
        const Span sp = L.span[k];
        const int rx0 = max(sp.x0 - ox, 0), rx1 = min(sp.x1 - ox, 7);
        const int ry0 = max(sp.y0 - oy, 0), ry1 = min(sp.y1 - oy, 7);
        // face frame -> this sub-tile: columns shift by WX0 - span.x0, rows by the centre offset
        const float xo = (float)(ox - sp.x0);
        const float dref = ysb - px_cy(M, H, sp.y0);
        // (the wave's first chunk: loaded by `pre` below, in flight with the stage's loads)
        float4 cl, ch;
        if (c == t.role) {
          cl = make_float4(p0, p1, p2, p3);
          ch = make_float4(p4, p5, p6, p7);
        } else {
          cl = a.bb.cull[2 * (lo + L.f[k])];
          ch = a.bb.cull[2 * (lo + L.f[k]) + 1];
        }
        const float l0 = cl.x - xo, l2 = cl.z - xo, h0 = ch.x - xo, h2 = ch.z - xo;
        // only the rows of the face's own span (a lane's loop: the wave runs the longest span,
        // not all 8 rows); drow[r] is recomputed from sy (px_cy's first factor: the same bits)
        for (int r = ry0; r <= ry1; ++r) {
          const float d = (sy * (float)(H - 2 * (oy + r) - 1) - ysb) + dref;
          const float plo = fmaxf(fmaf(cl.y, d, l0), fmaf(cl.w, d, l2)) - kSlack;
          const float phi = fminf(fmaf(ch.y, d, h0), fmaf(ch.w, d, h2)) + kSlack;
          const int xs = max((int)ceilf(__builtin_amdgcn_fmed3f(plo, -1.f, 9.f)), rx0);
          const int xe = min((int)floorf(__builtin_amdgcn_fmed3f(phi, -1.f, 9.f)), rx1);
          const uint32_t bits = xs <= xe ? ((2u << xe) - (1u << xs)) : 0u;
          fm |= (uint64_t)bits << (8 * r);
        }
      }
      // lane = pixel: candidate mask over the chunk, pairs placed by a DPP scan
      uint64_t m = wave_transpose64(fm);
      const int cnt = __popcll(m);
      const int incl = wave_incl_scan(cnt);
      const int ctot = __builtin_amdgcn_readlane(incl, 63);
      if (CLK) {
        const long long t1 = now_clk();
        cyc[0] += t1 - tc0;
        tc0 = t1;
        cyc[5] += ctot;
      }
      // pairs placed rank-major: step r writes every pixel lane's r-th candidate, packed by
      // the lanes still holding one (ballot + mbcnt), so every window of kRasterPairCap pairs
      // is filled by all lanes at once -- pixel-major runs let only the few lanes whose runs
      // cover a window work on it (the poles: ~2000 pairs per wave and chunk).  Pass B does
      // not depend on the order (the key maximum).
      (void)ctot;
      int pos = total;
      const int qbits = (lane << 8) | (c << 6);
      while (true) {
        const bool act = m != 0ull;
        const uint64_t am = __ballot(act);
        if (!am) break;
        const int n = __popcll(am);
        const int slot = pos + mbcnt(am);
        const unsigned short pr = (unsigned short)(qbits | (act ? (int)__builtin_ctzll(m) : 0));
        const bool now = act && slot < kRasterPairCap;
        if (now) s_pair[w][slot] = pr;
        if (pos + n > kRasterPairCap) {  // the window filled within this step
          if (CLK) {
            const long long t1 = now_clk();
            cyc[1] += t1 - tc0;
            tc0 = t1;
          }
          test_batch(kRasterPairCap);
          if (CLK) tc0 = now_clk();
          if (act && !now) s_pair[w][slot - kRasterPairCap] = pr;
          pos += n - kRasterPairCap;
        } else {
          pos += n;
        }
        m &= m - 1ull;
      }
      if (CLK) {
        const long long t1 = now_clk();
        cyc[1] += t1 - tc0;
        tc0 = t1;
      }
      total = pos;
    }
    if (total) test_batch(total);
  };
  tile_rounds(L, a.bb, (int)(hi - lo), b, lo, t, stage, round, fs.dbg, NeverDone(), pre);
  if (CLK && KD_DIAG && clk && threadIdx.x == 0) {
    const int64_t nb = (int64_t)gridDim.x * gridDim.y, slot = blockIdx.y * gridDim.x + blockIdx.x;
    clk[slot] = wall_clock64();
#pragma unroll
    for (int i = 0; i < 8; ++i) clk[(1 + i) * nb + slot] = cyc[i];  // wave 0's phase counts
  }

  if (t.role != 0 || !t.inimg || ablate(fs.dbg, 8192)) return;
  const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
  const T x0 = (T)px_cx(M, W, t.px), y0 = (T)px_cy(M, H, t.py);
  int best = -1;
  T bw0 = (T)0, bw1 = (T)0, bw2 = (T)0;
  bool replay = (s_nan[kw] >> lane) & 1ull;
  // the winner's features (D <= kFr) are loaded with its corners: one round trip, not two
  constexpr int kFr = 4;
  const bool fr_ok = a.D <= kFr;
  T fr[3][kFr];
  if (!replay && s_key[kw][lane] != 0ull) {
    best = (int)(0xffffffffu - (uint32_t)(s_key[kw][lane] & 0xffffffffull));
    T v[6];
    load_corners(fs, lo + best, v);
    const T *zz = a.fvz + (lo + best) * a.fvz_fs;
    const T za = zz[0], zb = zz[a.fvz_cs], zc = zz[2 * a.fvz_cs];
    if (fr_ok) {
      const T *r = a.feat + (lo + best) * 3 * a.D;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int d = 0; d < kFr; ++d) fr[i][d] = d < a.D ? r[i * a.D + d] : (T)0;
    }
    T z0;
    raster_face_test<T>(x0, y0, v[0], v[1], v[2], v[3], v[4], v[5], za, zb, zc, a.eps, bw0, bw1,
                        bw2, z0);
    // fp64: the key's face is the winner only if its depth is the exact maximum
    if constexpr (kF64) replay = ordered_f64((double)z0) != S.zx[kw][lane];
  }
  if (replay) {
    // the reference's sequential loop over this pixel's coarse bin (ascending faces)
    best = -1;
    bw0 = bw1 = bw2 = (T)0;
    const BinGeom &g = a.bb.g;
    const int ct = (t.py >> g.sh) * g.nctx + (t.px >> g.sh);
    int n;
    const int *bin = bin_list(a.bb, b, ct, lo, (int)(hi - lo), -1, n);
    T max_z0 = (T)-INFINITY;
    for (int e = 0; e < n; ++e) {
      const int f = bin ? bin[e] : e;
      if (!pspan_has(pack_span(a.bb.spans[lo + f]), t.px, t.py)) continue;
      T v[6];
      load_corners(fs, lo + f, v);
      const T *zz = a.fvz + (lo + f) * a.fvz_fs;
      T w0, w1, w2, z0;
      if (!raster_face_test<T>(x0, y0, v[0], v[1], v[2], v[3], v[4], v[5], zz[0],
                               zz[a.fvz_cs], zz[2 * a.fvz_cs], a.eps, w0, w1, w2, z0))
        continue;
      if (z0 <= max_z0) continue;
      max_z0 = z0;
      best = f;
      bw0 = w0;
      bw1 = w1;
      bw2 = w2;
    }
  }
  a.face_idx[p] = best;
  if (uncm && best < 0) atomicOr(&uncm[t.sub], 1ull << lane);
  T *wo = a.weights + p * 3;
  T *io = a.interp + p * a.D;
  if (a.D == 3 && (best < 0 || (fr_ok && !replay))) {  // one store per row (bw* stay 0: no face)
    store3(wo, bw0, bw1, bw2);
    T i0 = (T)0, i1 = (T)0, i2 = (T)0;
    if (best >= 0) {
      i0 = bw0 * fr[0][0] + bw1 * fr[1][0] + bw2 * fr[2][0];
      i1 = bw0 * fr[0][1] + bw1 * fr[1][1] + bw2 * fr[2][1];
      i2 = bw0 * fr[0][2] + bw1 * fr[1][2] + bw2 * fr[2][2];
    }
    store3(io, i0, i1, i2);
  } else if (best >= 0) {
    wo[0] = bw0;
    wo[1] = bw1;
    wo[2] = bw2;
    if (fr_ok && !replay) {
#pragma unroll
      for (int d = 0; d < kFr; ++d)
        if (d < a.D) io[d] = bw0 * fr[0][d] + bw1 * fr[1][d] + bw2 * fr[2][d];
    } else {
      const T *r = a.feat + (lo + best) * 3 * a.D;
      for (int d = 0; d < a.D; ++d)
        io[d] = bw0 * r[d] + bw1 * r[a.D + d] + bw2 * r[2 * a.D + d];
    }
  } else {
    wo[0] = (T)0;
    wo[1] = (T)0;
    wo[2] = (T)0;
    for (int d = 0; d < a.D; ++d) io[d] = (T)0;
  }
}

}  // namespace kd
