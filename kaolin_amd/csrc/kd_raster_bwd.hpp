// kd_raster_bwd.hpp -- the raster backward's tile body (kd_raster_bwd_tile), shared with the
// merged DIB-R backward launch (kd_dibr_bwd in kd_softpair.hip).
#pragma once

#include "kd_raster.hpp"
#include "kd_tile.hpp"

namespace kd {

template <typename T>
struct RasterBwdArgs {
  int B, H, W;
  int64_t F;
  int D;
  const T *grad;
  const int64_t *face_idx;
  const T *weights, *fvi, *feat;
  float eps;
  T *grad_fvi, *grad_feat;
  int dbg;
  VertexOut<T> vo;  // vo.grad set: the corner gradients go to the vertices (VTX bodies)
};

// ------------------------------------------------------------------------------------------
// Backward terms of one covered pixel (rasterization_cuda.cu:271-399) into out[]: out[0..5]
// the 6 corner terms summed over the D features, out[6 + ii*DMAX + d] the feature terms
// (register array, static indices only).  v: the 6 corner coordinates, c: the corner features
// as [3][DMAX] (register arrays).
// ------------------------------------------------------------------------------------------
template <typename T, int DMAX>
__device__ __forceinline__ void raster_bwd_pixel(const T *v, const T wts[3], const T *g,
                                                 const T *c, int D, float eps,
                                                 T out[6 + 3 * DMAX]) {
  T gd[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) gd[d] = d < D ? g[d] : (T)0;
#pragma unroll
  for (int ii = 0; ii < 3; ++ii)
#pragma unroll
    for (int d = 0; d < DMAX; ++d) out[6 + ii * DMAX + d] = gd[d] * wts[ii];
  const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
  const T aw = wts[0], bw = wts[1], cw = wts[2];
  const T x0 = aw * ax + bw * bx + cw * cx;
  const T y0 = aw * ay + bw * by + cw * cy;
  const T m = bx - ax, p = by - ay, n = cx - ax, q = cy - ay, s = x0 - ax, t = y0 - ay;
  const T k1 = s * q - n * t;
  const T k2 = m * t - s * p;
  T k3 = m * q - n * p;
  k3 = (T)((double)k3 + copysign((double)eps, (double)k3));
  const T zero = (T)0;
  const T dk1dm = zero, dk1dn = -t, dk1dp = zero, dk1dq = s, dk1ds = q, dk1dt = -n;
  const T dk2dm = t, dk2dn = zero, dk2dp = -s, dk2dq = zero, dk2ds = -p, dk2dt = m;
  const T dk3dm = q, dk3dn = -p, dk3dp = -n, dk3dq = m, dk3ds = zero, dk3dt = zero;
  const T dw1dm = dk1dm * k3 - dk3dm * k1, dw1dn = dk1dn * k3 - dk3dn * k1;
  const T dw1dp = dk1dp * k3 - dk3dp * k1, dw1dq = dk1dq * k3 - dk3dq * k1;
  const T dw1ds = dk1ds * k3 - dk3ds * k1, dw1dt = dk1dt * k3 - dk3dt * k1;
  const T dw2dm = dk2dm * k3 - dk3dm * k2, dw2dn = dk2dn * k3 - dk3dn * k2;
  const T dw2dp = dk2dp * k3 - dk3dp * k2, dw2dq = dk2dq * k3 - dk3dq * k2;
  const T dw2ds = dk2ds * k3 - dk3ds * k2, dw2dt = dk2dt * k3 - dk3dt * k2;
  const T dw1[6] = {-(dw1dm + dw1dn + dw1ds), -(dw1dp + dw1dq + dw1dt), dw1dm, dw1dp, dw1dn,
                    dw1dq};
  const T dw2[6] = {-(dw2dm + dw2dn + dw2ds), -(dw2dp + dw2dq + dw2dt), dw2dm, dw2dp, dw2dn,
                    dw2dq};
  const T kk = k3 * k3;
  // fp32: one hardware reciprocal (1 ulp) for the D quotients g_d / k3^2 -- gradient accuracy, not
  // bit-exactness, is the bar here (the reference's own float atomics reorder these sums)
  T rkk = (T)0;
  if constexpr (sizeof(T) == 4) rkk = __builtin_amdgcn_rcpf(kk);
#pragma unroll
  for (int j = 0; j < 6; ++j) out[j] = (T)0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if (d < D) {
      const T c0 = c[d], c1 = c[DMAX + d], c2 = c[2 * DMAX + d];  // (c: [3][DMAX])
      const T dldI = sizeof(T) == 4 ? gd[d] * rkk : gd[d] / kk;
#pragma unroll
      for (int j = 0; j < 6; ++j) out[j] += dldI * ((c1 - c0) * dw1[j] + (c2 - c0) * dw2[j]);
    }
  }
}

// A workgroup's samples, at most one per lane (p < 0: none), summed per face.  Every sample writes
// its terms to LDS; samples are grouped by face: an LDS hash table gives each face a slot, the
// slot's LDS counter gives each sample its rank among the slot's samples, a prefix sum over the
// slots turns (slot, rank) into a position, and the group sum of each (face, term) is then added
// by one lane and flushed with one float atomic per (group, face, term), a face's terms on
// adjacent lanes (its 6 corner terms and its 3*D feature terms are contiguous in memory).
// (Summation order varies with the LDS counters, as it does across groups with the float atomics.)
// ROWKEY: the lanes' samples may belong to different views b, so the keys are the rows b*F + f
// (the launcher checks B*F < 2^31); otherwise all lanes share view b and the keys are faces.
template <typename T, int DMAX, bool VTX, bool ROWKEY>
__device__ __forceinline__ void raster_bwd_group(const RasterBwdArgs<T> &ra, int64_t p, int b) {
  const int D = ra.D, dbg = ra.dbg;
  const int64_t F = ra.F;
  const T *__restrict__ grad = ra.grad;
  const int64_t *__restrict__ face_idx = ra.face_idx;
  const T *__restrict__ weights = ra.weights;
  const T *__restrict__ fvi = ra.fvi;
  const T *__restrict__ feat = ra.feat;
  const float eps = ra.eps;
  T *grad_fvi = ra.grad_fvi;
  T *grad_feat = ra.grad_feat;
  constexpr int SMAX = 6 + 3 * DMAX;
  // fp64: the table holds one pass of terms at a time -- the 6 geometry terms, then the 3 D
  // feature terms -- so it is 20 KB instead of 32 and the kernel keeps five workgroups per CU
  constexpr bool kSplit = sizeof(T) == 8;
  constexpr int CW = kSplit ? (3 * DMAX > 6 ? 3 * DMAX : 6) : SMAX;  // table columns
  // odd row stride (in 4-byte words): a sample's row write (lanes on different rows, one term)
  // and a slot's column sums (lanes on one row, consecutive terms) are both bank-conflict free
  constexpr int SROW = (CW * (int)sizeof(T) / 4) % 2 ? CW : CW + 1;
  constexpr int HT = kBlock;  // slots >= distinct faces of a group
  __shared__ int s_key[HT];
  __shared__ int s_n[HT];  // samples per slot (their ranks come from the counter)
  __shared__ T s_con[kBlock][SROW];
  __shared__ short s_off[HT];
  __shared__ int s_list[HT];
  __shared__ int s_cnt[4];
  const int S = 6 + 3 * D;
  const int tid = threadIdx.x;
  s_key[tid] = -1;
  s_n[tid] = 0;
  __syncthreads();
  int h = -1, rank = 0;
  T c[SMAX];
  if (p >= 0) {
    // the sample's weights and incoming gradient do not depend on its face: issued with it
    const int64_t f = face_idx[p];
    const T wts[3] = {weights[p * 3], weights[p * 3 + 1], weights[p * 3 + 2]};
    T gd[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) gd[d] = d < D ? grad[p * D + d] : (T)0;
    if (f >= 0 && f < F) {
      const int64_t tf = (int64_t)b * F + f;
      // the face's corners and features first: their round trip overlaps the LDS hash insert
      // below (the compiler keeps global loads after an LDS atomic loop)
      T fv[6], fc[3 * DMAX];
#pragma unroll
      for (int j = 0; j < 6; ++j) fv[j] = fvi[tf * 6 + j];
#pragma unroll
      for (int ii = 0; ii < 3; ++ii)
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          fc[ii * DMAX + d] = d < D ? feat[tf * 3 * D + ii * D + d] : (T)0;
      const int key = ROWKEY ? (int)tf : (int)f;
      // slot = the key's low bits (linear probing): neighbouring faces take neighbouring slots, so
      // the slot-ordered flush below adds consecutive face rows in one atomic instruction
      unsigned u = (unsigned)key & (HT - 1);
      for (;;) {  // <= 256 keys in 256 slots: terminates
        const int old = atomicCAS(&s_key[u], -1, key);
        if (old == -1 || old == key) break;
        u = (u + 1) & (HT - 1);
      }
      h = (int)u;
      rank = atomicAdd(&s_n[h], 1);
      raster_bwd_pixel<T, DMAX>(fv, wts, gd, fc, D, eps, c);
    }
  }
  __syncthreads();
  // slot sizes -> positions (prefix sum over slots), and the list of occupied slots
  const int sz = s_n[tid];
  int total;
  const int off = wg_exclusive_scan(sz, s_cnt, total);
  s_off[tid] = (short)off;
  int nocc;
  const bool occ = sz > 0;
  const int pos = wg_compact(occ, s_cnt, nocc);
  if (occ) s_list[pos] = tid;
  __syncthreads();
  // the sample's terms go to its position in slot order, so a slot's terms are contiguous rows;
  // pass q holds terms [c0, c1) (one pass of all S terms unless kSplit)
  for (int q = 0; q < (kSplit ? 2 : 1); ++q) {
    const int c0 = kSplit && q ? 6 : 0, c1 = kSplit && !q ? 6 : S;
    if (q) __syncthreads();  // the previous pass's sums are done with the table
    if (h >= 0) {
      const int ps = s_off[h] + rank;
      if (c0 == 0) {
#pragma unroll
        for (int j = 0; j < 6; ++j) s_con[ps][j] = c[j];
      }
      if (c1 > 6) {
#pragma unroll
        for (int ii = 0; ii < 3; ++ii)
#pragma unroll
          for (int d = 0; d < DMAX; ++d)
            if (d < D) s_con[ps][6 + ii * D + d - c0] = c[6 + ii * DMAX + d];
      }
    }
    __syncthreads();
    // items of the pass: VTX corners 0..2 of a face (terms 2k, 2k+1 -> the corner's vertex),
    // then single terms g0..c1-1
    const int ncorner = VTX && c0 == 0 ? 3 : 0;
    const int g0 = ncorner ? 6 : c0;
    const int SI = ncorner + (c1 - g0);
    // !VTX: every slot's grad_fvi terms of the pass first, then its feature terms, so that an
    // atomic instruction's lanes add consecutive slots' rows of one array (float atomics execute
    // at the memory side, one request per 64-byte segment an instruction touches)
    const int nA = VTX ? 0 : max(0, min(c1, 6) - g0);  // grad_fvi terms per slot
    const int gB = max(g0, 6), nB = c1 - gB;            // feature terms per slot
    for (int idx = tid; idx < nocc * SI; idx += kBlock) {
      int i, jj;
      if constexpr (VTX) {
        i = idx / SI;
        jj = idx - i * SI;  // (the item index j; the term below)
      } else if (idx < nocc * nA) {
        i = idx / nA;
        jj = g0 + (idx - i * nA);
      } else {
        const int k2 = idx - nocc * nA;
        i = k2 / nB;
        jj = gB + (k2 - i * nB);
      }
      const int slot = s_list[i];
      const int ns = s_n[slot];
      const int o = s_off[slot];
      const int64_t row = ROWKEY ? (int64_t)s_key[slot] : (int64_t)b * F + s_key[slot];
      if constexpr (VTX) {
        const int j = jj;
        if (j < ncorner) {
          T vx = (T)0, vy = (T)0;
          for (int r = 0; r < ns; ++r) {  // independent reads: pipelined
            vx += s_con[o + r][2 * j];
            vy += s_con[o + r][2 * j + 1];
          }
          vertex_add(ra.vo, row, j, vx, vy);
          continue;
        }
        jj = g0 + (j - ncorner);
      }
      T v = (T)0;
      for (int r = 0; r < ns; ++r) v += s_con[o + r][jj - c0];  // independent reads: pipelined
      if (v == (T)0 || ablate(dbg, 128)) continue;
      if (jj < 6)
        atomicAdd(grad_fvi + row * 6 + jj, v);
      else if (grad_feat)
        atomicAdd(grad_feat + row * 3 * D + (jj - 6), v);
    }
  }
}

// One workgroup per 16x16 tile of a view's pixels (rasterization_cuda.cu:238-402 per pixel).
template <typename T, int DMAX, bool VTX = false>
__device__ __forceinline__ void raster_bwd_tile_body(const RasterBwdArgs<T> &ra, int d, int n,
                                                     int ntl) {
  const int H = ra.H, W = ra.W;
  const int tid = threadIdx.x;
  const int ntx = (W + kTile - 1) / kTile;
  // XCD-aware: workgroups are dealt to the 8 XCDs round-robin (d % 8 is the XCD: callers keep
  // it so), so XCD x gets the contiguous band of tiles [x n/8, (x+1) n/8): neighbouring tiles
  // (which share faces) share one L2
  if ((n & 7) == 0 && !ablate(ra.dbg, (1 << 17))) d = (d & 7) * (n >> 3) + (d >> 3);
  const int b = d / ntl, tl = d - b * ntl;
  const int px = (tl % ntx) * kTile + (tid & 15);
  const int py = (tl / ntx) * kTile + (tid >> 4);
  const int64_t p = px < W && py < H ? ((int64_t)b * H + py) * W + px : -1;
  raster_bwd_group<T, DMAX, VTX, false>(ra, p, b);
}

}  // namespace kd
