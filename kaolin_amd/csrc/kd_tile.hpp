// kd_tile.hpp -- the per-tile face-list machinery shared by the raster and soft-mask kernels.
//
// A 256-thread workgroup owns a 16x16 pixel tile of one view; wave w owns the 8x8 sub-tile
// (w & 1, w >> 1).  tile_rounds() walks the tile's ordered coarse bin, keeps the faces whose exact
// pixel span touches the tile (ballot compaction keeps ascending face order), lets the caller
// stage their data in LDS (stage(k, row)), builds per-wave sub-lists of the faces touching each
// 8x8 sub-tile, and calls round(nsub) once per batch of at most CAP faces.  Across batches the
// faces keep ascending order, so a caller that processes batches in sequence sees the faces in
// exactly the order the reference loop does (minus faces whose box misses the pixel).
#pragma once

#include "kd_binning.hpp"

namespace kd {

struct TileGeom {
  int X0, X1, Y0, Y1;      // tile pixel rect (inclusive)
  int WX0, WX1, WY0, WY1;  // this wave's 8x8 sub-tile
  int px, py;              // this lane's pixel
  bool inimg, wave_live;
};

__device__ __forceinline__ TileGeom tile_geom(int H, int W) {
  const int ntx = (W + kTile - 1) / kTile;
  const int tx = blockIdx.x % ntx, ty = blockIdx.x / ntx;
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
  return t;
}

template <int CAP>
struct TileLists {
  int f[CAP];                   // local face index (ascending)
  Span span[CAP];
  unsigned short sub[4][CAP];   // per-wave sub-list: indices into f[]
  int cnt[4];
};

// Stage(k, face_row) fills the caller's LDS arrays for list entry k;
// Round(nsub, cnt) processes one batch of cnt tile faces (called by every thread; nsub, the
// length of this wave's sub-list, is wave-uniform).
template <int CAP, typename Stage, typename Round>
__device__ __forceinline__ void tile_rounds(TileLists<CAP> &L, const BinBuffers &bb, int64_t N,
                                            int b, int64_t lo, const TileGeom &t, Stage stage,
                                            Round round) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const BinGeom &g = bb.g;
  const int ct = (t.Y0 / g.ct) * g.nctx + (t.X0 / g.ct);
  const int n = bb.totals[(int64_t)b * g.nct() + ct];
  const int *bin = bb.bins + (int64_t)ct * N + lo;
  int cnt = 0;
  for (int base = 0; base < n; base += kBlock) {
    const int e = base + tid;
    int f = 0;
    bool ov = false;
    Span sp;
    if (e < n) {
      f = bin[e];
      sp = bb.spans[lo + f];
      ov = span_overlaps(sp, t.X0, t.X1, t.Y0, t.Y1);
    }
    int tot;
    const int pos = wg_compact(ov, L.cnt, tot);
    if (ov) {
      L.f[cnt + pos] = f;
      L.span[cnt + pos] = sp;
    }
    cnt += tot;
    if (cnt > CAP - kBlock || base + kBlock >= n) {
      __syncthreads();
      for (int k = tid; k < cnt; k += kBlock) stage(k, lo + L.f[k]);
      int nsub = 0;
      for (int k0 = 0; k0 < cnt; k0 += kWave) {
        const int k = k0 + lane;
        const bool ok =
            t.wave_live && k < cnt && span_overlaps(L.span[k], t.WX0, t.WX1, t.WY0, t.WY1);
        const uint64_t m = __ballot(ok);
        if (ok) L.sub[w][nsub + mbcnt(m)] = (unsigned short)k;
        nsub += __popcll(m);
      }
      __syncthreads();
      round(nsub, cnt);
      __syncthreads();
      cnt = 0;
    }
  }
}

// Orders LDS traffic between lanes of one wave (LDS ops of a wave complete in order; this keeps
// the compiler from moving them across the phase boundary).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace kd
