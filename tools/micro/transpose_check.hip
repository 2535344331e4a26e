// Checks kd::wave_transpose64 (gfx950 lane movers, no branches) against the block-swap form
// (wave_transpose64_blocks) and a plain LDS transpose on random and structured bit matrices.
//   hipcc -O3 --offload-arch=gfx950 -I kaolin_amd/csrc tools/micro/transpose_check.hip -o /tmp/tc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

#include "kd_tile.hpp"

__global__ void k_transpose(const uint64_t *in, uint64_t *out_new, uint64_t *out_blk,
                            uint64_t *out_lds) {
  __shared__ uint64_t s[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t x = in[i];
  out_new[i] = kd::wave_transpose64(x);
  out_blk[i] = kd::wave_transpose64_blocks(x);
  s[w][lane] = x;
  __syncthreads();
  uint64_t t = 0;
  for (int j = 0; j < 64; ++j) t |= ((s[w][j] >> lane) & 1ull) << j;
  out_lds[i] = t;
}

int main() {
  const int nblk = 512, n = nblk * 256;
  std::vector<uint64_t> h(n);
  std::mt19937_64 rng(7);
  for (int i = 0; i < n; ++i) {
    const int kind = (i / 64) % 4;
    uint64_t v = rng();
    if (kind == 1) v &= rng();            // sparse
    if (kind == 2) v = 1ull << (i % 64);  // identity
    if (kind == 3) v = (i & 1) ? ~0ull : 0ull;
    h[i] = v;
  }
  uint64_t *d_in, *d_a, *d_b, *d_c;
  (void)hipMalloc(&d_in, n * 8);
  (void)hipMalloc(&d_a, n * 8);
  (void)hipMalloc(&d_b, n * 8);
  (void)hipMalloc(&d_c, n * 8);
  (void)hipMemcpy(d_in, h.data(), n * 8, hipMemcpyHostToDevice);
  k_transpose<<<nblk, 256>>>(d_in, d_a, d_b, d_c);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("launch failed\n");
    return 2;
  }
  std::vector<uint64_t> a(n), b(n), c(n);
  (void)hipMemcpy(a.data(), d_a, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), d_b, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(c.data(), d_c, n * 8, hipMemcpyDeviceToHost);
  int bad_new = 0, bad_blk = 0;
  for (int i = 0; i < n; ++i) {
    bad_new += a[i] != c[i];
    bad_blk += b[i] != c[i];
    if (a[i] != c[i] && bad_new <= 4)
      printf("lane %d: new %016llx lds %016llx\n", i, (unsigned long long)a[i],
             (unsigned long long)c[i]);
  }
  printf("transpose check: %d lanes, wave_transpose64 mismatches %d, block form %d\n", n, bad_new,
         bad_blk);
  return (bad_new || bad_blk) ? 1 : 0;
}
