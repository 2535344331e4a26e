// Microbenchmark: no-return fp32 global atomicAdd throughput on gfx950 for different lane->address
// patterns (how many distinct cache lines one wave instruction touches).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

__global__ void k_atomic(const int *idx, const float *val, int n, float *out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(out + idx[i], val[i]);
}
__global__ void k_store(const int *idx, const float *val, int n, float *out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[idx[i]] = val[i];
}

static void run(const char *name, const std::vector<int> &h, float *d_out, bool store = false) {
  const int n = (int)h.size();
  int *d_idx; float *d_val;
  (void)hipMalloc(&d_idx, n * 4); (void)hipMalloc(&d_val, n * 4);
  (void)hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemset(d_val, 0, n * 4);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    float ms;
    (void)hipEventRecord(a);
    if (store) k_store<<<n / 256, 256>>>(d_idx, d_val, n, d_out);
    else k_atomic<<<n / 256, 256>>>(d_idx, d_val, n, d_out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  printf("%-44s %9d ops %8.1f us %7.1f Gop/s\n", name, n, best * 1e3, n / best / 1e6);
  (void)hipFree(d_idx); (void)hipFree(d_val);
}

int main() {
  const int n = 8 << 20, nf = 400000 * 6;
  float *d_out; (void)hipMalloc(&d_out, nf * 4); (void)hipMemset(d_out, 0, nf * 4);
  std::mt19937 g(1);
  std::vector<int> h(n);
  for (int i = 0; i < n; ++i) h[i] = (int)(g() % nf);
  run("random lanes (64 lines / instr)", h, d_out);
  run("random lanes, plain store", h, d_out, true);
  for (int i = 0; i < n; i += 64) { int base = (int)(g() % (nf / 64)) * 64; for (int l = 0; l < 64; ++l) h[i + l] = base + l; }
  run("64 consecutive floats (4 lines / instr)", h, d_out);
  for (int i = 0; i < n; i += 16) { int base = (int)(g() % (nf / 16)) * 16; for (int l = 0; l < 16; ++l) h[i + l] = base + l; }
  run("4 x 16 consecutive floats (4 lines, scattered)", h, d_out);
  for (int i = 0; i < n; i += 6) { int base = (int)(g() % (nf / 6)) * 6; for (int l = 0; l < 6 && i + l < n; ++l) h[i + l] = base + l; }
  run("runs of 6 floats (a face's corners)", h, d_out);
  for (int i = 0; i < n; i += 64) { int base = (int)(g() % (nf / 64)) * 64; for (int l = 0; l < 64; ++l) h[i + l] = base + (l % 8); }
  run("64 lanes on 8 addresses (same line)", h, d_out);
  return 0;
}
