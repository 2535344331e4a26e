// Workgroup dispatch-rate probe: kernels whose workgroups do almost nothing, at the binning
// kernels' grid sizes and resource footprints (kernarg size, LDS, VGPRs), timed by rocprofv3
// --kernel-trace.  hipcc --offload-arch=gfx950 -O3 dispatch_rate.hip -o dispatch_rate
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big {
  int v[128];  // 512-byte kernarg, like BinJobs
};

__global__ __launch_bounds__(256) void k_empty(int *out) {
  if (threadIdx.x == 999) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_bigarg(Big a, int *out) {
  if (threadIdx.x == 999) out[0] = a.v[blockIdx.z];
}
__global__ __launch_bounds__(256) void k_lds(int *out) {
  __shared__ int s[5 * 1024];  // 20 KB
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (s[(threadIdx.x + 1) & 255] == 999) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_load(const int *in, int *out) {
  // one dependent global load + store per thread (a trivially short workgroup)
  const int i = (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
  out[i] = in[i] + 1;
}
__global__ __launch_bounds__(256) void k_strided(const int *in, int *out, int stride) {
  // like kd_bin_scan: 4-byte loads at a large stride (one cache line per lane)
  const int i = (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
  int s = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) s += in[((int64_t)i * stride + k * 64) % (1 << 24)];
  out[i] = s;
}

int main() {
  int *in, *out;
  hipMalloc(&in, sizeof(int) << 24);
  hipMalloc(&out, sizeof(int) << 24);
  hipMemset(in, 0, sizeof(int) << 24);
  Big b{};
  for (int rep = 0; rep < 20; ++rep) {
    for (int n : {1024, 1584, 8192}) {
      dim3 g(n / 8, 8, 1);
      hipLaunchKernelGGL(k_empty, g, dim3(256), 0, 0, out);
      hipLaunchKernelGGL(k_bigarg, dim3(n / 16, 8, 2), dim3(256), 0, 0, b, out);
      hipLaunchKernelGGL(k_lds, g, dim3(256), 0, 0, out);
      hipLaunchKernelGGL(k_load, g, dim3(256), 0, 0, in, out);
      hipLaunchKernelGGL(k_strided, g, dim3(256), 0, 0, in, out, 256);
    }
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
