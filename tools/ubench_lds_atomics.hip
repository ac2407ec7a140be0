// Micro-benchmark: LDS atomic throughput on gfx950 (ds_add_f32 / ds_add_u32 /
// ds_add_rtn_u32 / plain ds_write), distinct addresses per lane, no conflicts.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_atomics.hip -o /tmp/ub
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  __shared__ float sf[4096];
  __shared__ unsigned su[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += 256) { sf[i] = 0.f; su[i] = 0; }
  __syncthreads();
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int a = (t + j * 256 + it) & 4095;
      if (MODE == 0) atomicAdd(&sf[a], 1.0f);
      if (MODE == 1) atomicAdd(&su[a], 1u);
      if (MODE == 2) acc += atomicAdd(&su[a], 1u);
      if (MODE == 3) sf[a] = (float)it;
      if (MODE == 4) { // same address per 16-lane group (4 distinct per wave)
        atomicAdd(&sf[(t / 16 + j * 64) & 4095], 1.0f);
      }
    }
  }
  __syncthreads();
  out[blockIdx.x * 256 + t] = sf[t] + (float)su[t] + (float)acc;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 256 * 4);
  const int blocks = 256 * 4, iters = 2000;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_rtn_u32", "ds_write_b32",
                         "ds_add_f32_16way_same"};
  for (int mode = 0; mode < 5; ++mode) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      switch (mode) {
        case 0: k<0><<<blocks, 256>>>(out, iters); break;
        case 1: k<1><<<blocks, 256>>>(out, iters); break;
        case 2: k<2><<<blocks, 256>>>(out, iters); break;
        case 3: k<3><<<blocks, 256>>>(out, iters); break;
        case 4: k<4><<<blocks, 256>>>(out, iters); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 256 * iters * 8;
    printf("%-24s %8.3f ms  %8.2f Gop/s  %6.3f lane-ops/clk/CU(@2.1GHz)\n", names[mode], ms,
           ops / ms / 1e6, ops / (ms * 1e-3) / 256 / 2.1e9);
  }
  return 0;
}
