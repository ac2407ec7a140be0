// Quasi-Monte Carlo pi (PiEstimator map, src/examples/.../PiEstimator.java):
// count the points of the 2-D Halton sequence (bases 2 and 3) with index in
// [offset, offset + n) that fall inside the circle inscribed in the unit
// square.  Bit-exact with the numpy mapper in hbmr/examples/pi.py: the radical
// inverse is evaluated with the same IEEE double operation sequence
// (f = 1/base, r += f * digit, f /= base) and FP contraction is off, so no FMA
// changes a rounding.  fp64 VALU work; one 64-bit atomic per wavefront.
#include "common.h"

namespace {

#pragma clang fp contract(off)
__device__ __forceinline__ double radical_inverse(long long i, int base) {
  double f = 1.0 / (double)base;
  double r = 0.0;
  while (i > 0) {
    const long long q = i / base;
    r += f * (double)(i - q * base);
    i = q;
    f /= (double)base;
  }
  return r;
}

__global__ __launch_bounds__(256) void pi_halton_kernel(long long offset, long long n,
                                                        unsigned long long* inside) {
#pragma clang fp contract(off)
  unsigned long long cnt = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const long long idx = offset + k + 1;  // the reference's index + 1
    const double x = radical_inverse(idx, 2) - 0.5;
    const double y = radical_inverse(idx, 3) - 0.5;
    const double xx = x * x;
    const double yy = y * y;
    cnt += (xx + yy <= 0.25) ? 1ull : 0ull;
  }
  for (int o = HBMR_WAVE / 2; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, HBMR_WAVE);
  if ((threadIdx.x & (HBMR_WAVE - 1)) == 0 && cnt) atomicAdd(inside, cnt);
}

}  // namespace

extern "C" {

// inside: one device uint64, accumulated into (zero it first for a fresh count).
int hbmr_pi_halton(long long offset, long long n, unsigned long long* inside,
                   hipStream_t stream) {
  if (n <= 0) return 0;
  const long long threads = 256;
  long long blocks = (n + threads * 16 - 1) / (threads * 16);  // ~16 points per lane
  if (blocks > 32768) blocks = 32768;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pi_halton_kernel, dim3((unsigned)blocks), dim3((unsigned)threads), 0, stream,
                     offset, n, inside);
  return (int)hipGetLastError();
}

}  // extern "C"
