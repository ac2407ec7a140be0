// Shared helpers for the hbmr CDNA4 (gfx950) kernels.
//
// Every kernel in native/kernels is written for MI355X directly: 64-lane
// wavefronts, MFMA matrix cores, 160 KiB LDS per CU, 8 XCDs.  Launchers take
// raw device pointers plus a hipStream_t so the same objects link into both the
// Python runtime (libhbmr.so, loaded next to PyTorch) and the standalone Pipes
// GPU task binaries (native/apps).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define HBMR_WAVE 64
#define HBMR_NXCD 8

#define HBMR_RETURN_IF_ERROR(expr)                 \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) return (int)_e;          \
  } while (0)

// bf16 <-> f32 by bit manipulation (round-to-nearest-even on the way down).
__device__ __forceinline__ float hbmr_bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ uint16_t hbmr_f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // keep NaN a NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Unpack 8 bf16 held in a uint4 into 8 floats.
__device__ __forceinline__ void hbmr_unpack8(const uint4 v, float f[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

// acc[j] += round_half_even(f[j] * scale) for the int64 fixed-point combiner.
// __float2ll_rn is a ~15-op sequence; when every scaled value fits in int32
// (|x| < 128 at scale 2^24 — the normal case) v_rndne + v_cvt_i32 is exact
// and 3 ops.  The per-lane branch skips the slow path when no lane needs it.
__device__ __forceinline__ void hbmr_fx_accum8(const float f[8], float scale, long long acc[8]) {
  float y[8];
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    y[j] = f[j] * scale;
    m = fmaxf(m, fabsf(y[j]));
  }
  if (m < 2147483520.f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (long long)(int)__builtin_rintf(y[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += __float2ll_rn(y[j]);
  }
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 T1):
// consecutive logical tiles land on the same XCD (same L2).
__device__ __forceinline__ uint32_t hbmr_xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t q = nwg / HBMR_NXCD, r = nwg % HBMR_NXCD;
  const uint32_t xcd = bid % HBMR_NXCD, idx = bid / HBMR_NXCD;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
