// bf16 GEMM on the MFMA matrix cores (the Mars-style
// matmul map task of BASELINE config 4).
//
//   C[M, N] (fp32 or bf16) = A[M, K] · B[K, N],   A row-major, B given as
//   Bt[N, K] row-major (both operands K-contiguous), fp32 accumulation.
//
// Structure (cdna_hip_programming.md §5, CDNA4):
// * 256×256 output tile per 512-thread workgroup (8 waves as 2 (M) × 4 (N),
//   each wave 128×64 = 8×4 tiles of v_mfma_f32_16x16x32_bf16);
// * K-steps of 64: the next step's A and B tiles (2 × 32 KiB) are staged with
//   global_load_lds (16-B LDS-DMA, no VGPR round trip) into the other half of a
//   double-buffered 128 KiB LDS image while the current step computes;
// * LDS rows are 128 B; 16-B chunk c of row r is stored at chunk c ^ (r & 7)
//   (XOR applied to the DMA's SOURCE address, since the DMA writes lane-linear)
//   so the 16 rows a ds_read_b128 fragment load touches spread over the banks;
// * one barrier per K-step; bijective XCD-aware tile order (each XCD's L2
//   serves neighbouring tiles of the same A row-panel).
// Ragged shapes run natively in v1 (any M, N; K % 8 == 0): operand tiles are
// staged by buffer_load … lds through a per-tile buffer resource whose range
// ends at the operand's last valid row, and a piece past K gets an offset
// beyond the range, so the hardware's range check zero-fills every piece
// outside the matrix (no padded copies, no predicated VGPR path); stores are
// masked to M × N.  v2 (HBMR_GEMM=2) keeps the tile-multiple contract.
#include "common.h"

#include <cstdlib>
#include "../include/hbmr/hbmr.h"

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kGemmThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;            // one operand tile: 32 KiB
constexpr int kStageBytes = 2 * kTileBytes;          // A + B
constexpr int kGemmLds = 2 * kStageBytes;            // double buffered: 128 KiB

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Buffer resource over rows [row0, min(row0 + 256, rows)) of a K-contiguous
// operand: reads past its last valid row return zero.  Built from
// wave-uniform values only (kernel arguments and blockIdx).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const __bf16* G, long ld, long row0,
                                                            long rows) {
  const long nr = rows - row0 < kBM ? rows - row0 : kBM;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(G + row0 * ld), 0, (int)(nr * ld * 2),
                                           0x00020000);
}

// stage_tile through a tile resource: piece (r, c) at k = k0 + 8 src_c; a
// piece at k >= K is sent past the range (zero-filled) — K % 8 == 0 keeps
// every 16-B piece wholly inside or outside the matrix.
__device__ __forceinline__ void stage_tile_rs(char* lds, __amdgpu_buffer_rsrc_t rs, long ld,
                                              long k0, long K, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = i * kGemmThreads + tid;
    const int r = p >> 3, c = p & 7;
    const long k = k0 + ((c ^ (r & 7)) << 3);
    const uint32_t off = k < K ? (uint32_t)((r * ld + k) * 2) : 0x80000000u;
    char* dst = lds + (size_t)(i * kGemmThreads + (tid & ~63)) * 16;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, off, 0, 0, 0);
  }
}

template <bool OUT_BF16>
__global__ __launch_bounds__(kGemmThreads, 1) void gemm_bf16_tn_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, void* __restrict__ Cv, long M,
    long N, long K, float alpha, double* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // 2 × 4 waves
  const long tiles_n = (N + kBN - 1) / kBN;
  const uint32_t t = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const long bm = t / tiles_n, bn = t % tiles_n;
  const long m0 = bm * kBM, n0 = bn * kBN;
  const int nk = (int)((K + kBK - 1) / kBK);
  const __amdgpu_buffer_rsrc_t ra = tile_rsrc(A, K, m0, M);
  const __amdgpu_buffer_rsrc_t rb = tile_rsrc(Bt, K, n0, N);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_tile_rs(smem, ra, K, 0, K, tid);
  stage_tile_rs(smem + kTileBytes, rb, K, 0, K, tid);

  const int fr = lane & 15;    // fragment row (A) / column (B) within a 16-tile
  const int fq = lane >> 4;    // k-group: elements k = 8 fq .. 8 fq + 7 of a 32-wide k-step

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * kStageBytes;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
      stage_tile_rs(nxt, ra, K, (long)(kt + 1) * kBK, K, tid);
      stage_tile_rs(nxt + kTileBytes, rb, K, (long)(kt + 1) * kBK, K, tid);
    }
    const char* la = cur;
    const char* lb = cur + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + fq;  // logical 16-B chunk of the row
      bf16x8_t a[8], b[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wm * 128 + i * 16 + fr;
        a[i] = *reinterpret_cast<const bf16x8_t*>(la + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + fr;
        b[j] = *reinterpret_cast<const bf16x8_t*>(lb + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // C/D map of 16x16x32: col = lane & 15, row = 4 (lane >> 4) + reg.
  // partials != null: the tile's sum of the stored C values (fp64), one per
  // workgroup — the map task's checksum without a second pass over C.
  double csum = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long col = n0 + wn * 64 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long row = m0 + wm * 128 + i * 16 + fq * 4 + r;
        if (row >= M || col >= N) continue;        // ragged edge tile
        const float v = acc[i][j][r] * alpha;
        if (OUT_BF16) {
          const uint16_t h = hbmr_f32_to_bf16(v);
          reinterpret_cast<uint16_t*>(Cv)[row * N + col] = h;
          csum += (double)__uint_as_float((uint32_t)h << 16);
        } else {
          reinterpret_cast<float*>(Cv)[row * N + col] = v;
          csum += (double)v;
        }
      }
    }
  }
  if (partials) {
    __shared__ double s_red[kGemmThreads / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
    if (lane == 0) s_red[wave] = csum;
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < kGemmThreads / 64; ++w) s += s_red[w];
      partials[blockIdx.x] = s;
    }
  }
}

// ---- v2: 4 waves of 128×128 (v_mfma_f32_32x32x16_bf16) ----------------------
// Same 256×256 tile, K-step, LDS image (XOR-swizzled 128-B rows) and DMA
// staging as v1, but 4 waves as 2 (M) × 2 (N), each owning a 128×128 block =
// 4×4 tiles of 32×32: per K-step a wave reads its 128 A rows and 128 B rows
// once (128 KiB of LDS reads per workgroup instead of v1's 192 KiB for the
// same 8.4 MFLOP), and issues 64 MFMAs of 32x32x16 (256 accumulators per lane,
// AGPR-resident).  32x32x16 fragments: lane l holds row (l & 31) at k-offset
// 8 (l >> 5) of a 16-wide step; C register r of lane l is row
// (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31.
constexpr int kGemmThreads2 = 256;

__device__ __forceinline__ void stage_tile2(char* lds, const __bf16* __restrict__ G, long ld,
                                            long row0, long k0, int tid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = i * kGemmThreads2 + tid;  // 16-B piece index in the tile image
    const int r = p >> 3, c = p & 7;
    const int src_c = c ^ (r & 7);
    const __bf16* g = G + (row0 + r) * ld + k0 + src_c * 8;
    char* dst = lds + (size_t)(i * kGemmThreads2 + (tid & ~63)) * 16;
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)dst, 16, 0, 0);
  }
}

template <bool OUT_BF16>
__global__ __launch_bounds__(kGemmThreads2, 1) void gemm_bf16_tn_v2_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, void* __restrict__ Cv, long M,
    long N, long K, float alpha, double* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;   // 2 × 2 waves
  const long tiles_n = N / kBN;
  const uint32_t t = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const long bm = t / tiles_n, bn = t % tiles_n;
  const long m0 = bm * kBM, n0 = bn * kBN;
  const int nk = (int)(K / kBK);

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  stage_tile2(smem, A, K, m0, 0, tid);
  stage_tile2(smem + kTileBytes, Bt, K, n0, 0, tid);

  const int fr = lane & 31;   // fragment row (A) / column (B) within a 32-tile
  const int h = lane >> 5;    // k-offset 8h within a 16-wide step

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * kStageBytes;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
      stage_tile2(nxt, A, K, m0, (long)(kt + 1) * kBK, tid);
      stage_tile2(nxt + kTileBytes, Bt, K, n0, (long)(kt + 1) * kBK, tid);
    }
    const char* la = cur;
    const char* lb = cur + kTileBytes;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + h;  // logical 16-B chunk of the 128-B row
      bf16x8_t a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 128 + i * 32 + fr;
        a[i] = *reinterpret_cast<const bf16x8_t*>(la + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 128 + j * 32 + fr;
        b[j] = *reinterpret_cast<const bf16x8_t*>(lb + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // per (i, j) one lane base pointer; the 16 rows of a register block are
  // uniform multiples of N (scalar offsets)
  double csum = 0.0;
  const long lane_off = (m0 + wm * 128 + 4 * h) * N + n0 + wn * 128 + fr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long base = lane_off + (long)(i * 32) * N + j * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long off = base + (long)((r & 3) + 8 * (r >> 2)) * N;
        const float v = acc[i][j][r] * alpha;
        if (OUT_BF16) {
          const uint16_t hv = hbmr_f32_to_bf16(v);
          reinterpret_cast<uint16_t*>(Cv)[off] = hv;
          csum += (double)__uint_as_float((uint32_t)hv << 16);
        } else {
          reinterpret_cast<float*>(Cv)[off] = v;
          csum += (double)v;
        }
      }
    }
  }
  if (partials) {
    __shared__ double s_red2[kGemmThreads2 / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
    if (lane == 0) s_red2[wave] = csum;
    __syncthreads();
    if (tid == 0) {
      double sum = 0.0;
#pragma unroll
      for (int w = 0; w < kGemmThreads2 / 64; ++w) sum += s_red2[w];
      partials[blockIdx.x] = sum;
    }
  }
}


// Ring kernels (HBMR_GEMM=3 / 4 / 5 / 6): WM × WN waves, each owning a
// (256/WM) × (256/WN) block of 32×32 tiles (v_mfma_f32_32x32x16_bf16), over a
// 4-slot ring of K-steps of 32 (4 × 32 KiB of LDS): the loads of K-step k+4
// are issued in the middle of step k (into step k's slot, once every wave
// holds its last fragments of it), so a step's operands have three steps to
// arrive from L2 / HBM instead of one, and a step waits only for its own
// pieces (a counted vmcnt: the younger steps stay in flight across the
// barrier, which is a bare s_barrier — __syncthreads()'s release fence waits
// for every outstanding LDS-DMA, vmcnt(0), and would drain the ring).
// Fragments are software-pipelined: the second 16-wide half of a K-step
// loads while the first half's MFMAs run, the next K-step's first half while
// the second half's run.  PRIO: s_setprio(1) over the MFMA blocks.
// LDS image of a 256×32 operand tile: rows r and r+1 share a 128-B line
// L = r/2 (16-B chunk q = 4 (r & 1) + c), chunk q at slot q ^ ((L >> 1) & 3):
// the 16 lanes of a ds_read_b128 pass (16 consecutive rows, one k-chunk) hit
// 16 distinct bank groups.
constexpr int kBKr = 32;
constexpr int kTiler = kBM * kBKr * 2;    // 16 KiB
constexpr int kStager = 2 * kTiler;       // A + B: 32 KiB
constexpr int kRingr = 4;
constexpr int kLdsr = kRingr * kStager;   // 128 KiB

template <int THREADS>
__device__ __forceinline__ void stage_ring(char* lds, const __bf16* __restrict__ G, long ld,
                                           long row0, long k0, int tid) {
#pragma unroll
  for (int i = 0; i < kTiler / 16 / THREADS; ++i) {
    const int p = i * THREADS + tid;        // 16-B slot in the image (line-major)
    const int L = p >> 3, slot = p & 7;
    const int q = slot ^ ((L >> 1) & 3);
    const int r = 2 * L + (q >> 2), c = q & 3;
    const __bf16* g = G + (row0 + r) * ld + k0 + c * 8;
    char* dst = lds + (size_t)(i * THREADS + (tid & ~63)) * 16;
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)dst, 16, 0, 0);
  }
}

// s_waitcnt vmcnt(PER · n) for n in 0..3 (the count is an immediate)
template <int PER>
__device__ __forceinline__ void vmcnt_steps(int n) {
  if (n >= 3)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * PER) : "memory");
  else if (n == 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PER) : "memory");
  else if (n == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// a fragment read in inline asm: hipcc's own lgkmcnt for compiler-visible
// ds_reads is conservative at the loop head (it waited for the half-step
// loaded behind the one the MFMAs need); these are counted by hand
// (lgkm_wait + sched_barrier: the MFMAs are register-only and would be
// scheduled past a bare asm wait)
__device__ __forceinline__ bf16x8_t frag_ring(const char* t, int r, int c) {
  const int L = r >> 1;
  const int slot = (((r & 1) << 2) | c) ^ ((L >> 1) & 3);
  const __attribute__((address_space(3))) char* p =
      (const __attribute__((address_space(3))) char*)(t + L * 128 + slot * 16);
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
  return v;
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool OUT_BF16, int WM, int WN, bool PRIO>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_bf16_tn_ring_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, void* __restrict__ Cv, long M,
    long N, long K, float alpha, double* __restrict__ partials) {
  constexpr int THREADS = 64 * WM * WN;
  constexpr int TI = kBM / WM / 32, TJ = kBN / WN / 32;   // 32×32 tiles per wave
  constexpr int PER = 2 * (kTiler / 16 / THREADS);        // pieces per thread per K-step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long tiles_n = N / kBN;
  const uint32_t t = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const long bm = t / tiles_n, bn = t % tiles_n;
  const long m0 = bm * kBM, n0 = bn * kBN;
  const int nk = (int)(K / kBKr);

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < kRingr; ++s) {
    if (s < nk) {
      stage_ring<THREADS>(smem + s * kStager, A, K, m0, (long)s * kBKr, tid);
      stage_ring<THREADS>(smem + s * kStager + kTiler, Bt, K, n0, (long)s * kBKr, tid);
    }
  }
  const int fr = lane & 31;
  const int h = lane >> 5;
  const int ra = wm * (kBM / WM) + fr, rb = wn * (kBN / WN) + fr;

  bf16x8_t a0[TI], b0[TJ], a1[TI], b1[TJ];
  {
    vmcnt_steps<PER>(nk - 1 < 3 ? nk - 1 : 3);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < TI; ++i) a0[i] = frag_ring(smem, ra + i * 32, h);
#pragma unroll
    for (int j = 0; j < TJ; ++j) b0[j] = frag_ring(smem + kTiler, rb + j * 32, h);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const char* la = smem + (kt & (kRingr - 1)) * kStager;
#pragma unroll
    for (int i = 0; i < TI; ++i) a1[i] = frag_ring(la, ra + i * 32, 2 + h);
#pragma unroll
    for (int j = 0; j < TJ; ++j) b1[j] = frag_ring(la + kTiler, rb + j * 32, 2 + h);
    lgkm_wait<TI + TJ>();        // F0 landed (F1's reads may be in flight)
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < nk) {
      lgkm_wait<0>();
      vmcnt_steps<PER>(nk - 2 - kt < 2 ? nk - 2 - kt : 2);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + kRingr < nk) {
        char* nxt = smem + (kt & (kRingr - 1)) * kStager;
        stage_ring<THREADS>(nxt, A, K, m0, (long)(kt + kRingr) * kBKr, tid);
        stage_ring<THREADS>(nxt + kTiler, Bt, K, n0, (long)(kt + kRingr) * kBKr, tid);
      }
      const char* ln = smem + ((kt + 1) & (kRingr - 1)) * kStager;
#pragma unroll
      for (int i = 0; i < TI; ++i) a0[i] = frag_ring(ln, ra + i * 32, h);
#pragma unroll
      for (int j = 0; j < TJ; ++j) b0[j] = frag_ring(ln + kTiler, rb + j * 32, h);
    } else {
      lgkm_wait<0>();            // F1 landed (the branch above waited before its barrier)
    }
    __builtin_amdgcn_sched_barrier(0);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  double csum = 0.0;
  const long lane_off = (m0 + wm * (kBM / WM) + 4 * h) * N + n0 + wn * (kBN / WN) + fr;
#pragma unroll
  for (int i = 0; i < TI; ++i) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const long base = lane_off + (long)(i * 32) * N + j * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long off = base + (long)((r & 3) + 8 * (r >> 2)) * N;
        const float v = acc[i][j][r] * alpha;
        if (OUT_BF16) {
          const uint16_t hv = hbmr_f32_to_bf16(v);
          reinterpret_cast<uint16_t*>(Cv)[off] = hv;
          csum += (double)__uint_as_float((uint32_t)hv << 16);
        } else {
          reinterpret_cast<float*>(Cv)[off] = v;
          csum += (double)v;
        }
      }
    }
  }
  if (partials) {
    // (reuses the staging array: a second __shared__ object can make hipcc
    // wait vmcnt(0) before the loop's first ds_read)
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
    if (lane == 0) red[wave] = csum;
    __syncthreads();
    if (tid == 0) {
      double sum = 0.0;
#pragma unroll
      for (int w = 0; w < WM * WN; ++w) sum += red[w];
      partials[blockIdx.x] = sum;
    }
  }
}

template <bool OUT_BF16, int WM, int WN, bool PRIO>
int launch_ring(const void* A, const void* Bt, void* C, long M, long N, long K, float alpha,
                double* partials, long tiles, hipStream_t st) {
  static bool set = false;
  if (!set) {
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute(
        (const void*)gemm_bf16_tn_ring_kernel<OUT_BF16, WM, WN, PRIO>,
        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsr));
    set = true;
  }
  hipLaunchKernelGGL((gemm_bf16_tn_ring_kernel<OUT_BF16, WM, WN, PRIO>), dim3((unsigned)tiles),
                     dim3(64 * WM * WN), kLdsr, st, reinterpret_cast<const __bf16*>(A),
                     reinterpret_cast<const __bf16*>(Bt), C, M, N, K, alpha, partials);
  return (int)hipGetLastError();
}

template <bool OUT_BF16>
int launch_ring_ver(int ver, const void* A, const void* Bt, void* C, long M, long N, long K,
                    float alpha, double* partials, long tiles, hipStream_t st) {
  switch (ver) {
    case 3: return launch_ring<OUT_BF16, 2, 2, false>(A, Bt, C, M, N, K, alpha, partials, tiles, st);
    case 4: return launch_ring<OUT_BF16, 2, 2, true>(A, Bt, C, M, N, K, alpha, partials, tiles, st);
    case 5: return launch_ring<OUT_BF16, 2, 4, false>(A, Bt, C, M, N, K, alpha, partials, tiles, st);
    default: return launch_ring<OUT_BF16, 2, 4, true>(A, Bt, C, M, N, K, alpha, partials, tiles, st);
  }
}

bool g_gemm_lds_set = false;

}  // namespace

extern "C" {

// C = alpha · A · Btᵀ; out_bf16 selects a bf16 C (else fp32).  partials (may be
// null): ceil(M/256)·ceil(N/256) doubles, each workgroup's sum of its stored
// C tile.  Any M, N; K % 8 == 0.
int hbmr_gemm_bf16_tn_ex(const void* A, const void* Bt, void* C, long M, long N, long K,
                         float alpha, int out_bf16, double* partials, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  // 16-B pieces: K % 8 (and 16-B aligned operands); buffer offsets are 32-bit
  if (K % 8 || ((uintptr_t)A | (uintptr_t)Bt) % 16 || (long)kBM * K * 2 >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if (!g_gemm_lds_set) {
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute((const void*)gemm_bf16_tn_kernel<false>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds));
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute((const void*)gemm_bf16_tn_kernel<true>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds));
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute((const void*)gemm_bf16_tn_v2_kernel<false>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds));
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute((const void*)gemm_bf16_tn_v2_kernel<true>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds));
    g_gemm_lds_set = true;
  }
  const long tiles = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  if (tiles > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const bool ragged = M % kBM || N % kBN || K % kBK;
  // HBMR_GEMM=2: the 4-wave 128x128 / 32x32x16 double-buffered variant;
  // 3..6: the ring kernels (A/B against v1), read per call (a bench switches
  // between them in one process)
  const char* ev = getenv("HBMR_GEMM");
  const int ver = ev && *ev >= '2' && *ev <= '6' ? *ev - '0' : 1;
  if (ver >= 3 && !ragged && K % kBKr == 0)
    return out_bf16 ? launch_ring_ver<true>(ver, A, Bt, C, M, N, K, alpha, partials, tiles, st)
                    : launch_ring_ver<false>(ver, A, Bt, C, M, N, K, alpha, partials, tiles, st);
  if (ver == 2 && !ragged) {
    if (out_bf16)
      hipLaunchKernelGGL(gemm_bf16_tn_v2_kernel<true>, dim3((unsigned)tiles), dim3(kGemmThreads2),
                         kGemmLds, st, reinterpret_cast<const __bf16*>(A),
                         reinterpret_cast<const __bf16*>(Bt), C, M, N, K, alpha, partials);
    else
      hipLaunchKernelGGL(gemm_bf16_tn_v2_kernel<false>, dim3((unsigned)tiles),
                         dim3(kGemmThreads2), kGemmLds, st, reinterpret_cast<const __bf16*>(A),
                         reinterpret_cast<const __bf16*>(Bt), C, M, N, K, alpha, partials);
    return (int)hipGetLastError();
  }
  if (out_bf16)
    hipLaunchKernelGGL(gemm_bf16_tn_kernel<true>, dim3((unsigned)tiles), dim3(kGemmThreads),
                       kGemmLds, st, reinterpret_cast<const __bf16*>(A),
                       reinterpret_cast<const __bf16*>(Bt), C, M, N, K, alpha, partials);
  else
    hipLaunchKernelGGL(gemm_bf16_tn_kernel<false>, dim3((unsigned)tiles), dim3(kGemmThreads),
                       kGemmLds, st, reinterpret_cast<const __bf16*>(A),
                       reinterpret_cast<const __bf16*>(Bt), C, M, N, K, alpha, partials);
  return (int)hipGetLastError();
}

int hbmr_gemm_bf16_tn(const void* A, const void* Bt, void* C, long M, long N, long K, float alpha,
                      int out_bf16, hipStream_t st) {
  return hbmr_gemm_bf16_tn_ex(A, Bt, C, M, N, K, alpha, out_bf16, nullptr, st);
}

}  // extern "C"
