// K-Means map-side kernels for MI355X (gfx950).
//
// These are the GPU "map function + combiner" of a K-Means MapReduce
// iteration.  In the reference the GPU map task is an external Pipes binary
// launched per task (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/pipes/
// Application.java:162-181, PipesGPUMapRunner.java:66-118) and the combiner is
// the C++ CombineRunner (src/c++/pipes/impl/HadoopPipes.cc:660-705); there is no
// GPU code in the reference, so these kernels are designed from scratch
// (SURVEY.md §2.11 K1-K3).
//
//  kmeans_assign   : labels[i] = argmin_j ||x_i - c_j||^2 computed as an MFMA
//                    GEMM  S = C · Xᵀ  (v_mfma_f32_32x32x16_bf16, fp32 accum)
//                    with the centroid tiles staged in LDS by global_load_lds
//                    and a fused running-argmax epilogue on
//                    score = x·c - ||c||²/2 (the -||c||²/2 term is loaded as
//                    the MFMA's initial accumulator, so no subtraction).
//                    Points sit on the MFMA *column* (lane) axis so each
//                    lane's arg-max is register-local: no cross-lane
//                    reduction until the very end.
//  kmeans_accum_*  : per-cluster partial sums / counts (the combiner) with
//                    LDS-privatised accumulators; one global atomic flush per
//                    workgroup instead of one per point (global f32 atomics
//                    run at ≈1.3 TB/s chip-wide: MI355X_MICROARCH.md).
//  kmeans_update   : reduce side: c_j = sum_j / count_j, emits the bf16
//                    centroid image + -||c||²/2 for the next iteration.
#include "common.h"
#include "../include/hbmr/hbmr.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * HBMR_WAVE;
constexpr int kCK = 64;  // clusters per LDS chunk (two 32-row MFMA blocks)

// One 32x32x16 MFMA on 16-bit operands held as bf16x8 bit patterns: bf16, or
// fp16 (F16) — exact mode's default, whose 11 significant bits round the
// points and centroids 8x closer than bf16's 8 at the same matrix-core rate,
// so 8x fewer points fail the certification (kmeans_refine_*).
template <bool F16>
__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int D> struct AssignCfg {
  static constexpr int KS = D / 16;             // MFMA k-steps (K=16 each)
  static constexpr int CPR = D / 8;             // 16-byte pieces per row
  static constexpr int SWZ = CPR >= 16 ? 15 : CPR - 1;
  static constexpr int PB = D <= 128 ? 2 : 1;   // 32-point blocks per wave
  static constexpr int PTS = kWaves * PB * 32;  // points per workgroup
  static constexpr int CHUNK_BYTES = kCK * D * 2;
  static constexpr int BUF_BYTES = CHUNK_BYTES + kCK * 4;
  static constexpr int LDS_BYTES = 2 * BUF_BYTES;
};

// Stage centroid chunk `chunk` (kCK rows × D bf16) plus its -||c||²/2 values
// into LDS buffer `buf`.  The LDS image is lane-linear (global_load_lds writes
// base + lane*16) so the bank-conflict XOR swizzle is applied to the SOURCE
// address: LDS piece (row, p) holds global piece (row, p ^ (row & SWZ))
// (cdna_hip_programming.md §5.4 rule 21).
template <int D>
__device__ __forceinline__ void stage_chunk(char* buf, const __bf16* __restrict__ C,
                                            const float* __restrict__ chalf, int chunk,
                                            int wave, int lane) {
  using Cfg = AssignCfg<D>;
  constexpr int PIECES = kCK * Cfg::CPR;  // 16-B pieces in the chunk
  constexpr int ROUNDS = PIECES / kThreads;
  static_assert(PIECES % kThreads == 0, "chunk must tile the workgroup");
  const char* gbase = reinterpret_cast<const char*>(C) + (size_t)chunk * Cfg::CHUNK_BYTES;
#pragma unroll
  for (int i = 0; i < ROUNDS; ++i) {
    const int base = (i * kWaves + wave) * HBMR_WAVE;
    const int p = base + lane;
    const int row = p / Cfg::CPR;
    const int cpos = p % Cfg::CPR;
    const int src = cpos ^ (row & Cfg::SWZ);
    const char* g = gbase + row * (D * 2) + src * 16;
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)(buf + base * 16), 16, 0, 0);
  }
  if (wave == 0) {
    const float* g = chalf + (size_t)chunk * kCK + lane;
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)(buf + Cfg::CHUNK_BYTES), 4, 0, 0);
  }
}

__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Packed running arg-max of one lane over 32-row MFMA tiles (points on lanes,
// clusters on the 16 accumulator registers).  The low lb = 4 + log2(tiles)
// mantissa bits of every score are overwritten with a (tile, register) code,
// so the running maximum needs no index registers: per tile and 32-point block
// it costs 16 v_and_or_b32 + 8 v_max3_f32 into two partial maxima.  lb ≤ 12,
// i.e. ≤ 2^-12 relative perturbation — below the bf16 operand rounding (2^-8).
// v_max3_f32 goes through asm because __builtin_fmaxf canonicalises both
// operands in IEEE mode (an extra v_max_f32 x,x,x per input, which made the
// epilogue as long as the MFMA chain); the and_or stays compiler-visible so
// MFMA→VALU read hazards are still padded.
struct PackedArgMax {
  uint32_t vmask;  // VGPR copy of ~((1 << lb) - 1): VOP3 reads only one SGPR
  uint32_t top;    // (2^tb - 1) << 4
  float b0, b1;

  __device__ __forceinline__ void init(int ntiles) {
    int tb = 0;
    while ((1 << tb) < ntiles) ++tb;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmask) : "s"(~((1u << (tb + 4)) - 1u)));
    top = ((1u << tb) - 1u) << 4;
    b0 = b1 = -3.0e38f;
  }
  __device__ __forceinline__ void update(const f32x16& acc, int t) {
    const uint32_t base = top - ((uint32_t)t << 4);
    // per-register codes laundered into opaque SGPRs, else the or-constant is
    // folded into a v_and + v_or3 pair instead of one v_and_or_b32.  (The asm
    // is empty: a real s_or_b32 in it would clobber SCC under the loop branch.)
    uint32_t code[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      code[r] = base | (15u - r);
      asm("" : "+s"(code[r]));
    }
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const float u0 = __uint_as_float((__float_as_uint(acc[r + 0]) & vmask) | code[r + 0]);
      const float u1 = __uint_as_float((__float_as_uint(acc[r + 1]) & vmask) | code[r + 1]);
      const float u2 = __uint_as_float((__float_as_uint(acc[r + 2]) & vmask) | code[r + 2]);
      const float u3 = __uint_as_float((__float_as_uint(acc[r + 3]) & vmask) | code[r + 3]);
      b0 = vmax3(b0, u0, u1);
      b1 = vmax3(b1, u2, u3);
    }
  }
  // best packed score of this lane and its cluster (lane half h)
  __device__ __forceinline__ float best() const { return fmaxf(b0, b1); }
  __device__ __forceinline__ int cluster(float bv, int h) const {
    const uint32_t code = __float_as_uint(bv) & ~vmask;
    const int tile = (int)(top >> 4) - (int)(code >> 4);
    const int r = 15 - (int)(code & 15u);
    return tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
  }
  __device__ __forceinline__ float score(float bv) const {
    return __uint_as_float(__float_as_uint(bv) & vmask);
  }
};

__device__ __forceinline__ float vmed3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Packed running TOP-3 (exact mode, hbmr.kmeans.exact): same (tile, register)
// codes as PackedArgMax, but each of two register-parity tracks keeps its best
// three b >= s >= t.  Inserting u: t = med3(s, t, u), s = med3(b, s, u),
// b = max(b, u) (the middle of a sorted pair and u is the new lower member) —
// 3 VALU ops per score instead of 0.5, two independent chains per 32 points.
struct PackedTop3 : PackedArgMax {
  float s0, s1, t0, t1;
  __device__ __forceinline__ void init(int ntiles) {
    PackedArgMax::init(ntiles);
    s0 = s1 = t0 = t1 = -3.0e38f;
  }
  __device__ __forceinline__ static void insert(float& b, float& s, float& t, float u) {
    t = vmed3(s, t, u);
    s = vmed3(b, s, u);
    b = vmax3(b, u, u);
  }
  __device__ __forceinline__ void update(const f32x16& acc, int tt) {
    const uint32_t base = top - ((uint32_t)tt << 4);
    uint32_t code[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      code[r] = base | (15u - r);
      asm("" : "+s"(code[r]));
    }
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const float u0 = __uint_as_float((__float_as_uint(acc[r + 0]) & vmask) | code[r + 0]);
      const float u1 = __uint_as_float((__float_as_uint(acc[r + 1]) & vmask) | code[r + 1]);
      insert(b0, s0, t0, u0);
      insert(b1, s1, t1, u1);
    }
  }
  __device__ __forceinline__ void top3(float& b, float& s, float& t) const {
    b = b0; s = s0; t = t0;
    insert(b, s, t, b1);
    insert(b, s, t, s1);
    insert(b, s, t, t1);
  }
};

// Packed running TOP-2 per TRACK (exact mode default): the 16 accumulator
// registers of a lane form 8 tracks (register r -> track r & 7), each keeping
// its best two: s = med3(b, s, u), b = max(b, u) — 2 VALU ops per score (+ the
// and_or that packs the code) instead of PackedTop3's 3.  With K = 128 one
// 32x32 output tile is 8 MFMAs (256 MFMA cycles per SIMD, 64 of them blocking
// vector issue): the top-3 epilogue's 4 issue slots per score did not fit the
// remaining 192 cycles (top-3 assign ran 20 % behind the plain arg-max), 3 do.
// Together with the lane half h, a cluster's track is its index bits 0-2 (4
// tracks, r & 3) or 0-3 (8 tracks, r & 7): cluster = tile*32 + (r&3) +
// 8(r>>2) + 4h.  The top 3 of a point are the
// top 3 of the 32 track candidates; every cluster that is not a candidate
// scores <= its track's second, which is <= the third — unless the best and
// the second share a track, which finish_point flags (t = b, margin 0: step 2
// of the certification then defers the point to the neighbour scan).
// workgroups per CU the exact (top-3) assign kernels are built for: 3 keeps
// them at <= 168 VGPRs, i.e. 3 waves per SIMD like the plain arg-max kernel
#ifndef HBMR_EXACT_MINB
#define HBMR_EXACT_MINB 3
#endif
#ifndef HBMR_EXACT_TRACKS
#define HBMR_EXACT_TRACKS 4   // register tracks per lane (4: r & 3; 8: r & 7)
#endif
#ifndef HBMR_EXACT_PAIRINS
#define HBMR_EXACT_PAIRINS 1  // insert a track's two scores of a tile at once
#endif
struct PackedTop2x8 : PackedArgMax {
  static constexpr int NT = HBMR_EXACT_TRACKS;
  static constexpr uint32_t TMASK = NT == 8 ? 15u : 7u;   // cluster bits of a track
  float tb[NT], ts[NT];
  __device__ __forceinline__ void init(int ntiles) {
    PackedArgMax::init(ntiles);
#pragma unroll
    for (int i = 0; i < NT; ++i) tb[i] = ts[i] = -3.0e38f;
  }
  __device__ __forceinline__ void update(const f32x16& acc, int tt) {
    const uint32_t base = top - ((uint32_t)tt << 4);
    uint32_t code[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      code[r] = base | (15u - r);
      asm("" : "+s"(code[r]));
    }
#if HBMR_EXACT_PAIRINS
    // registers r and r + NT belong to one track: both are inserted at once —
    // the second of {b >= s, u, v} is max(med3(b, u, v), s) — 3 VALU ops per
    // two scores instead of 4 (the epilogue is what bounds this kernel)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if ((r / NT) % 2) continue;
      const float u = __uint_as_float((__float_as_uint(acc[r]) & vmask) | code[r]);
      const float v = __uint_as_float((__float_as_uint(acc[r + NT]) & vmask) | code[r + NT]);
      const float m = vmed3(tb[r % NT], u, v);
      ts[r % NT] = vmax3(m, ts[r % NT], ts[r % NT]);
      tb[r % NT] = vmax3(tb[r % NT], u, v);
    }
#else
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float u = __uint_as_float((__float_as_uint(acc[r]) & vmask) | code[r]);
      ts[r % NT] = vmed3(tb[r % NT], ts[r % NT], u);
      tb[r % NT] = vmax3(tb[r % NT], u, u);
    }
#endif
  }
  __device__ __forceinline__ void top3(float& b, float& s, float& t) const {
    b = s = t = -3.0e38f;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      PackedTop3::insert(b, s, t, tb[i]);
      PackedTop3::insert(b, s, t, ts[i]);
    }
  }
  static constexpr bool kTracks = true;
};

template <class AM, class = void> struct HasTracks { static constexpr bool value = false; };
template <class AM> struct HasTracks<AM, std::void_t<decltype(AM::kTracks)>> {
  static constexpr bool value = AM::kTracks;
};

#ifndef HBMR_EXACT_TOP3
#define HBMR_EXACT_TOP3 0   // 1: the full running top-3 (PackedTop3)
#endif
template <bool EXACT>
using ArgMaxT = typename std::conditional<
    EXACT, typename std::conditional<HBMR_EXACT_TOP3 != 0, PackedTop3, PackedTop2x8>::type,
    PackedArgMax>::type;

// (score, cluster) insertion into a sorted triple; ties to the lower cluster
__device__ __forceinline__ void insert3(float (&v)[3], int (&c)[3], float u, int cu) {
  auto gt = [](float a, int ca, float b, int cb) { return a > b || (a == b && ca < cb); };
  if (gt(u, cu, v[2], c[2])) {
    v[2] = u; c[2] = cu;
    if (gt(v[2], c[2], v[1], c[1])) {
      float tv = v[1]; v[1] = v[2]; v[2] = tv;
      int tc = c[1]; c[1] = c[2]; c[2] = tc;
      if (gt(v[1], c[1], v[0], c[0])) {
        tv = v[0]; v[0] = v[1]; v[1] = tv;
        tc = c[0]; c[0] = c[1]; c[1] = tc;
      }
    }
  }
}

// Finish one point: lane-local arg-max (exact mode: top 3), then across the
// two lane halves (each half saw a different set of cluster rows).  Exact mode
// writes the runner-ups cand[p], cand[n+p] and the score margins best-second,
// best-third (masked scores) to margin[p], margin[n+p].
template <bool EXACT, class AM>
__device__ __forceinline__ void finish_point(const AM& am, int h, long p, long n,
                                             int32_t* __restrict__ labels,
                                             int32_t* __restrict__ cand,
                                             float* __restrict__ scores,
                                             float* __restrict__ margin,
                                             uint32_t* __restrict__ hist, long cs = -1) {
  // cs: stride of the second candidate / margin (n for one split; the batch
  // size when a grouped launch writes a batch's arrays)
  if (cs < 0) cs = n;
  if constexpr (!EXACT) {
    float bv = am.best();
    int cluster = am.cluster(bv, h);
    const float ov = __shfl_xor(bv, 32);
    const int oc = __shfl_xor(cluster, 32);
    if (ov > bv || (ov == bv && oc < cluster)) { bv = ov; cluster = oc; }
    if (h == 0 && p < n) {
      labels[p] = cluster;
      if (scores) scores[p] = am.score(bv);
      if (hist) atomicAdd(hist + cluster, 1u);  // fused histogram for the sorted combiner
    }
  } else {
    float v[3];
    int c[3];
    am.top3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = am.cluster(v[i], h);
    float ov[3];
    int oc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ov[i] = __shfl_xor(v[i], 32);
      oc[i] = __shfl_xor(c[i], 32);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) insert3(v, c, ov[i], oc[i]);
    if constexpr (HasTracks<AM>::value) {
      // best and second in one track: the rest is bounded only by the second
      if (((c[0] ^ c[1]) & AM::TMASK) == 0) {
        v[2] = v[0];
        c[2] = c[0];
      }
    }
    if (h == 0 && p < n) {
      labels[p] = c[0];
      cand[p] = c[1];
      cand[cs + p] = c[2];
      const float bs = am.score(v[0]);
      scores[p] = bs;
      margin[p] = bs - am.score(v[1]);
      margin[cs + p] = bs - am.score(v[2]);
      if (hist) atomicAdd(hist + c[0], 1u);
    }
  }
}

// One workgroup's tile of points [blk*PTS, (blk+1)*PTS) of one split.
template <int D, bool EXACT = false, bool F16 = false>
__device__ __forceinline__ void assign_tile(const __bf16* __restrict__ X, long n,
                                            const __bf16* __restrict__ C,
                                            const float* __restrict__ chalf, int nchunks,
                                            int32_t* __restrict__ labels,
                                            float* __restrict__ scores,
                                            uint32_t* __restrict__ hist, long blk, char* smem,
                                            int32_t* __restrict__ cand = nullptr,
                                            float* __restrict__ margin = nullptr) {
  using Cfg = AssignCfg<D>;
  constexpr int KS = Cfg::KS, PB = Cfg::PB;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / HBMR_WAVE);
  const int lane = tid & (HBMR_WAVE - 1);
  const int h = lane >> 5;   // lane half: selects k-offset 8h in A/B fragments
  const int col = lane & 31;
  const long p0 = blk * Cfg::PTS + (long)wave * PB * 32;

  // Kick off chunk 0 first so it overlaps the point-fragment loads.
  stage_chunk<D>(smem, C, chalf, 0, wave, lane);

  // B operand = points: lane holds X[p][16s + 8h .. +7] for its column p.
  bf16x8 bfrag[PB][KS];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    long p = p0 + pb * 32 + col;
    if (p >= n) p = n - 1;
    const uint4* row = reinterpret_cast<const uint4*>(X + p * D);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint4 v = row[2 * s + h];
      bfrag[pb][s] = __builtin_bit_cast(bf16x8, v);
    }
  }

  ArgMaxT<EXACT> am[PB];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) am[pb].init(nchunks * (kCK / 32));

  // Retire the fragment loads here and launder the registers through an asm
  // so hipcc's waitcnt pass does not see them as pending inside the chunk loop
  // (it would otherwise emit vmcnt(0) at the first MFMA and drain the next
  // chunk's global_load_lds prefetch every iteration).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int pb = 0; pb < PB; ++pb)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(bfrag[pb][s]));
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    char* cur = smem + (c & 1) * Cfg::BUF_BYTES;
    if (c + 1 < nchunks)
      stage_chunk<D>(smem + ((c + 1) & 1) * Cfg::BUF_BYTES, C, chalf, c + 1, wave, lane);
    const float* ch = reinterpret_cast<const float*>(cur + Cfg::CHUNK_BYTES);
#pragma unroll
    for (int cb = 0; cb < kCK / 32; ++cb) {
      f32x16 acc[PB];
      // Initial accumulator = -||c||²/2 of the cluster on this register's row:
      // row(reg, lane) = (reg & 3) + 8 * (reg >> 2) + 4 * h.
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(ch + cb * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
          acc[pb][4 * g + 0] = v[0];
          acc[pb][4 * g + 1] = v[1];
          acc[pb][4 * g + 2] = v[2];
          acc[pb][4 * g + 3] = v[3];
        }
      }
      const int arow = cb * 32 + col;
      const char* abase = cur + arow * (D * 2);
      const int aswz = arow & Cfg::SWZ;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int q = 2 * s + h;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abase + ((q ^ aswz) << 4));
#pragma unroll
        for (int pb = 0; pb < PB; ++pb)
          acc[pb] = mfma32x32x16<F16>(a, bfrag[pb][s], acc[pb]);
      }
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) am[pb].update(acc[pb], c * (kCK / 32) + cb);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

#pragma unroll
  for (int pb = 0; pb < PB; ++pb)
    finish_point<EXACT>(am[pb], h, p0 + pb * 32 + col, n, labels, cand, scores, margin, hist);
}

// ---------------------------------------------------------------------------
// v2: software-pipelined variant for D ≤ 128 (PB = 2).
// The centroid stream advances in 32-cluster tiles through an NS-deep LDS
// ring; the A fragments (and -|c|²/2) of tile t+1 are read into registers
// while tile t's 16 MFMAs run, so the MFMA chain never waits on an LDS read,
// and there is ONE barrier per tile:
//   wait own DMA(t+1) + lgkmcnt(0) → barrier → DMA(t+NS) into tile t's slot
//   (its LDS→register reads retired by the lgkmcnt) → ds_read tile t+1 →
//   MFMAs + arg-max epilogue of tile t.
// A DMA thus has NS-1 tiles (≈(NS-1)·512 MFMA cycles) to land: with NS = 2 the
// L2 latency under full-chip load was exposed every tile.
template <int D, int NSV = 4> struct AssignV2 {
  static constexpr int KS = D / 16;
  static constexpr int NS = NSV;                         // ring depth
  static constexpr int TILE_BYTES = 32 * D * 2;          // 32 clusters
  static constexpr int BUF = TILE_BYTES + 32 * 4;        // + -|c|²/2
  static constexpr int LDS_BYTES = NS * BUF;
  static constexpr int PIECES = 32 * (D / 8);            // 16-B pieces per tile
  // waves per workgroup sharing one centroid stream; 8 (2 per SIMD, half the
  // L2→LDS traffic per FLOP) measured 16–19 % slower than 4 at 100M×1024×128
  // (profiles/kmeans_assign_tuning.md); HBMR_KMEANS_V2_WAVES picks at build time
#ifndef HBMR_KMEANS_V2_WAVES
#define HBMR_KMEANS_V2_WAVES 4
#endif
  static constexpr int WAVES = PIECES >= HBMR_KMEANS_V2_WAVES * HBMR_WAVE ? HBMR_KMEANS_V2_WAVES : 4;
  static constexpr int THREADS = WAVES * HBMR_WAVE;
  static constexpr int MINB = WAVES == 8 ? 1 : 2;        // → ≤ 256 VGPRs either way
  static constexpr int P = PIECES / THREADS;             // DMAs per lane per tile
};

template <int N> __device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most `y` tile-DMAs of this wave are outstanding (wave 0 issues
// one extra DMA per tile for -|c|²/2).  y is wave-uniform, ≤ Y.
template <int P, int Y>
__device__ __forceinline__ void wait_tile_dmas(int y, bool w0) {
  if constexpr (Y > 0) {
    if (y == Y) {
      if (w0) vm_wait<Y * (P + 1)>(); else vm_wait<Y * P>();
      return;
    }
    wait_tile_dmas<P, Y - 1>(y, w0);
  } else {
    vm_wait<0>();
  }
}

template <int D>
__device__ __forceinline__ void stage_tile32(char* buf, const __bf16* __restrict__ C,
                                             const float* __restrict__ chalf, int tile, int wave,
                                             int lane) {
  using V = AssignV2<D>;
  constexpr int CPR = D / 8;
  constexpr int SWZ = AssignCfg<D>::SWZ;
  const char* gbase = reinterpret_cast<const char*>(C) + (size_t)tile * V::TILE_BYTES;
#pragma unroll
  for (int i = 0; i < V::P; ++i) {
    const int base = (i * V::WAVES + wave) * HBMR_WAVE;
    const int p = base + lane;
    const int row = p / CPR, cpos = p % CPR;
    const char* g = gbase + row * (D * 2) + ((cpos ^ (row & SWZ)) * 16);
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)(buf + base * 16), 16, 0, 0);
  }
  if (wave == 0 && lane < 32) {
    const float* g = chalf + (size_t)tile * 32 + lane;
    __builtin_amdgcn_global_load_lds((const void*)g, (void*)(buf + V::TILE_BYTES), 4, 0, 0);
  }
}

template <int D>
__device__ __forceinline__ void read_tile32(const char* buf, int col, int h, bf16x8 (&a)[D / 16],
                                            f32x16& bias) {
  constexpr int SWZ = AssignCfg<D>::SWZ;
  const char* abase = buf + col * (D * 2);
  const int aswz = col & SWZ;
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    a[s] = *reinterpret_cast<const bf16x8*>(abase + (((2 * s + h) ^ aswz) << 4));
  const float* ch = reinterpret_cast<const float*>(buf + AssignV2<D>::TILE_BYTES);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(ch + 8 * g + 4 * h);
    bias[4 * g + 0] = v[0];
    bias[4 * g + 1] = v[1];
    bias[4 * g + 2] = v[2];
    bias[4 * g + 3] = v[3];
  }
}

struct NoFin {};   // assign_tile_v2's default finish (finish_point)

// the fused exact kernel: 3 = v3 (default), 2 = v2 (HBMR_EXACT_V3=v2, read once;
// hbmr_kmeans_set_exact_kernel overrides it in-process)
int g_exact_kernel = -1;
inline int exact_kernel() {
  static const int env = [] {
    const char* e = getenv("HBMR_EXACT_V3");
    return e && strcmp(e, "v2") == 0 ? 2 : 3;
  }();
  return g_exact_kernel > 0 ? g_exact_kernel : env;
}

template <int D, int PB, bool EXACT = false, bool F16 = false, bool TOP3 = false,
          class Fin = NoFin>
__device__ __forceinline__ void assign_tile_v2(const __bf16* __restrict__ X, long n,
                                               const __bf16* __restrict__ C,
                                               const float* __restrict__ chalf, int ntiles,
                                               int32_t* __restrict__ labels,
                                               float* __restrict__ scores, long blk, char* smem,
                                               int32_t* __restrict__ cand = nullptr,
                                               float* __restrict__ margin = nullptr,
                                               long cs = -1, const Fin* fin = nullptr) {
  static_assert(D <= 128, "v2 keeps PB point blocks of D ≤ 128 in registers");
  using V = AssignV2<D>;
  constexpr int KS = V::KS;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / HBMR_WAVE);
  const int lane = tid & (HBMR_WAVE - 1);
  const int h = lane >> 5;
  const int col = lane & 31;
  const long p0 = blk * (V::WAVES * PB * 32) + (long)wave * PB * 32;

#pragma unroll
  for (int i = 0; i < V::NS; ++i)
    if (i < ntiles) stage_tile32<D>(smem + i * V::BUF, C, chalf, i, wave, lane);

  bf16x8 bfrag[PB][KS];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    long p = p0 + pb * 32 + col;
    if (p >= n) p = n - 1;
    const uint4* row = reinterpret_cast<const uint4*>(X + p * D);
#pragma unroll
    for (int s = 0; s < KS; ++s) bfrag[pb][s] = __builtin_bit_cast(bf16x8, row[2 * s + h]);
  }
  typename std::conditional<EXACT, typename std::conditional<TOP3, PackedTop3, PackedTop2x8>::type,
                            PackedArgMax>::type am[PB];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) am[pb].init(ntiles);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int pb = 0; pb < PB; ++pb)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(bfrag[pb][s]));
  __syncthreads();

  // Rolling register prefetch: right after the two MFMAs that consume k-step s
  // of tile t, fragment s of tile t+1 is read into the same registers, so each
  // LDS read has the rest of the tile's MFMAs to land and only one register
  // set of A (and of -|c|²/2) is live.
  bf16x8 a[KS];
  f32x16 bias;
  read_tile32<D>(smem, col, h, a, bias);
  constexpr int SWZ = AssignCfg<D>::SWZ;
  const int aswz = col & SWZ;

  const bool w0 = wave == 0;
  int slot = 0;  // t % NS
  for (int t = 0; t < ntiles; ++t) {
    // tile t+1's DMA has landed for every wave (younger DMAs in flight: tiles
    // t+2 .. min(t+NS-1, ntiles-1)), and this wave's reads of tile t have
    // retired → tile t's slot is free
    wait_tile_dmas<V::P, V::NS - 2>(max(0, min(V::NS - 2, ntiles - 2 - t)), w0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + V::NS < ntiles) stage_tile32<D>(smem + slot * V::BUF, C, chalf, t + V::NS, wave, lane);
    slot = slot + 1 == V::NS ? 0 : slot + 1;
    // (past the last tile the reads hit a stale slot: harmless and branch-free)
    const char* nbuf = smem + slot * V::BUF;
    const char* nrow = nbuf + col * (D * 2);
    f32x16 acc[PB];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int pb = 0; pb < PB; ++pb)
        acc[pb] = mfma32x32x16<F16>(a[s], bfrag[pb][s], s == 0 ? bias : acc[pb]);
      a[s] = *reinterpret_cast<const bf16x8*>(nrow + (((2 * s + h) ^ aswz) << 4));
    }
    {
      const float* ch = reinterpret_cast<const float*>(nbuf + V::TILE_BYTES);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(ch + 8 * g + 4 * h);
        bias[4 * g + 0] = v[0];
        bias[4 * g + 1] = v[1];
        bias[4 * g + 2] = v[2];
        bias[4 * g + 3] = v[3];
      }
    }
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) am[pb].update(acc[pb], t);
  }

  if constexpr (!std::is_same<Fin, NoFin>::value) {
    (*fin)(am, h, p0, col, n, labels);        // e.g. the fused step-1 certification
  } else {
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
      finish_point<EXACT>(am[pb], h, p0 + pb * 32 + col, n, labels, cand, scores, margin,
                          nullptr, cs);
  }
}

template <int D>
__global__ __launch_bounds__(kThreads, 2) void kmeans_assign_kernel(
    const __bf16* __restrict__ X, long n, const __bf16* __restrict__ C,
    const float* __restrict__ chalf, int nchunks, int32_t* __restrict__ labels,
    float* __restrict__ scores) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  assign_tile<D>(X, n, C, chalf, nchunks, labels, scores, nullptr,
                 hbmr_xcd_remap(blockIdx.x, gridDim.x), smem);
}

template <int D, int PB>
__global__ __launch_bounds__(AssignV2<D>::THREADS, AssignV2<D>::MINB) void kmeans_assign_v2_kernel(
    const __bf16* __restrict__ X, long n, const __bf16* __restrict__ C,
    const float* __restrict__ chalf, int ntiles, int32_t* __restrict__ labels,
    float* __restrict__ scores) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  assign_tile_v2<D, PB>(X, n, C, chalf, ntiles, labels, scores,
                    hbmr_xcd_remap(blockIdx.x, gridDim.x), smem);
}

// Exact mode: the same kernels with the top-3 epilogue (bf16 or fp16 operands;
// the 16-bit rows travel as bf16 bit patterns either way).
template <int D, bool F16>
__global__ __launch_bounds__(kThreads, 2) void kmeans_assign_top3_kernel(
    const __bf16* __restrict__ X, long n, const __bf16* __restrict__ C,
    const float* __restrict__ chalf, int nchunks, int32_t* __restrict__ labels,
    int32_t* __restrict__ cand, float* __restrict__ scores, float* __restrict__ margin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  assign_tile<D, true, F16>(X, n, C, chalf, nchunks, labels, scores, nullptr,
                            hbmr_xcd_remap(blockIdx.x, gridDim.x), smem, cand, margin);
}

template <int D, int PB, bool F16, bool TOP3 = false>
__global__ __launch_bounds__(AssignV2<D>::THREADS, HBMR_EXACT_MINB) void kmeans_assign_top3_v2_kernel(
    const __bf16* __restrict__ X, long n, const __bf16* __restrict__ C,
    const float* __restrict__ chalf, int ntiles, int32_t* __restrict__ labels,
    int32_t* __restrict__ cand, float* __restrict__ scores, float* __restrict__ margin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  assign_tile_v2<D, PB, true, F16, TOP3>(X, n, C, chalf, ntiles, labels, scores,
                                         hbmr_xcd_remap(blockIdx.x, gridDim.x), smem, cand,
                                         margin);
}

// 1 = the chunked kernel above, 2 = the pipelined v2 (D ≤ 128); HBMR_KMEANS_ASSIGN
inline int assign_version(int D) {
  static const int v = [] {
    const char* e = getenv("HBMR_KMEANS_ASSIGN");
    return e && e[0] == '1' ? 1 : 2;
  }();
  return D <= 128 ? v : 1;
}

// v2 point blocks (32 points) per wave: 2 or 3; HBMR_KMEANS_PB
inline int v2_pb() {
  static const int pb = [] {
    const char* e = getenv("HBMR_KMEANS_PB");
    return e && e[0] == '3' ? 3 : 2;
  }();
  return pb;
}

// points per workgroup of the assign kernel launch_*assign picks
template <int D> int assign_pts(bool hist) {
  if constexpr (D <= 128)
    if (assign_version(D) == 2 && !hist) return AssignV2<D>::WAVES * v2_pb() * 32;
  return AssignCfg<D>::PTS;
}

// ---------------------------------------------------------------------------
// Grouped (batched) map kernels: one launch covers every split of a batch of
// map tasks.  Each workgroup finds its split in a small table passed by value.
constexpr int kMaxGroup = 64;

struct SplitTable {
  int nsplit;
  int k;
  const __bf16* X[kMaxGroup];
  long n[kMaxGroup];
  long off[kMaxGroup];        // offset of the split's points in the batch arrays
  long blk[kMaxGroup + 1];    // prefix sum of workgroups per split (per kernel)
};

__device__ __forceinline__ int find_split(const SplitTable& t, long b) {
  int lo = 0, hi = t.nsplit;  // t.blk[lo] <= b < t.blk[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (t.blk[mid] <= b) lo = mid; else hi = mid;
  }
  return lo;
}

template <int D>
__global__ __launch_bounds__(kThreads, 2) void kmeans_assign_grouped_kernel(
    const SplitTable tbl, const __bf16* __restrict__ C, const float* __restrict__ chalf,
    int nchunks, int32_t* __restrict__ labels, uint32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long b = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, b));
  assign_tile<D>(tbl.X[s], tbl.n[s], C, chalf, nchunks, labels + tbl.off[s], nullptr,
                 hist + (size_t)s * tbl.k, b - tbl.blk[s], smem);
}

template <int D, int PB>
__global__ __launch_bounds__(AssignV2<D>::THREADS, AssignV2<D>::MINB) void kmeans_assign_grouped_v2_kernel(
    const SplitTable tbl, const __bf16* __restrict__ C, const float* __restrict__ chalf,
    int ntiles, int32_t* __restrict__ labels) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long b = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, b));
  assign_tile_v2<D, PB>(tbl.X[s], tbl.n[s], C, chalf, ntiles, labels + tbl.off[s], nullptr,
                    b - tbl.blk[s], smem);
}

// Exact mode over a batch of splits in ONE launch (a per-split launch of the
// top-3 assign ran at 57 % MFMA busy against 67 % for a long dispatch): the
// batch's labels / scores and the two-row cand / margin arrays are indexed by
// the batch position (split offset + row), second rows at stride tbl.off[nsplit]
template <int D, int PB, bool F16, bool TOP3>
__global__ __launch_bounds__(AssignV2<D>::THREADS, HBMR_EXACT_MINB) void
kmeans_assign_top3_grouped_v2_kernel(const SplitTable tbl, const __bf16* __restrict__ C,
                                     const float* __restrict__ chalf, int ntiles,
                                     int32_t* __restrict__ labels, int32_t* __restrict__ cand,
                                     float* __restrict__ scores, float* __restrict__ margin,
                                     long total) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long b = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, b));
  const long o = tbl.off[s];
  assign_tile_v2<D, PB, true, F16, TOP3>(tbl.X[s], tbl.n[s], C, chalf, ntiles, labels + o,
                                         scores + o, b - tbl.blk[s], smem, cand + o, margin + o,
                                         total);
}

// ---------------------------------------------------------------------------
// Combiner: per-cluster sums and counts, LDS-privatised, in 64-bit FIXED POINT.
//
// gfx950 executes ds_add_f32 at ~0.4 lane-ops/clk/CU versus ~14.5 for
// ds_add_u32 (tools/ubench_lds_atomics.hip, profiles/lds_atomics.txt), so the
// partial sums are accumulated as int64 = round(x · 2^shift) with integer LDS
// atomics (ds_add_u64) and flushed with integer global atomics.  Integer sums
// are associative: the combiner output is bitwise identical for any task
// placement, kernel schedule or GPU count (and stays exact through the RCCL
// all-reduce).  bf16 inputs are exact in fixed point whenever |x| ≥ 2^(shift-31)
// ... i.e. every bf16 with ulp ≥ 2^-shift (shift = 24: |x| ≥ 2^-17).
//
// LDS image of the sums: element (row r, dim i) at r*RS + i + (i >> 3) (u64
// units).  A point is handled by D/8 lanes, lane `sub` owning dims
// [8 sub, 8 sub + 8) (one 16-B global load); at step j the 16 lanes of a point
// touch dwords 2(9 sub + j) + {0,1}: all 32 banks exactly once.
typedef unsigned long long u64;

template <int D> struct AccCfg {
  static constexpr int RS = D + D / 8 + 1;  // padded row stride (u64 elements)
  static constexpr int TPP = D / 8;         // lanes per point
};

// Eight consecutive features of one row, as loaded by one lane: bf16 rows
// (the normal path, one 16-B load) or fp32 rows (exact mode, two 16-B loads).
// `ld` is the padded row length in elements.
template <typename T> struct Row8;
template <> struct Row8<__bf16> {
  uint4 v;
  __device__ __forceinline__ void load(const __bf16* X, size_t row, int ld, int sub) {
    v = reinterpret_cast<const uint4*>(X + row * ld)[sub];
  }
  __device__ __forceinline__ void unpack(float f[8]) const { hbmr_unpack8(v, f); }
};
template <> struct Row8<float> {
  uint4 a, b;
  __device__ __forceinline__ void load(const float* X, size_t row, int ld, int sub) {
    const uint4* r = reinterpret_cast<const uint4*>(X + row * ld) + 2 * sub;
    a = r[0];
    b = r[1];
  }
  __device__ __forceinline__ void unpack(float f[8]) const {
    f[0] = __uint_as_float(a.x); f[1] = __uint_as_float(a.y);
    f[2] = __uint_as_float(a.z); f[3] = __uint_as_float(a.w);
    f[4] = __uint_as_float(b.x); f[5] = __uint_as_float(b.y);
    f[6] = __uint_as_float(b.z); f[7] = __uint_as_float(b.w);
  }
};

template <int D, typename T>
__device__ __forceinline__ void lds_add_row(u64* s_rows, int r, int sub, const Row8<T>& v,
                                            float scale) {
  float f[8];
  v.unpack(f);
  u64* dst = s_rows + r * AccCfg<D>::RS + sub * 9;
  long long q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hbmr_fx_accum8(f, scale, q);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (q[j]) atomicAdd(dst + j, (u64)q[j]);
}

template <int D>
__device__ __forceinline__ void flush_rows(const u64* s_rows, const uint32_t* s_cnt, int c0, int cc,
                                           long long* __restrict__ sums,
                                           long long* __restrict__ counts, int tid, int nt) {
  for (int e = tid; e < cc * D; e += nt) {
    const int r = e / D, i = e % D;
    const u64 v = s_rows[r * AccCfg<D>::RS + i + (i >> 3)];
    if (v) atomicAdd(reinterpret_cast<u64*>(sums) + (size_t)(c0 + r) * D + i, v);
  }
  for (int r = tid; r < cc; r += nt) {
    const uint32_t v = s_cnt[r];
    if (v) atomicAdd(reinterpret_cast<u64*>(counts) + c0 + r, (u64)v);
  }
}

// Small k: every workgroup holds all k rows in LDS; grid-stride over points.
// Each lane group keeps U rows (and labels) in flight before its LDS adds.
template <typename T, int D, int U>
__global__ __launch_bounds__(256) void kmeans_accum_lds_kernel(
    const T* __restrict__ X, long n, const int32_t* __restrict__ labels, int k,
    long long* __restrict__ sums, long long* __restrict__ counts, float scale) {
  using A = AccCfg<D>;
  extern __shared__ __attribute__((aligned(16))) u64 s_acc[];  // k*RS sums, then k counts
  const int tid = threadIdx.x;
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_acc + k * A::RS);
  for (int i = tid; i < k * A::RS; i += 256) s_acc[i] = 0ull;
  for (int i = tid; i < k; i += 256) s_cnt[i] = 0u;
  __syncthreads();
  constexpr int PPI = 256 / A::TPP;  // point slots per workgroup
  const int sub = tid % A::TPP;
  const int pi = tid / A::TPP;
  const long stride = (long)gridDim.x * PPI;
  long p = (long)blockIdx.x * PPI + pi;
  for (; p + (U - 1) * stride < n; p += U * stride) {
    int lab[U];
    Row8<T> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lab[u] = labels[p + u * stride];
      v[u].load(X, p + u * stride, D, sub);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lds_add_row<D>(s_acc, lab[u], sub, v[u], scale);
      if (sub == 0) atomicAdd(s_cnt + lab[u], 1u);
    }
  }
  for (; p < n; p += stride) {
    const int l0 = labels[p];
    Row8<T> v0;
    v0.load(X, p, D, sub);
    lds_add_row<D>(s_acc, l0, sub, v0, scale);
    if (sub == 0) atomicAdd(s_cnt + l0, 1u);
  }
  __syncthreads();
  flush_rows<D>(s_acc, s_cnt, 0, k, sums, counts, tid, 256);
}

// Large k: grid.y walks cluster chunks of CC clusters.  Each wave scans 256
// labels per step (one int4 per lane), compacts the points whose label falls in
// this workgroup's chunk into a wave-private LDS queue (ballot + prefix count),
// then drains the queue with U rows in flight per lane group.  Every row is
// gathered exactly once over the whole grid; labels are re-read per chunk
// (from L2 / Infinity Cache when the split is small, as map splits are).
constexpr int kAccWaves = 8;
constexpr int kQueue = 256;  // queue entries per wave (one step's worth)

template <typename T, int D, int U>
__global__ __launch_bounds__(512) void kmeans_accum_chunked_kernel(
    const T* __restrict__ X, long n, const int32_t* __restrict__ labels, int k, int CC,
    long pts_per_block, long long* __restrict__ sums, long long* __restrict__ counts,
    float scale) {
  using A = AccCfg<D>;
  extern __shared__ __attribute__((aligned(16))) u64 s_acc[];
  // layout: CC*RS u64 sums | kAccWaves*kQueue u32 queue | CC u32 counts
  constexpr int NT = kAccWaves * HBMR_WAVE;
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * CC;
  const int cc = min(CC, k - c0);
  for (int i = tid; i < CC * A::RS; i += NT) s_acc[i] = 0ull;
  uint32_t* s_q = reinterpret_cast<uint32_t*>(s_acc + CC * A::RS);
  uint32_t* s_cnt = s_q + kAccWaves * kQueue;
  for (int i = tid; i < CC; i += NT) s_cnt[i] = 0u;
  __syncthreads();
  const int wave = tid / HBMR_WAVE, lane = tid & 63;
  uint32_t* q = s_q + wave * kQueue;
  constexpr int GPW = HBMR_WAVE / A::TPP;  // points per wave-instruction
  const int grp = lane / A::TPP, sub = lane % A::TPP;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  const long pb = (long)blockIdx.x * pts_per_block;
  const long pe = min(n, pb + pts_per_block);
  for (long base = pb + (long)wave * kQueue; base < pe; base += (long)kAccWaves * kQueue) {
    int lab[4];
    const long p4 = base + 4 * lane;
    if (p4 + 3 < pe) {
      const int4 l4 = *reinterpret_cast<const int4*>(labels + p4);
      lab[0] = l4.x; lab[1] = l4.y; lab[2] = l4.z; lab[3] = l4.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) lab[t] = (p4 + t < pe) ? labels[p4 + t] : -1;
    }
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int rel = lab[t] - c0;
      const bool mine = (unsigned)rel < (unsigned)cc;
      const unsigned long long m = __ballot(mine);
      if (mine) q[cnt + __popcll(m & lt_mask)] = ((uint32_t)(4 * lane + t) << 16) | (uint32_t)rel;
      cnt += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    for (int e = 0; e < cnt; e += U * GPW) {
      Row8<T> v[U];
      uint32_t ent[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = e + u * GPW + grp;
        ent[u] = idx < cnt ? q[idx] : 0xffffffffu;
        if (ent[u] != 0xffffffffu) v[u].load(X, base + (ent[u] >> 16), D, sub);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ent[u] != 0xffffffffu) {
          const int r = (int)(ent[u] & 0xffffu);
          lds_add_row<D>(s_acc, r, sub, v[u], scale);
          if (sub == 0) atomicAdd(s_cnt + r, 1u);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  flush_rows<D>(s_acc, s_cnt, c0, cc, sums, counts, tid, NT);
}

// ---------------------------------------------------------------------------
// Sorted (counting-sort) combiner for large k: no LDS float/int atomics in
// the hot loop at all.
//   1. kmeans_hist      : hist[label]++            (LDS u32 atomics, 1/point)
//   2. kmeans_scan      : offsets = exclusive_scan(hist); cursor = offsets;
//                         counts += hist
//   3. kmeans_scatter   : perm[offsets[l] + rank] = i, rank from a per-block
//                         LDS histogram (ds_add_rtn_u32) + one global atomic
//                         per (block, present label)
//   4. kmeans_segsum    : walk perm in order; each 16-lane group accumulates
//                         whole rows of one cluster in int64 registers and
//                         flushes once per cluster run (global u64 atomics).
// The gather in (4) re-reads each row once; run right after the assign kernel
// on a split of ≤ ~128 MB the rows come from the 256 MiB Infinity Cache.
constexpr int kScatterPts = 4096;  // points per scatter workgroup (16 per thread)

__global__ __launch_bounds__(256) void kmeans_hist_kernel(const int32_t* __restrict__ labels,
                                                          long n, int k,
                                                          uint32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];
  for (int i = threadIdx.x; i < k; i += 256) s_h[i] = 0u;
  __syncthreads();
  const long n4 = n / 4;
  const int4* l4 = reinterpret_cast<const int4*>(labels);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const int4 v = l4[i];
    atomicAdd(s_h + v.x, 1u);
    atomicAdd(s_h + v.y, 1u);
    atomicAdd(s_h + v.z, 1u);
    atomicAdd(s_h + v.w, 1u);
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256) atomicAdd(s_h + labels[i], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += 256)
    if (s_h[i]) atomicAdd(hist + i, s_h[i]);
}

// single workgroup: exclusive scan of hist (k ≤ 1024*64), counts += hist
__global__ __launch_bounds__(1024) void kmeans_scan_kernel(const uint32_t* __restrict__ hist,
                                                           int k, uint32_t* __restrict__ offsets,
                                                           uint32_t* __restrict__ cursor,
                                                           long long* __restrict__ counts) {
  __shared__ uint32_t s_part[1024];
  const int t = threadIdx.x;
  const int per = (k + 1023) / 1024;
  const int lo = min(k, t * per), hi = min(k, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += hist[i];
  s_part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= off ? s_part[t - off] : 0u;
    __syncthreads();
    s_part[t] += v;
    __syncthreads();
  }
  uint32_t run = s_part[t] - s;  // exclusive prefix of this thread's range
  for (int i = lo; i < hi; ++i) {
    const uint32_t h = hist[i];
    offsets[i] = run;
    cursor[i] = run;
    if (counts) counts[i] += h;
    run += h;
  }
  if (t == 1023) offsets[k] = s_part[1023];
}

__global__ __launch_bounds__(256) void kmeans_scatter_kernel(const int32_t* __restrict__ labels,
                                                             long n, int k,
                                                             uint32_t* __restrict__ cursor,
                                                             uint32_t* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // k counters, then k bases
  uint32_t* s_base = s_h + k;
  const int t = threadIdx.x;
  for (int i = t; i < k; i += 256) s_h[i] = 0u;
  __syncthreads();
  constexpr int PER = kScatterPts / 256;
  const long p0 = (long)blockIdx.x * kScatterPts + (long)t * PER;
  int lab[PER];
  uint32_t rank[PER];
#pragma unroll
  for (int j = 0; j < PER; j += 4) {
    if (p0 + j + 3 < n) {
      const int4 v = *reinterpret_cast<const int4*>(labels + p0 + j);
      lab[j] = v.x; lab[j + 1] = v.y; lab[j + 2] = v.z; lab[j + 3] = v.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) lab[j + q] = (p0 + j + q < n) ? labels[p0 + j + q] : -1;
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) rank[j] = lab[j] >= 0 ? atomicAdd(s_h + lab[j], 1u) : 0u;
  __syncthreads();
  for (int i = t; i < k; i += 256) {
    const uint32_t c = s_h[i];
    s_base[i] = c ? atomicAdd(cursor + i, c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (lab[j] >= 0) perm[s_base[lab[j]] + rank[j]] = (uint32_t)(p0 + j);
}

// Segmented row sum of the rows perm[s0:e) (sorted by cluster; cluster c owns
// perm[offsets[c]:offsets[c+1])) into out[c] (int64 fixed point).  The wave
// walks its range one cluster segment at a time: the GPW row groups split a
// segment's rows, U rows per group in flight (index load → row gather), and
// at the segment end the groups are reduced with xor-shuffles so each cluster
// costs one 128-value atomic flush per wave — spread over all groups — rather
// than one per group.  Segment bounds are wave-uniform (scalar loads).
// Row indirection of a segsum entry: the plain combiner's perm holds row
// indices; the delta combiner's holds (mover << 1 | sign) — see kmeans_delta_*.
struct IdentityRows {
  __device__ __forceinline__ uint32_t row(uint32_t i) const { return i; }
  __device__ __forceinline__ bool neg(uint32_t) const { return false; }
};

template <typename T, int D, int U, class Rows = IdentityRows>
__device__ __forceinline__ void segsum_range(const T* __restrict__ X,
                                             const uint32_t* __restrict__ pm,
                                             const uint32_t* __restrict__ of, int k, long s0,
                                             long e, u64* __restrict__ out, float scale,
                                             Rows rows = Rows()) {
  constexpr int TPP = D / 8;            // lanes per row
  constexpr int GPW = HBMR_WAVE / TPP;  // row groups per wave
  const int lane = threadIdx.x & 63;
  const int grp = lane / TPP, sub = lane % TPP;
  // first cluster whose segment contains s0: upper_bound(of, s0) - 1
  int lo = 0, hi = k;  // invariant of[lo] <= s0 < of[hi] (of[k] = n)
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if ((long)of[mid] <= s0) lo = mid; else hi = mid;
  }
  int cur = __builtin_amdgcn_readfirstlane(lo);
  long p = s0;
  while (p < e) {
    const long segE = min(e, (long)(uint32_t)__builtin_amdgcn_readfirstlane(of[cur + 1]));
    if (segE > p) {
      long long acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0;
      for (long base = p + grp; base < segE; base += (long)U * GPW) {
        uint32_t idx[U];
        Row8<T> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long q = base + (long)u * GPW;
          idx[u] = q < segE ? pm[q] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long q = base + (long)u * GPW;
          if (q < segE) v[u].load(X, rows.row(idx[u]), D, sub);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long q = base + (long)u * GPW;
          if (q < segE) {
            float f[8];
            v[u].unpack(f);
            if (rows.neg(idx[u])) {
              // round-half-even fixed point is odd-symmetric: fx(-x) = -fx(x)
#pragma unroll
              for (int j = 0; j < 8; ++j) f[j] = -f[j];
            }
            hbmr_fx_accum8(f, scale, acc);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int off = TPP; off < HBMR_WAVE; off <<= 1) acc[j] += __shfl_xor(acc[j], off);
      }
      u64* dst = out + (size_t)cur * D + sub * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j % GPW == grp % 8 && acc[j]) atomicAdd(dst + j, (u64)acc[j]);
      p = segE;
    }
    ++cur;
  }
}

template <typename T, int D, int U>
__global__ __launch_bounds__(256) void kmeans_segsum_kernel(
    const T* __restrict__ X, long n, const uint32_t* __restrict__ perm,
    const uint32_t* __restrict__ offsets, int k, long chunk, long long* __restrict__ sums,
    float scale) {
  const long wid = (long)blockIdx.x * (blockDim.x / HBMR_WAVE) + threadIdx.x / HBMR_WAVE;
  const long s = wid * chunk;
  if (s >= n) return;
  segsum_range<T, D, U>(X, perm, offsets, k, s, min(n, s + chunk), reinterpret_cast<u64*>(sums),
                        scale);
}

// ---- grouped sorted combiner ------------------------------------------------------
// hist[s][k] comes fused from the grouped assign.  Every scatter workgroup
// rebuilds the exclusive scan of its split's histogram in LDS (k ≤ 8192: a few
// µs) so no separate scan launch or grid-wide sync is needed; the workgroup
// with local index 0 of each split also publishes offsets[s] (for the segsum
// launch) and adds the histogram to that task's counts.
__device__ void block_exclusive_scan(const uint32_t* __restrict__ in, int k, uint32_t* out,
                                     uint32_t* total) {
  __shared__ uint32_t s_part[256];
  const int t = threadIdx.x;
  const int per = (k + 255) / 256;
  const int lo = min(k, t * per), hi = min(k, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += in[i];
  // wave-level inclusive scan, then across the 4 waves
  const int lane = t & 63, w = t >> 6;
  uint32_t v = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) s_part[w] = v;
  __syncthreads();
  uint32_t wbase = 0;
  for (int i = 0; i < w; ++i) wbase += s_part[i];
  uint32_t run = wbase + v - s;
  for (int i = lo; i < hi; ++i) {
    out[i] = run;
    run += in[i];
  }
  if (t == 255) *total = wbase + v;
  __syncthreads();
}

// Per-split label histogram from the labels array (alternative to the fused
// histogram atomics in the assign epilogue): LDS bins, one flush per block.
constexpr long kHistPts = 16384;
__global__ __launch_bounds__(256) void kmeans_hist_grouped_kernel(const SplitTable tbl,
                                                                  const int32_t* __restrict__ labels,
                                                                  uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t s_bins[];
  const int k = tbl.k;
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, blockIdx.x));
  const long local = blockIdx.x - tbl.blk[s];
  const long n = tbl.n[s];
  for (int i = threadIdx.x; i < k; i += 256) s_bins[i] = 0u;
  __syncthreads();
  const int32_t* lab = labels + tbl.off[s];
  const long p1 = min(n, (local + 1) * kHistPts);
  for (long p = local * kHistPts + threadIdx.x; p < p1; p += 256) atomicAdd(s_bins + lab[p], 1u);
  __syncthreads();
  uint32_t* hs = hist + (size_t)s * k;
  for (int i = threadIdx.x; i < k; i += 256)
    if (s_bins[i]) atomicAdd(hs + i, s_bins[i]);
}

__global__ __launch_bounds__(256) void kmeans_scatter_grouped_kernel(
    const SplitTable tbl, const int32_t* __restrict__ labels, const uint32_t* __restrict__ hist,
    uint32_t* __restrict__ cursor, uint32_t* __restrict__ offsets, uint32_t* __restrict__ perm,
    long long* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // off[k] | cnt[k] | base[k]
  const int k = tbl.k;
  uint32_t* s_off = s_h;
  uint32_t* s_cnt = s_h + k;
  uint32_t* s_base = s_h + 2 * k;
  __shared__ uint32_t s_total;
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, blockIdx.x));
  const long local = blockIdx.x - tbl.blk[s];
  const long n = tbl.n[s];
  const uint32_t* hs = hist + (size_t)s * k;
  const int t = threadIdx.x;
  for (int i = t; i < k; i += 256) s_cnt[i] = 0u;
  block_exclusive_scan(hs, k, s_off, &s_total);
  if (local == 0) {
    uint32_t* os = offsets + (size_t)s * (k + 1);
    for (int i = t; i < k; i += 256) {
      os[i] = s_off[i];
      counts[(size_t)s * k + i] += hs[i];
    }
    if (t == 0) os[k] = s_total;
  }
  constexpr int PER = kScatterPts / 256;
  const int32_t* lab_s = labels + tbl.off[s];
  const long p0 = local * kScatterPts + (long)t * PER;
  int lab[PER];
  uint32_t rank[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) lab[j] = (p0 + j < n) ? lab_s[p0 + j] : -1;
#pragma unroll
  for (int j = 0; j < PER; ++j) rank[j] = lab[j] >= 0 ? atomicAdd(s_cnt + lab[j], 1u) : 0u;
  __syncthreads();
  uint32_t* cur_s = cursor + (size_t)s * k;
  for (int i = t; i < k; i += 256) {
    const uint32_t c = s_cnt[i];
    s_base[i] = c ? s_off[i] + atomicAdd(cur_s + i, c) : 0u;
  }
  __syncthreads();
  uint32_t* perm_s = perm + tbl.off[s];
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (lab[j] >= 0) perm_s[s_base[lab[j]] + rank[j]] = (uint32_t)(p0 + j);
}

template <int D, int U>
__global__ __launch_bounds__(256) void kmeans_segsum_grouped_kernel(
    const SplitTable tbl, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ offsets,
    long chunk, long long* __restrict__ sums, float scale) {
  const int k = tbl.k;
  const long wid = (long)blockIdx.x * (blockDim.x / HBMR_WAVE) + threadIdx.x / HBMR_WAVE;
  // tbl.blk holds the prefix sum of WAVES (chunks) per split for this launch
  if (wid >= tbl.blk[tbl.nsplit]) return;
  const int sidx = __builtin_amdgcn_readfirstlane(find_split(tbl, wid));
  const long n = tbl.n[sidx];
  const long s0 = (wid - tbl.blk[sidx]) * chunk;
  segsum_range<__bf16, D, U>(tbl.X[sidx], perm + tbl.off[sidx], offsets + (size_t)sidx * (k + 1), k, s0,
                     min(n, s0 + chunk), reinterpret_cast<u64*>(sums) + (size_t)sidx * k * D,
                     scale);
}

// ---- delta combiner --------------------------------------------------------------
// The combiner output of a split is a function of its points and their labels
// only.  Given a reference partition g of the split (labels of an earlier
// pass) with its exact int64 sums S0[c] = Σ_{g(p)=c} fx(x_p) and counts N0,
// the sums for the new labels l are
//     S[c] = S0[c] + Σ_{l(p)=c, g(p)≠c} fx(x_p) - Σ_{g(p)=c, l(p)≠c} fx(x_p)
// (integer arithmetic: bit-identical to the direct combiner for ANY g).  Only
// the points whose label changed ("movers") are gathered, so once K-Means
// settles the combiner no longer re-reads the split: it is a pass over the
// labels plus a few thousand rows.  Afterwards (S0, N0, g) := (S, N, l), which
// the diff kernel does for g in place.
//
//   kmeans_slab_copy      : sums[t] = S0[t], counts[t] = N0[t]
//   kmeans_delta_diff     : movers (p, new << 16 | old), hist[c] = #entries,
//                           counts[t] += in - out, g[p] = l
//   kmeans_delta_scatter  : entries e = (mover << 1 | sign) sorted by cluster
//                           (+new for sign 0, -old for sign 1)
//   kmeans_delta_segsum   : segmented signed row sums of the entries into sums[t]
struct SlabTable {
  const long long* s[kMaxGroup];
  const long long* c[kMaxGroup];
};
struct GTable {
  int32_t* g[kMaxGroup];
};

__global__ __launch_bounds__(256) void kmeans_slab_copy_kernel(const SlabTable src, long slab,
                                                               int k, long long* __restrict__ sums,
                                                               long long* __restrict__ counts) {
  const int t = blockIdx.y;
  const long long* s = src.s[t];
  long long* d = sums + (size_t)t * slab;
  // slab = k * dp int64 (dp ≥ 64): whole 16-byte pieces
  const long npc = slab / 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < npc; i += (long)gridDim.x * 256)
    reinterpret_cast<int4*>(d)[i] = reinterpret_cast<const int4*>(s)[i];
  if (blockIdx.x == 0) {
    const long long* c = src.c[t];
    for (int i = threadIdx.x; i < k; i += 256) counts[(size_t)t * k + i] = c[i];
  }
}

constexpr long kDiffPts = 8192;  // points per diff workgroup
constexpr int kDiffPer = (int)(kDiffPts / 256);  // points per thread

// Every thread loads its 32 (label, reference label) pairs up front (strided
// by the workgroup width, so each load instruction is coalesced) — the loads
// are in flight together instead of one dependent round trip per 64 points —
// then the workgroup reserves room for all of its movers with ONE atomic on
// the split's mover count (a prefix sum over the threads' mover counts places
// each thread's movers).  Mover order is irrelevant downstream: the scatter
// sorts entries by cluster and the row sums are integer.
__global__ __launch_bounds__(256) void kmeans_delta_diff_kernel(
    const SplitTable tbl, const GTable gt, const int32_t* __restrict__ labels,
    uint2* __restrict__ movers, uint32_t* __restrict__ mcount, uint32_t* __restrict__ hist,
    long long* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_bins[];  // in[k] | out[k]
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_first;
  const int k = tbl.k;
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, blockIdx.x));
  const long local = blockIdx.x - tbl.blk[s];
  const long n = tbl.n[s];
  const int t = threadIdx.x;
  for (int i = t; i < 2 * k; i += 256) s_bins[i] = 0u;
  const int32_t* lab = labels + tbl.off[s];
  int32_t* g = gt.g[s];
  uint2* mv = movers + tbl.off[s];
  const int lane = t & 63, wave = t >> 6;
  const long p0 = local * kDiffPts + t;
  const long p1 = min(n, (local + 1) * kDiffPts);
  int32_t l[kDiffPer], o[kDiffPer];
  // branch-free: every load is issued (index clamped into the workgroup's
  // range, which holds at least one point) and out-of-range pairs zeroed by a
  // select, so all 64 loads of a thread are in flight together
#pragma unroll
  for (int j = 0; j < kDiffPer; ++j) {
    const long p = p0 + (long)j * 256;
    const bool in = p < p1;
    const long pc = in ? p : p1 - 1;
    const int32_t a = lab[pc], b = g[pc];
    l[j] = in ? a : 0;
    o[j] = in ? b : 0;
  }
  // (a label outside [0, k) would index past the bins and the slabs: such a
  // point is never a mover — the bit-exactness tests catch it)
  uint32_t chm = 0u;
  uint32_t pk[kDiffPer];  // new << 16 | old (k <= 8192)
#pragma unroll
  for (int j = 0; j < kDiffPer; ++j) {
    const bool ch = l[j] != o[j] && (unsigned)l[j] < (unsigned)k && (unsigned)o[j] < (unsigned)k;
    chm |= (uint32_t)ch << j;
    pk[j] = ((uint32_t)l[j] << 16) | ((uint32_t)o[j] & 0xffffu);
  }
  const uint32_t cnt = (uint32_t)__popc(chm);
  uint32_t x = cnt;  // inclusive prefix over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  if (t == 0) {
    const uint32_t tot = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    s_first = tot ? atomicAdd(mcount + s, tot) : 0u;
  }
  __syncthreads();
  if (chm) {
    uint32_t i = s_first + x - cnt;
    for (int w = 0; w < wave; ++w) i += s_wsum[w];
#pragma unroll
    for (int j = 0; j < kDiffPer; ++j) {
      if ((chm >> j) & 1u) {
        const uint32_t p = (uint32_t)(p0 + (long)j * 256);
        const uint32_t nl = pk[j] >> 16, ol = pk[j] & 0xffffu;
        mv[i++] = make_uint2(p, pk[j]);
        g[p] = (int32_t)nl;
        atomicAdd(s_bins + nl, 1u);
        atomicAdd(s_bins + k + ol, 1u);
      }
    }
  }
  __syncthreads();
  uint32_t* hs = hist + (size_t)s * k;
  u64* cs = reinterpret_cast<u64*>(counts) + (size_t)s * k;
  for (int c = t; c < k; c += 256) {
    const uint32_t in = s_bins[c], out = s_bins[k + c];
    if (in | out) {
      atomicAdd(hs + c, in + out);
      if (in != out) atomicAdd(cs + c, (u64)((long long)in - (long long)out));
    }
  }
}

// tbl.blk: prefix of scatter workgroups per split sized for the worst case
// (every point moved: 2n entries); surplus workgroups leave after the scan.
__global__ __launch_bounds__(256) void kmeans_delta_scatter_kernel(
    const SplitTable tbl, const uint2* __restrict__ movers, const uint32_t* __restrict__ mcount,
    const uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor,
    uint32_t* __restrict__ offsets, uint32_t* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // off[k] | cnt[k] | base[k]
  const int k = tbl.k;
  __shared__ uint32_t s_total;
  const int s = __builtin_amdgcn_readfirstlane(find_split(tbl, blockIdx.x));
  const long local = blockIdx.x - tbl.blk[s];
  const long ne = 2L * (long)__builtin_amdgcn_readfirstlane(mcount[s]);
  if (local > 0 && local * kScatterPts >= ne) return;   // uniform: nothing for this block
  uint32_t* s_off = s_h;
  uint32_t* s_cnt = s_h + k;
  uint32_t* s_base = s_h + 2 * k;
  const int t = threadIdx.x;
  for (int i = t; i < k; i += 256) s_cnt[i] = 0u;
  block_exclusive_scan(hist + (size_t)s * k, k, s_off, &s_total);
  if (local == 0) {
    uint32_t* os = offsets + (size_t)s * (k + 1);
    for (int i = t; i < k; i += 256) os[i] = s_off[i];
    if (t == 0) os[k] = s_total;
  }
  constexpr int PER = kScatterPts / 256;
  const uint2* mv = movers + tbl.off[s];
  const long e0 = local * kScatterPts + (long)t * PER;
  int cl[PER];
  uint32_t rank[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const long e = e0 + j;
    cl[j] = -1;
    if (e < ne) {
      const uint32_t y = mv[e >> 1].y;
      cl[j] = (e & 1) ? (int)(y & 0xffffu) : (int)(y >> 16);
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) rank[j] = cl[j] >= 0 ? atomicAdd(s_cnt + cl[j], 1u) : 0u;
  __syncthreads();
  uint32_t* cur_s = cursor + (size_t)s * k;
  for (int i = t; i < k; i += 256) {
    const uint32_t c = s_cnt[i];
    s_base[i] = c ? s_off[i] + atomicAdd(cur_s + i, c) : 0u;
  }
  __syncthreads();
  uint32_t* perm_s = perm + 2 * tbl.off[s];
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (cl[j] >= 0) perm_s[s_base[cl[j]] + rank[j]] = (uint32_t)(e0 + j);
}

struct MoverRows {
  const uint2* mv;
  __device__ __forceinline__ uint32_t row(uint32_t e) const { return mv[e >> 1].x; }
  __device__ __forceinline__ bool neg(uint32_t e) const { return (e & 1u) != 0u; }
};

// Persistent grid: wave items (split, chunk of `chunk` entries) in split order,
// counted from the device-side mover counts.
template <typename T, int D, int U>
__global__ __launch_bounds__(256) void kmeans_delta_segsum_kernel(
    const SplitTable tbl, const uint2* __restrict__ movers, const uint32_t* __restrict__ mcount,
    const uint32_t* __restrict__ perm, const uint32_t* __restrict__ offsets, long chunk,
    long long* __restrict__ sums, float scale) {
  const int k = tbl.k;
  const long nw = (long)gridDim.x * (blockDim.x / HBMR_WAVE);
  long wid = (long)blockIdx.x * (blockDim.x / HBMR_WAVE) + threadIdx.x / HBMR_WAVE;
  int s = 0;
  long sbase = 0;
  long items = (2L * (long)__builtin_amdgcn_readfirstlane(mcount[0]) + chunk - 1) / chunk;
  for (; ; wid += nw) {
    while (wid >= sbase + items) {
      sbase += items;
      if (++s >= tbl.nsplit) return;
      items = (2L * (long)__builtin_amdgcn_readfirstlane(mcount[s]) + chunk - 1) / chunk;
    }
    const long ne = 2L * (long)__builtin_amdgcn_readfirstlane(mcount[s]);
    const long e0 = (wid - sbase) * chunk;
    segsum_range<T, D, U, MoverRows>(
        reinterpret_cast<const T*>(tbl.X[s]), perm + 2 * tbl.off[s],
        offsets + (size_t)s * (k + 1), k, e0, min(ne, e0 + chunk),
        reinterpret_cast<u64*>(sums) + (size_t)s * k * D, scale, MoverRows{movers + tbl.off[s]});
  }
}

// Reduce side + next-iteration prep.  One workgroup per cluster.
// sums are fixed-point int64 [k, dp], counts int64 [k].
__global__ __launch_bounds__(128) void kmeans_update_kernel(
    const long long* __restrict__ sums, const long long* __restrict__ counts, int k, int d,
    int dp, float inv_scale, float* __restrict__ cen, __bf16* __restrict__ cbf,
    float* __restrict__ chalf, float* __restrict__ shift2) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ float red[2][128];
  const long long cnt = counts ? counts[j] : 0;
  const double inv = cnt > 0 ? (double)inv_scale / (double)cnt : 0.0;
  float nrm = 0.f, dsq = 0.f;
  uint16_t* cb = reinterpret_cast<uint16_t*>(cbf) + (size_t)j * dp;
  for (int i = tid; i < dp; i += 128) {
    float v = 0.f;
    if (i < d) {
      const float old = cen[(size_t)j * d + i];
      v = cnt > 0 ? (float)((double)sums[(size_t)j * dp + i] * inv) : old;
      dsq += (v - old) * (v - old);
      cen[(size_t)j * d + i] = v;
    }
    const uint16_t b = hbmr_f32_to_bf16(v);
    cb[i] = b;
    const float vb = hbmr_bf16_to_f32(b);
    nrm += vb * vb;
  }
  red[0][tid] = nrm;
  red[1][tid] = dsq;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0) {
    chalf[j] = -0.5f * red[0][0];
    if (shift2) shift2[j] = red[1][0];
  }
}

__global__ __launch_bounds__(256) void f32_to_bf16_pad_kernel(const float* __restrict__ src,
                                                              long n, int d, int dp,
                                                              uint16_t* __restrict__ dst) {
  const long total = n * dp;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long r = e / dp;
    const int c = (int)(e - r * dp);
    dst[e] = c < d ? hbmr_f32_to_bf16(src[r * d + c]) : (uint16_t)0;
  }
}

__global__ void kmeans_pad_clusters_kernel(__bf16* cbf, float* chalf, int k, int k_pad, int dp) {
  const int j = k + blockIdx.x;
  if (j >= k_pad) return;
  uint16_t* cb = reinterpret_cast<uint16_t*>(cbf) + (size_t)j * dp;
  for (int i = threadIdx.x; i < dp; i += blockDim.x) cb[i] = 0;
  if (threadIdx.x == 0) chalf[j] = -1.0e30f;
}

template <int D>
int launch_assign(const void* X, long n, const void* C, const float* chalf, int k_pad,
                  int32_t* labels, float* scores, hipStream_t st) {
  using Cfg = AssignCfg<D>;
  if (n <= 0) return 0;
  if (k_pad % kCK) return (int)hipErrorInvalidValue;
  const int pts = assign_pts<D>(false);
  const long nblk = (n + pts - 1) / pts;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  if constexpr (D <= 128) {
    if (assign_version(D) == 2) {
      auto kern = v2_pb() == 3 ? kmeans_assign_v2_kernel<D, 3> : kmeans_assign_v2_kernel<D, 2>;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(AssignV2<D>::THREADS),
                         AssignV2<D>::LDS_BYTES, st, reinterpret_cast<const __bf16*>(X), n,
                         reinterpret_cast<const __bf16*>(C), chalf, k_pad / 32, labels, scores);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL(kmeans_assign_kernel<D>, dim3((unsigned)nblk), dim3(kThreads),
                     Cfg::LDS_BYTES, st, reinterpret_cast<const __bf16*>(X), n,
                     reinterpret_cast<const __bf16*>(C), chalf, k_pad / kCK, labels, scores);
  return (int)hipGetLastError();
}

template <int D>
void launch_grouped_assign(long nb, const SplitTable& t, const void* C, const float* chalf,
                           int k_pad, int32_t* labels, uint32_t* hist, hipStream_t st) {
  if constexpr (D <= 128) {
    if (assign_version(D) == 2 && hist == nullptr) {
      auto kern = v2_pb() == 3 ? kmeans_assign_grouped_v2_kernel<D, 3>
                               : kmeans_assign_grouped_v2_kernel<D, 2>;
      hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(AssignV2<D>::THREADS),
                         AssignV2<D>::LDS_BYTES, st, t, reinterpret_cast<const __bf16*>(C),
                         chalf, k_pad / 32, labels);
      return;
    }
  }
  hipLaunchKernelGGL(kmeans_assign_grouped_kernel<D>, dim3((unsigned)nb), dim3(kThreads),
                     AssignCfg<D>::LDS_BYTES, st, t, reinterpret_cast<const __bf16*>(C), chalf,
                     k_pad / kCK, labels, hist);
}

template <typename T, int D>
int launch_accum(const void* Xv, long n, const int32_t* labels, int k, long long* sums,
                 long long* counts, float scale, int num_cu, hipStream_t st) {
  using A = AccCfg<D>;
  if (n <= 0) return 0;
  const T* X = reinterpret_cast<const T*>(Xv);
  const size_t small_bytes = (size_t)k * A::RS * 8 + (size_t)k * 4;
  if (small_bytes <= 76 * 1024) {
    constexpr int U = 8;
    const long per_block = 256 / A::TPP * U;
    long grid = std::min<long>((n + per_block - 1) / per_block, (long)num_cu * 2);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((kmeans_accum_lds_kernel<T, D, U>), dim3((unsigned)grid), dim3(256),
                       small_bytes, st, X, n, labels, k, sums, counts, scale);
  } else {
    // one workgroup per CU: CC u64 rows + queues + counts within ~150 KiB
    constexpr int U = 8;
    const size_t qbytes = (size_t)kAccWaves * kQueue * 4;
    int CC = (int)((150 * 1024 - qbytes) / ((size_t)A::RS * 8 + 4));
    CC = (CC / 8) * 8;
    if (CC > k) CC = k;
    const int nchunk = (k + CC - 1) / CC;
    long nb = ((long)num_cu + nchunk - 1) / nchunk;
    long ppb = (n + nb - 1) / nb;
    ppb = ((ppb + 2047) / 2048) * 2048;
    nb = (n + ppb - 1) / ppb;
    const size_t lds = (size_t)CC * A::RS * 8 + qbytes + (size_t)CC * 4;
    hipLaunchKernelGGL((kmeans_accum_chunked_kernel<T, D, U>), dim3((unsigned)nb, (unsigned)nchunk),
                       dim3(kAccWaves * HBMR_WAVE), lds, st, X, n, labels, k, CC, ppb, sums,
                       counts, scale);
  }
  return (int)hipGetLastError();
}

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

bool set_lds_limits() {
  // Opt every kernel that asks for >64 KiB of dynamic LDS into the full 160 KiB.
  // The limit is static + dynamic, so a kernel with static __shared__ arrays
  // may ask for less; a refused opt-in must not leave a sticky error behind
  // for the next launch's hipGetLastError.
  static bool done = false;
  if (!done) {
    auto optin = [](const void* fn) {
      hipFuncAttributes at{};
      size_t stat = 0;
      if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(160 * 1024 - stat)) != hipSuccess)
        (void)hipGetLastError();
    };
#define HBMR_LDS_OPTIN(fn) optin((const void*)(fn))
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<__bf16, 64, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<__bf16, 128, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<__bf16, 256, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<__bf16, 64, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<__bf16, 128, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<__bf16, 256, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<float, 64, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<float, 128, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_lds_kernel<float, 256, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<float, 64, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<float, 128, 8>));
    HBMR_LDS_OPTIN((kmeans_accum_chunked_kernel<float, 256, 8>));
    HBMR_LDS_OPTIN(kmeans_scatter_grouped_kernel);
    HBMR_LDS_OPTIN(kmeans_delta_scatter_kernel);
    HBMR_LDS_OPTIN(kmeans_delta_diff_kernel);
#undef HBMR_LDS_OPTIN
    done = true;
  }
  return done;
}

// ---------------------------------------------------------------------------
// Exact mode, step 2: certify each point's bf16 arg-max against its fp32 data
// and re-score the uncertain points in fp64.
//
// The assign kernel ranks s~_j = x~.c~_j - |c~_j|^2/2 (x~, c~ = bf16 of the fp32
// x, c; fp32 accumulation), i.e. the bf16 distances D~_j = |x~ - c~_j|^2.  With
// the rounding errors themselves, e_x = |x - x~| and e_j = |c_j - c~_j| (fp64,
// rounded up; the worst case u = 2^-8 of bf16's 8 significant bits would give
// u|x|, u|c_j| — about 3.5x looser for round-to-nearest data, and the flagged
// fraction scales with it)
// |(x~ - c~_j) - (x - c_j)| <= a_j = e_x + e_j, so
// |D~_j - D_j| <= a_j (2 sqrt(D~_j) + a_j).  In score units (D/2), adding the
// fp32 accumulation error e_acc and the arg-max packing truncation e_pack:
//     E_j = a_j (2 sqrt(D~_j) + a_j) / 2 + e_acc_j + e_pack_j,   |s~_j - s_j| <= E_j.
// Any cluster t ranked below a cluster r by the kernel (s~_t <= s~_r, so
// D~_t >= D~_r) has  s_t <= s~_r + E_max(r)  (E with |c_t| <= cmax and
// e_t <= e_max; the score falls faster than E_t grows once sqrt(D~_r) >= 2 a_max).  Hence, with the
// kernel's top three b, s, t:
//   1. margin(b, s) > E_b + E_max(s)                 -> b is the exact winner;
//   2. else D_b, D_s, D_t in fp64 from the fp32 rows; the winner w of the three
//      (ties to the lower index) is exact if (|x|^2 - D_w)/2 > s~_t + E_max(t);
//   3. else an Elkan scan: |x - c_j| >= |c_w - c_j| - |x - c_w|, so walking w's
//      centroid neighbours in ascending |c_w - c_j| (nbr_idx / nbr_dist, L per
//      centroid, distances rounded down) can stop at |c_w - c_j| > r_w + r_best;
//      a point that outruns its L neighbours scans every centroid.
// Steps 2-3 run on groups of 16 lanes (8 features per lane, fp64, the point
// held in registers), four flagged points per wave at a time.
// stats += (flagged, relabelled, points that needed step 3).
constexpr int kRefineGroup = 16;
constexpr int kRefineMaxDp = 256;
constexpr int kRefinePer = kRefineMaxDp / kRefineGroup;  // features per lane

// Error bound E of a kernel score sc (point norm xn, |x~|^2 = x2) against a
// centroid of norm cn whose distance vector carries rounding error <= a, and a
// lower bound of sqrt(D~) for the monotonicity test.
__device__ __forceinline__ void exact_bound(double sc, double ct, double xt, double x2, double a,
                                            double gam, double pack_rel, double& e,
                                            double& dlo) {
  // ct, xt: upper bounds of |c~| and |x~| (|c| + |c - c~|, |x| + |x - x~|: no
  // relative-rounding assumption, so fp16 subnormals and saturation are covered)
  const double eacc = gam * (xt * ct + 0.5 * ct * ct);
  const double epack = fabs(sc) * pack_rel;
  const double slack = 2.0 * (eacc + epack) + x2 * 0x1p-22;
  const double dhi = fmax(0.0, x2 - 2.0 * sc) + slack;
  dlo = sqrt(fmax(0.0, x2 - 2.0 * sc - slack));
  e = a * (2.0 * sqrt(dhi) + a) * 0.5 + eacc + epack;
}

// Error of a kernel score sc against the exact rounded-operand score
// (accumulation + packing, eap) and an upper bound of sqrt(D~) (rdhi), for a
// centroid with |c~| <= ct and |x~| <= xt (see exact_bound).
__device__ __forceinline__ void score_err(double sc, double ct, double xt, double x2, double gam,
                                          double pack_rel, double& eap, double& rdhi) {
  const double eacc = gam * (xt * ct + 0.5 * ct * ct);
  eap = eacc + fabs(sc) * pack_rel;
  rdhi = sqrt(fmax(0.0, x2 - 2.0 * sc) + 2.0 * eap + x2 * 0x1p-22);
}

__device__ __forceinline__ double group_sum16(double v) {
#pragma unroll
  for (int off = 1; off < kRefineGroup; off <<= 1) v += __shfl_xor(v, off);
  return v;
}

// |x - c_j|^2 in fp64; xv holds this lane's features 8*sub + 128*m + (0..7)
__device__ __forceinline__ double group_dist2(const double (&xv)[kRefinePer],
                                              const float* __restrict__ c, int d, int sub) {
  double acc = 0.0;
#pragma unroll
  for (int m = 0; m < kRefinePer / 8; ++m) {
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int i = 8 * sub + 8 * kRefineGroup * m + jj;
      if (i < d) {
        const double e = xv[8 * m + jj] - (double)c[i];
        acc = fma(e, e, acc);
      }
    }
  }
  return group_sum16(acc);
}

// Four distances at once (the Elkan scan's candidates): the loads and FMA
// chains of four centroid rows interleave, and so do the four reductions —
// a scan step otherwise waits out one row's L2 latency and one shuffle chain.
__device__ __forceinline__ void group_dist2x4(const double (&xv)[kRefinePer],
                                              const float* __restrict__ c0,
                                              const float* __restrict__ c1,
                                              const float* __restrict__ c2,
                                              const float* __restrict__ c3, int d, int sub,
                                              double (&out)[4]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
  for (int m = 0; m < kRefinePer / 8; ++m) {
    const int b = 8 * sub + 8 * kRefineGroup * m;
    if (b + 8 <= d) {
      float v0[8], v1[8], v2[8], v3[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        v0[jj] = c0[b + jj];
        v1[jj] = c1[b + jj];
        v2[jj] = c2[b + jj];
        v3[jj] = c3[b + jj];
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const double x = xv[8 * m + jj];
        const double e0 = x - (double)v0[jj], e1 = x - (double)v1[jj];
        const double e2 = x - (double)v2[jj], e3 = x - (double)v3[jj];
        a0 = fma(e0, e0, a0);
        a1 = fma(e1, e1, a1);
        a2 = fma(e2, e2, a2);
        a3 = fma(e3, e3, a3);
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        if (b + jj < d) {
          const double x = xv[8 * m + jj];
          const double e0 = x - (double)c0[b + jj], e1 = x - (double)c1[b + jj];
          const double e2 = x - (double)c2[b + jj], e3 = x - (double)c3[b + jj];
          a0 = fma(e0, e0, a0);
          a1 = fma(e1, e1, a1);
          a2 = fma(e2, e2, a2);
          a3 = fma(e3, e3, a3);
        }
      }
    }
  }
#pragma unroll
  for (int off = 1; off < kRefineGroup; off <<= 1) {
    a0 += __shfl_xor(a0, off);
    a1 += __shfl_xor(a1, off);
    a2 += __shfl_xor(a2, off);
    a3 += __shfl_xor(a3, off);
  }
  out[0] = a0;
  out[1] = a1;
  out[2] = a2;
  out[3] = a3;
}

__global__ __launch_bounds__(256) void kmeans_refine_kernel(
    const float* __restrict__ X32, long n, int d, int ldx, const float* __restrict__ xnorm,
    const float* __restrict__ xbn2, const float* __restrict__ xerr,
    const float* __restrict__ C32, int k, const float* __restrict__ cnorm,
    const float* __restrict__ cmax, const float* __restrict__ cerr,
    const float* __restrict__ cerrmax, double pack_rel,
    const int32_t* __restrict__ nbr_idx, const float* __restrict__ nbr_dist, int L,
    int32_t* __restrict__ labels, const int32_t* __restrict__ cand,
    const float* __restrict__ score, const float* __restrict__ margin,
    unsigned long long* __restrict__ stats, int nstats) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  // the counters gather in LDS, one global atomic per counter and block: one
  // per event on a single address serialised ~10^6 atomics per 12.5M points
  __shared__ unsigned long long cnt[5];
  if (threadIdx.x < 5) cnt[threadIdx.x] = 0;
  __syncthreads();
  const double inflate = 1.0 + 0x1p-20;
  const double gam = (double)(d + 2) * 0x1p-23 * 1.01;
  const double cem = (double)cerrmax[0] * inflate;
  const double cm = (double)cmax[0] * inflate + cem;  // bound of |c~_j| for every j
  bool flag = false;
  int b = 0, s2 = 0, s3 = 0;
  double xn = 0.0, x2 = 0.0, sb = 0.0, m3 = 0.0, amax = 0.0;
  if (p < n) {
    b = labels[p];
    s2 = cand[p];
    s3 = cand[n + p];
    if (s2 < k) {  // a padded runner-up (-1e30) is never close: k == 1
      xn = ((double)xnorm[p] + (double)xerr[p]) * inflate;  // bound of |x~|
      x2 = (double)xbn2[p];
      sb = score[p];
      const double m2 = margin[p];
      m3 = margin[n + p];
      const double xe = (double)xerr[p];
      amax = (xe + cem) * inflate;
      double eb, es, dl_b, dl_s;
      exact_bound(sb, ((double)cnorm[b] + (double)cerr[b]) * inflate, xn, x2, (xe + (double)cerr[b]) * inflate,
                  gam, pack_rel, eb, dl_b);
      exact_bound(sb - m2, cm, xn, x2, amax, gam, pack_rel, es, dl_s);
      flag = !(m2 > eb + es && dl_s >= 2.0 * amax);
    }
  }
  unsigned long long mask = __ballot(flag);
  if (lane == 0 && mask) atomicAdd(&cnt[0], (unsigned long long)__popcll(mask));
  const int grp = lane / kRefineGroup, sub = lane % kRefineGroup;
  // four groups take the flagged points of this wave in turn
  while (mask) {
    unsigned long long m = mask;  // the grp-th set bit of mask (or none)
    for (int i = 0; i < grp && m; ++i) m &= m - 1;
    const bool have = m != 0;
    const int src = have ? __ffsll((long long)m) - 1 : 0;
    for (int i = 0; i < 4 && mask; ++i) mask &= mask - 1;
    const long q = __shfl(p, src);
    const int qb = __shfl(b, src), qs = __shfl(s2, src), qt = __shfl(s3, src);
    const double qsb = __shfl(sb, src), qm3 = __shfl(m3, src);
    const double qxn = __shfl(xn, src), qx2 = __shfl(x2, src), qamax = __shfl(amax, src);
    if (!have) continue;
    const float* xr = X32 + (size_t)q * ldx;
    double xv[kRefinePer];
#pragma unroll
    for (int mm = 0; mm < kRefinePer / 8; ++mm)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int i = 8 * sub + 8 * kRefineGroup * mm + jj;
        xv[8 * mm + jj] = i < d ? (double)xr[i] : 0.0;
      }
    const bool t_real = qt < k;
    const double db = group_dist2(xv, C32 + (size_t)qb * d, d, sub);
    const double ds = group_dist2(xv, C32 + (size_t)qs * d, d, sub);
    const double dt = t_real ? group_dist2(xv, C32 + (size_t)qt * d, d, sub) : 0.0;
    int w = qb;
    double dw = db;
    if (ds < dw || (ds == dw && qs < w)) { w = qs; dw = ds; }
    if (t_real && (dt < dw || (dt == dw && qt < w))) { w = qt; dw = dt; }
    bool certified = !t_real;
    if (t_real) {
      double et, dl_t;
      exact_bound(qsb - qm3, cm, qxn, qx2, qamax, gam, pack_rel, et, dl_t);
      // scores are on the bf16 point's baseline: s_t = (|x~|^2 - D_t)/2 with
      // exact D; |x~|^2 (qx2) was stored in fp32, hence the 2^-23 margin.
      // (|x|^2 of the fp32 row would differ by ~|x| e_x, a shift the bound
      // does not carry)
      certified = 0.5 * (qx2 - dw) - qx2 * 0x1p-23 > (qsb - qm3) + et &&
                  dl_t >= 2.0 * qamax;
    }
    if (!certified) {
      if (sub == 0) atomicAdd(&cnt[2], 1ull);
      // step 3: Elkan scan around w0 = w (exact distance r0)
      const int w0 = w;
      const double r0 = sqrt(dw);
      bool done = false;
      const int32_t* ni = nbr_idx + (size_t)w0 * L;
      const float* nd = nbr_dist + (size_t)w0 * L;
      // four neighbours per step: the exit bound r0 + r_best is taken at the
      // step's start (r_best only shrinks, so it admits a superset of the
      // candidates the one-at-a-time walk would visit; the minimum over a
      // superset is the same exact winner)
      const float* cw0 = C32 + (size_t)w0 * d;
      int evals = 0;
      for (int jj = 0; jj < L; jj += 4) {
        const double lim = (r0 + sqrt(dw)) * (1.0 + 0x1p-40);
        if ((double)nd[jj] > lim) {
          done = true;
          break;
        }
        int jv[4];
        const float* cp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = jj + u < L && (double)nd[jj + u] <= lim;
          jv[u] = ok ? ni[jj + u] : -1;
          cp[u] = ok ? C32 + (size_t)jv[u] * d : cw0;
        }
        double dj[4];
        group_dist2x4(xv, cp[0], cp[1], cp[2], cp[3], d, sub, dj);
        evals += 4;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (jv[u] >= 0 && (dj[u] < dw || (dj[u] == dw && jv[u] < w))) { w = jv[u]; dw = dj[u]; }
      }
      if (sub == 0) {
        atomicAdd(&cnt[3], (unsigned long long)evals);
        if (!done && L < k) atomicAdd(&cnt[4], 1ull);
      }
      if (!done && L < k) {
        for (int j = 0; j < k; j += 4) {  // outran the neighbour list: every centroid
          const float* cp[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) cp[u] = C32 + (size_t)(j + u < k ? j + u : j) * d;
          double dj[4];
          group_dist2x4(xv, cp[0], cp[1], cp[2], cp[3], d, sub, dj);
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j + u < k && (dj[u] < dw || (dj[u] == dw && j + u < w))) { w = j + u; dw = dj[u]; }
        }
      }
    }
    if (sub == 0 && w != qb) {
      labels[q] = w;
      atomicAdd(&cnt[1], 1ull);
    }
  }
  __syncthreads();
  if (threadIdx.x < (nstats < 5 ? 3 : 5) && cnt[threadIdx.x])
    atomicAdd(stats + threadIdx.x, cnt[threadIdx.x]);
}

// Refine v2: the same certification and the same fp64 sums, bit for bit, laid
// out for latency.  v1 (above) reads rows with 211 scalar dword loads and
// reduces with ds_bpermute shuffles at 163 VGPRs (3 waves per SIMD), so a
// flagged point waits out one L2 round trip per row.  v2 takes NM = ceil(d/128)
// chunks at compile time, loads every row as 16-byte vectors (d % 8 == 0,
// 16-byte aligned rows), issues the point row and all candidate rows before
// the first FMA, and reduces over the 16-lane group with DPP row operations
// (quad_perm, row_half_mirror, row_mirror — one DPP row is 16 lanes), which
// add in the same pairwise order as v1's xor butterfly.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += dpp_f64<0x141>(v);  // row_half_mirror: the other quad of the half-row
  v += dpp_f64<0x140>(v);  // row_mirror: the other half of the row
  return v;
}

template <int NM>
__device__ __forceinline__ void load_row8(const float* __restrict__ r, int d, int sub,
                                          float (&v)[8 * NM]) {
  // branch-free (see load_row16): clamped address + select, no per-load wait.
  // Lane sub of the 16-lane group owns features 128m + 64h + 4sub + (0..3):
  // each float4 load of the group reads 256 contiguous bytes of the row
#pragma unroll
  for (int m = 0; m < NM; ++m) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = 128 * m + 64 * h + 4 * sub;
      const bool ok = b < d;
      const float4 a = *reinterpret_cast<const float4*>(r + (ok ? b : 0));
      float* o = v + 8 * m + 4 * h;
      o[0] = ok ? a.x : 0.f; o[1] = ok ? a.y : 0.f; o[2] = ok ? a.z : 0.f; o[3] = ok ? a.w : 0.f;
    }
  }
}

// R rows' |x - c|^2 (features past d are zero on both sides: fma(0, 0, acc) = acc)
template <int NM, int R>
__device__ __forceinline__ void rows_dist2(const double (&xv)[8 * NM],
                                           const float* const (&rows)[R], int d, int sub,
                                           double (&out)[R]) {
  float cv[R][8 * NM];
#pragma unroll
  for (int r = 0; r < R; ++r) load_row8<NM>(rows[r], d, sub, cv[r]);
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
#pragma unroll
  for (int i = 0; i < 8 * NM; ++i)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double e = xv[i] - (double)cv[r][i];
      acc[r] = fma(e, e, acc[r]);
    }
#pragma unroll
  for (int r = 0; r < R; ++r) out[r] = row_sum16(acc[r]);
}

// neighbours per Elkan step: 2 keeps v2 at 128 VGPRs (4 waves per SIMD; 4 rows
// in flight take 134, 3 waves).  The exit bound refreshes every step, and the
// minimum over any superset of the one-at-a-time walk is the same winner.
#ifndef HBMR_ELKAN_STEP
#define HBMR_ELKAN_STEP 2
#endif
constexpr int kElkanStep = HBMR_ELKAN_STEP;

template <int NM>
__global__ __launch_bounds__(256) void kmeans_refine_v2_kernel(
    const float* __restrict__ X32, long n, int d, int ldx, const float* __restrict__ xnorm,
    const float* __restrict__ xbn2, const float* __restrict__ xerr,
    const float* __restrict__ C32, int k, const float* __restrict__ cnorm,
    const float* __restrict__ cmax, const float* __restrict__ cerr,
    const float* __restrict__ cerrmax, double pack_rel,
    const int32_t* __restrict__ nbr_idx, const float* __restrict__ nbr_dist, int L,
    int32_t* __restrict__ labels, const int32_t* __restrict__ cand,
    const float* __restrict__ score, const float* __restrict__ margin,
    unsigned long long* __restrict__ stats, int nstats) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  __shared__ unsigned long long cnt[5];
  if (threadIdx.x < 5) cnt[threadIdx.x] = 0;
  __syncthreads();
  const double inflate = 1.0 + 0x1p-20;
  const double gam = (double)(d + 2) * 0x1p-23 * 1.01;
  const double cem = (double)cerrmax[0] * inflate;
  const double cm = (double)cmax[0] * inflate + cem;  // bound of |c~_j| for every j
  bool flag = false;
  int b = 0, s2 = 0, s3 = 0;
  double xn = 0.0, x2 = 0.0, sb = 0.0, m3 = 0.0, amax = 0.0;
  if (p < n) {
    b = labels[p];
    s2 = cand[p];
    s3 = cand[n + p];
    if (s2 < k) {
      xn = ((double)xnorm[p] + (double)xerr[p]) * inflate;  // bound of |x~|
      x2 = (double)xbn2[p];
      sb = score[p];
      const double m2 = margin[p];
      m3 = margin[n + p];
      const double xe = (double)xerr[p];
      amax = (xe + cem) * inflate;
      double eb, es, dl_b, dl_s;
      exact_bound(sb, ((double)cnorm[b] + (double)cerr[b]) * inflate, xn, x2, (xe + (double)cerr[b]) * inflate,
                  gam, pack_rel, eb, dl_b);
      exact_bound(sb - m2, cm, xn, x2, amax, gam, pack_rel, es, dl_s);
      flag = !(m2 > eb + es && dl_s >= 2.0 * amax);
    }
  }
  unsigned long long mask = __ballot(flag);
  if (lane == 0 && mask) atomicAdd(&cnt[0], (unsigned long long)__popcll(mask));
  const int grp = lane / kRefineGroup, sub = lane % kRefineGroup;
  while (mask) {
    unsigned long long m = mask;
    for (int i = 0; i < grp && m; ++i) m &= m - 1;
    const bool have = m != 0;
    const int src = have ? __ffsll((long long)m) - 1 : 0;
    for (int i = 0; i < 4 && mask; ++i) mask &= mask - 1;
    const long q = __shfl(p, src);
    const int qb = __shfl(b, src), qs = __shfl(s2, src), qt = __shfl(s3, src);
    const double qsb = __shfl(sb, src), qm3 = __shfl(m3, src);
    const double qxn = __shfl(xn, src), qx2 = __shfl(x2, src), qamax = __shfl(amax, src);
    if (!have) continue;
    const bool t_real = qt < k;
    double xv[8 * NM];
    {
      float xf[8 * NM];
      load_row8<NM>(X32 + (size_t)q * ldx, d, sub, xf);
#pragma unroll
      for (int i = 0; i < 8 * NM; ++i) xv[i] = (double)xf[i];
    }
    double d3[3];
    {
      const float* const rows[3] = {C32 + (size_t)qb * d, C32 + (size_t)qs * d,
                                    C32 + (size_t)(t_real ? qt : qb) * d};
      rows_dist2<NM, 3>(xv, rows, d, sub, d3);
    }
    int w = qb;
    double dw = d3[0];
    if (d3[1] < dw || (d3[1] == dw && qs < w)) { w = qs; dw = d3[1]; }
    if (t_real && (d3[2] < dw || (d3[2] == dw && qt < w))) { w = qt; dw = d3[2]; }
    bool certified = !t_real;
    if (t_real) {
      double et, dl_t;
      exact_bound(qsb - qm3, cm, qxn, qx2, qamax, gam, pack_rel, et, dl_t);
      certified = 0.5 * (qx2 - dw) - qx2 * 0x1p-23 > (qsb - qm3) + et &&
                  dl_t >= 2.0 * qamax;
    }
    if (!certified) {
      if (sub == 0) atomicAdd(&cnt[2], 1ull);
      const int w0 = w;
      const double r0 = sqrt(dw);
      bool done = false;
      const int32_t* ni = nbr_idx + (size_t)w0 * L;
      const float* nd = nbr_dist + (size_t)w0 * L;
      const float* cw0 = C32 + (size_t)w0 * d;
      int evals = 0;
      for (int jj = 0; jj < L; jj += kElkanStep) {
        const double lim = (r0 + sqrt(dw)) * (1.0 + 0x1p-40);
        if ((double)nd[jj] > lim) {
          done = true;
          break;
        }
        int jv[kElkanStep];
        const float* cp[kElkanStep];
#pragma unroll
        for (int v = 0; v < kElkanStep; ++v) {
          const bool ok = jj + v < L && (double)nd[jj + v] <= lim;
          jv[v] = ok ? ni[jj + v] : -1;
          cp[v] = ok ? C32 + (size_t)jv[v] * d : cw0;
        }
        double dj[kElkanStep];
        rows_dist2<NM, kElkanStep>(xv, cp, d, sub, dj);
        evals += kElkanStep;
#pragma unroll
        for (int v = 0; v < kElkanStep; ++v)
          if (jv[v] >= 0 && (dj[v] < dw || (dj[v] == dw && jv[v] < w))) { w = jv[v]; dw = dj[v]; }
      }
      if (sub == 0) {
        atomicAdd(&cnt[3], (unsigned long long)evals);
        if (!done && L < k) atomicAdd(&cnt[4], 1ull);
      }
      if (!done && L < k) {
        for (int j = 0; j < k; j += 4) {
          const float* cp[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) cp[v] = C32 + (size_t)(j + v < k ? j + v : j) * d;
          double dj[4];
          rows_dist2<NM, 4>(xv, cp, d, sub, dj);
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (j + v < k && (dj[v] < dw || (dj[v] == dw && j + v < w))) { w = j + v; dw = dj[v]; }
        }
      }
    }
    if (sub == 0 && w != qb) {
      labels[q] = w;
      atomicAdd(&cnt[1], 1ull);
    }
  }
  __syncthreads();
  if (threadIdx.x < (nstats < 5 ? 3 : 5) && cnt[threadIdx.x])
    atomicAdd(stats + threadIdx.x, cnt[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// Exact mode staging.  A split's fp32 rows become the 16-bit MFMA copy (fp16 by
// default, saturated at ±65504; or bf16) plus, per point, |x| (fp64 → fp32),
// |x~|^2 (fp64 → fp32) and the rounding error |x - x~| (fp64, rounded UP):
// the certification's inputs.  16 lanes per row, 8 features per lane.
__device__ __forceinline__ uint16_t hbmr_f32_to_f16_sat(float v) {
  const _Float16 h = (_Float16)fminf(fmaxf(v, -65504.f), 65504.f);
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float hbmr_f16_to_f32(uint16_t b) {
  return (float)__builtin_bit_cast(_Float16, b);
}

__global__ __launch_bounds__(256) void kmeans_exact_prep_kernel(
    const float* __restrict__ x, long n, int d, int ldx, int dp, int f16,
    uint16_t* __restrict__ x16, float* __restrict__ xnorm, float* __restrict__ xn2,
    float* __restrict__ xerr) {
  const long row = (long)blockIdx.x * 16 + threadIdx.x / kRefineGroup;
  const int sub = threadIdx.x % kRefineGroup;
  const bool ok = row < n;
  const long r = ok ? row : n - 1;
  double a = 0.0, q = 0.0, e = 0.0;
  for (int i0 = 8 * sub; i0 < dp; i0 += 8 * kRefineGroup) {
    uint16_t hb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j;
      const float v = i < d ? x[r * ldx + i] : 0.f;
      const uint16_t b = f16 ? hbmr_f32_to_f16_sat(v) : hbmr_f32_to_bf16(v);
      const float vt = f16 ? hbmr_f16_to_f32(b) : hbmr_bf16_to_f32(b);
      hb[j] = b;
      a = fma((double)v, (double)v, a);
      q = fma((double)vt, (double)vt, q);
      const double df = (double)v - (double)vt;
      e = fma(df, df, e);
    }
    if (ok) {
      uint4 w;
      w.x = hb[0] | ((uint32_t)hb[1] << 16);
      w.y = hb[2] | ((uint32_t)hb[3] << 16);
      w.z = hb[4] | ((uint32_t)hb[5] << 16);
      w.w = hb[6] | ((uint32_t)hb[7] << 16);
      *reinterpret_cast<uint4*>(x16 + r * dp + i0) = w;
    }
  }
  a = row_sum16(a);
  q = row_sum16(q);
  e = row_sum16(e);
  if (ok && sub == 0) {
    xnorm[r] = (float)sqrt(a);
    xn2[r] = (float)q;
    xerr[r] = __double2float_ru(sqrt(e) * (1.0 + 0x1p-50));
  }
}

// Tiled copy of a 16-bit image [k_pad, dp] (dp = 64 / 128) for the v3 assign:
// tile T (32 rows) holds its 16-byte pieces piece-major, (q, r) at
// T * 32 * dp * 2 + q * 512 + r * 16 bytes (q = piece in the row, r = row).
__global__ __launch_bounds__(256) void kmeans_image16_tiled_kernel(const uint4* __restrict__ c16,
                                                                   int k_pad, int dp,
                                                                   uint4* __restrict__ c16t) {
  const long P = (long)blockIdx.x * 256 + threadIdx.x;
  const int cpr = dp / 8;
  if (P >= (long)k_pad * cpr) return;
  const long T = P / (32 * cpr);
  const int w = (int)(P % (32 * cpr));
  const int q = w / 32, r = w % 32;
  c16t[P] = c16[(T * 32 + r) * cpr + q];
}

// The 16-bit image of the fp32 centroids for exact mode (fp16 by default):
// c16 [k_pad, dp], chalf = -|c~|^2/2 (fp32, summed as kmeans_update sums the
// bf16 image's), |c| and |c - c~| (fp64, rounded up) and their maxima (as
// float bits: non-negative floats order as unsigned).  One workgroup per row.
__global__ __launch_bounds__(128) void kmeans_image16_kernel(
    const float* __restrict__ cen, int k, int d, int dp, int f16, uint16_t* __restrict__ c16,
    float* __restrict__ chalf, float* __restrict__ cnorm, float* __restrict__ cerr,
    unsigned* __restrict__ maxbits) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ float red[128];
  __shared__ double red64[2][128];
  float nrm = 0.f;
  double a = 0.0, e = 0.0;
  for (int i = tid; i < dp; i += 128) {
    const float v = (j < k && i < d) ? cen[(size_t)j * d + i] : 0.f;
    const uint16_t b = f16 ? hbmr_f32_to_f16_sat(v) : hbmr_f32_to_bf16(v);
    const float vt = f16 ? hbmr_f16_to_f32(b) : hbmr_bf16_to_f32(b);
    c16[(size_t)j * dp + i] = b;
    nrm += vt * vt;
    a = fma((double)v, (double)v, a);
    const double df = (double)v - (double)vt;
    e = fma(df, df, e);
  }
  red[tid] = nrm;
  red64[0][tid] = a;
  red64[1][tid] = e;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (tid < s) {
      red[tid] += red[tid + s];
      red64[0][tid] += red64[0][tid + s];
      red64[1][tid] += red64[1][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0) {
    chalf[j] = j < k ? -0.5f * red[0] : -1.0e30f;
    if (j < k) {
      const float cn = __double2float_ru(sqrt(red64[0][0]) * (1.0 + 0x1p-50));
      const float ce = __double2float_ru(sqrt(red64[1][0]) * (1.0 + 0x1p-50));
      cnorm[j] = cn;
      cerr[j] = ce;
      atomicMax(maxbits + 0, __float_as_uint(cn));
      atomicMax(maxbits + 1, __float_as_uint(ce));
    }
  }
}

// ---------------------------------------------------------------------------
// Refine v3: the certification as a compacted queue pipeline over a BATCH of
// splits.  v2 certifies each point in the thread that scanned it and then walks
// the wave's flagged points four at a time, each round a dependent row-load
// chain, so a wave waits out several L2/HBM round trips serially.  v3 splits
// the work by what each step needs:
//   q1 (per split, right after its top-3 assign): step 1 (margins vs bounds)
//       streams every point; the flagged ones are compacted into queue Q1;
//   q2 (once per batch): step 2 over Q1 on a persistent grid, 8 lanes per entry
//       (16 features each), 8 entries per wave, the next entries prefetched and
//       every row load issued before the first FMA; winners that the top three
//       cannot certify go to queue Q2;
//   q3 (once per batch): the Elkan neighbour scan over Q2 (≈1 % of points with
//       fp16 operands).
// The batch pays q2/q3's latency chains once instead of once per split.  Same
// bounds and ties as v1/v2; the fp64 distance sums differ only in summation
// order (labels can differ only on exact fp64 ties).
// Both queues are sharded 8 ways (by blockIdx % 8, i.e. per XCD under the
// round-robin placement): one counter word takes ≈88 atomics/µs
// (MI355X_MICROARCH.md, dequeue row).  Shard j holds its entries contiguously
// at [j * cap, j * cap + count_j).
struct ExactQ1 {
  uint32_t row, split;
  int32_t b, s, t;
  float sb, m3, x2, xn, xe, pad0, pad1;
};
struct ExactQ2 {
  uint32_t row, split;
  int32_t w, pad;
  double dw;
};
static_assert(sizeof(ExactQ1) == 48 && sizeof(ExactQ2) == 24, "queue entry layout");

constexpr int kQShards = 8;
constexpr int kQ1Per = 4;            // points per thread in the step-1 scan
constexpr int kQ2Lanes = 8;          // lanes per Q1 entry in step 2
constexpr int kQ2Per = HBMR_WAVE / kQ2Lanes;
constexpr int kRefineGrid = 2048;    // persistent grid of q2 and q3
// HBMR_REFINE_GRID (read once) overrides it, for tuning runs
inline long refine_grid() {
  static const long g = [] {
    const char* e = getenv("HBMR_REFINE_GRID");
    const long v = e ? atol(e) : 0;
    return v > 0 ? v : (long)kRefineGrid;
  }();
  return g;
}
// workspace header: Q1 / Q2 shard counts (8 + 8 u32) and the sharded stats
// (8 shards x 4 u64 at kStatsOff): one word per stat took every block's
// atomic at the kernels' tails; kmeans_refine_stats_kernel folds them
constexpr int kStatsOff = 64;
constexpr int kRefineHdr = 512;
constexpr int kHdrClear = kStatsOff + kQShards * 4 * 8;

struct RefineTable {                 // the batch's splits, by value
  int nsplit;
  const float* x32[kMaxGroup];
  int32_t* labels[kMaxGroup];
};

__host__ __device__ inline long ceil_div(long a, long b) { return (a + b - 1) / b; }

struct RefineLayout {
  long cap1, cap2;                   // entries per shard
  unsigned g2;
  size_t off1, off2, bytes;
};
inline RefineLayout refine_layout(int nsplit, const long* ns) {
  RefineLayout L;
  long total = 0, cap1 = 0, nb_fused = 0;
  for (int i = 0; i < nsplit; ++i) {
    total += ns[i];
    cap1 += ceil_div(ceil_div(ns[i], 256 * kQ1Per), kQShards) * 256 * kQ1Per;
    nb_fused += ceil_div(ns[i], 256);
  }
  // the fused top-3 epilogue appends from 256-point workgroups, shard =
  // blockIdx % kQShards: at most ceil(nb / kQShards) workgroups per shard
  L.cap1 = std::max<long>(cap1, ceil_div(nb_fused, kQShards) * 256);
  L.g2 = (unsigned)std::max<long>(1, std::min<long>(refine_grid(), ceil_div(total, 4 * kQ2Per)));
  const long per_iter = (long)L.g2 * 4 * kQ2Per;           // Q1 entries per grid iteration
  L.cap2 = ceil_div(L.g2, kQShards) * 4 * kQ2Per * std::max<long>(1, ceil_div(total, per_iter));
  L.off1 = kRefineHdr;
  L.off2 = L.off1 + ((kQShards * (size_t)L.cap1 * sizeof(ExactQ1) + 255) & ~(size_t)255);
  L.bytes = L.off2 + kQShards * (size_t)L.cap2 * sizeof(ExactQ2);
  return L;
}

// item i of the flattened sharded queue → its slot (counts of the 8 shards)
__device__ __forceinline__ long shard_slot(const uint32_t (&c)[kQShards], long cap, uint32_t i) {
  uint32_t acc = 0;
  long slot = 0;
#pragma unroll
  for (int j = 0; j < kQShards; ++j) {
    if (i >= acc && i < acc + c[j]) slot = (long)j * cap + (i - acc);
    acc += c[j];
  }
  return slot;
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Step 1's certification of one point (its kernel top-3 in e, best - second
// margin m2, cnb / ceb = |c_b|, |c_b - c~_b|): true = not certified, the point
// goes to step 2.  Shared by the step-1 scan and the fused top-3 epilogue.
__device__ __forceinline__ bool q1_flagged(const ExactQ1& e, float m2, float cnb, float ceb, int k,
                                           double gam, double cm, double cem, double pack_rel,
                                           const float* __restrict__ cnorm,
                                           const float* __restrict__ cerr,
                                           const float* __restrict__ dcc) {
  const double inflate = 1.0 + 0x1p-20;
  const double xn = ((double)e.xn + (double)e.xe) * inflate;
  const double x2 = (double)e.x2;
  const double sb = e.sb;
  const double mm = m2;
  const double amax = ((double)e.xe + cem) * inflate;
  double eb, es, dl_b, dl_s;
  exact_bound(sb, ((double)cnb + (double)ceb) * inflate, xn, x2,
              ((double)e.xe + (double)ceb) * inflate, gam, pack_rel, eb, dl_b);
  exact_bound(sb - mm, cm, xn, x2, amax, gam, pack_rel, es, dl_s);
  bool flag = !(mm > eb + es && dl_s >= 2.0 * amax);
  const int b = e.b, sc = e.s, t = e.t;
  if (flag && dcc != nullptr && t < k && t != b) {
    // Pair rule: D_s - D_b >= (D~_s - D~_b) - 2|c~_b - c~_s| e_x
    //   - 2 sqrt(D~_s) e_s - 2 sqrt(D~_b) e_b - (e_x + e_b)^2
    // (x - c_j = (x~ - c~_j) + (dx - dc_j); the dx terms of b and s
    // cancel up to (c~_b - c~_s).dx), with |c~_b - c~_s| <= |c_b - c_s|
    // + e_b + e_s — tighter than E_b + E_s where the two centroids are
    // close and the point is not.  Everything ranked at or below t is
    // beaten by the generic rule at t (margin b-t against E_b + E_max(t)).
    const double ex = (double)e.xe * inflate;
    const double ebb = (double)ceb * inflate;
    const double ess = (double)cerr[sc] * inflate;
    const double dbs = ((double)dcc[(size_t)b * k + sc] + (double)ceb + (double)cerr[sc]) *
                       inflate;
    double eap_b, rb, eap_s, rs;
    score_err(sb, ((double)cnb + (double)ceb) * inflate, xn, x2, gam, pack_rel, eap_b, rb);
    score_err(sb - mm, ((double)cnorm[sc] + (double)cerr[sc]) * inflate, xn, x2, gam,
              pack_rel, eap_s, rs);
    const double ep = dbs * ex + rs * ess + rb * ebb + 0.5 * (ex + ebb) * (ex + ebb) +
                      eap_b + eap_s;
    double et, dl_t;
    const double m3 = e.m3;
    exact_bound(sb - m3, cm, xn, x2, amax, gam, pack_rel, et, dl_t);
    if (mm > ep && m3 > eb + et && dl_t >= 2.0 * amax) flag = false;
  }
  return flag;
}

// Step 1 over one block of 256 * kQ1Per points of split sidx (block index blk
// within the split); cand / margin second rows at stride cs.
__device__ __forceinline__ void refine_q1_block(
    long n, int sidx, long blk, int d, int k, const float* __restrict__ xnorm,
    const float* __restrict__ xbn2, const float* __restrict__ xerr,
    const float* __restrict__ cnorm, const float* __restrict__ cmax,
    const float* __restrict__ cerr, const float* __restrict__ cerrmax, double pack_rel,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ cand,
    const float* __restrict__ score, const float* __restrict__ margin, long cs,
    uint32_t* __restrict__ qcount, ExactQ1* __restrict__ q1, long cap1,
    unsigned long long* __restrict__ stats, const float* __restrict__ dcc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int shard = blockIdx.x % kQShards;
  __shared__ uint32_t wcnt[4][kQ1Per];
  __shared__ uint32_t base_s;
  const double inflate = 1.0 + 0x1p-20;
  const double gam = (double)(d + 2) * 0x1p-23 * 1.01;
  const double cem = (double)cerrmax[0] * inflate;
  const double cm = (double)cmax[0] * inflate + cem;
  // every load of the four points first, then the dependent gathers, then math
  ExactQ1 e[kQ1Per];
  bool in[kQ1Per];
  float m2[kQ1Per];
#pragma unroll
  for (int i = 0; i < kQ1Per; ++i) {
    const long p = blk * (256 * kQ1Per) + i * 256 + tid;
    in[i] = p < n;
    const long q = in[i] ? p : n - 1;
    e[i].row = (uint32_t)q;
    e[i].split = (uint32_t)sidx;
    e[i].b = labels[q];
    e[i].s = cand[q];
    e[i].t = cand[cs + q];
    e[i].sb = score[q];
    m2[i] = margin[q];
    e[i].m3 = margin[cs + q];
    e[i].x2 = xbn2[q];
    e[i].xn = xnorm[q];
    e[i].xe = xerr[q];
  }
  float cnb[kQ1Per], ceb[kQ1Per];
#pragma unroll
  for (int i = 0; i < kQ1Per; ++i) {
    cnb[i] = cnorm[e[i].b];
    ceb[i] = cerr[e[i].b];
  }
  bool flag[kQ1Per];
  uint32_t rank[kQ1Per];
#pragma unroll
  for (int i = 0; i < kQ1Per; ++i) {
    flag[i] = in[i] && e[i].s < k &&
              q1_flagged(e[i], m2[i], cnb[i], ceb[i], k, gam, cm, cem, pack_rel, cnorm, cerr, dcc);
    const unsigned long long m = __ballot(flag[i]);
    rank[i] = lane_rank(m);
    if (lane == 0) wcnt[wave][i] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int i = 0; i < kQ1Per; ++i) {
        const uint32_t c = wcnt[w][i];
        wcnt[w][i] = tot;
        tot += c;
      }
    base_s = tot ? atomicAdd(qcount + shard, tot) : 0u;
    if (tot) atomicAdd(stats + 4 * shard, (unsigned long long)tot);
  }
  __syncthreads();
  ExactQ1* out = q1 + (long)shard * cap1 + base_s;
#pragma unroll
  for (int i = 0; i < kQ1Per; ++i)
    if (flag[i]) out[wcnt[wave][i] + rank[i]] = e[i];
}

__global__ __launch_bounds__(256) void kmeans_refine_q1_kernel(
    long n, int sidx, int d, int k, const float* __restrict__ xnorm,
    const float* __restrict__ xbn2, const float* __restrict__ xerr,
    const float* __restrict__ cnorm, const float* __restrict__ cmax,
    const float* __restrict__ cerr, const float* __restrict__ cerrmax, double pack_rel,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ cand,
    const float* __restrict__ score, const float* __restrict__ margin,
    uint32_t* __restrict__ qcount, ExactQ1* __restrict__ q1, long cap1,
    unsigned long long* __restrict__ stats, const float* __restrict__ dcc) {
  refine_q1_block(n, sidx, blockIdx.x, d, k, xnorm, xbn2, xerr, cnorm, cmax, cerr, cerrmax,
                  pack_rel, labels, cand, score, margin, n, qcount, q1, cap1, stats, dcc);
}

// the splits of a batch in one launch (after the grouped top-3 assign): the
// batch arrays hold split s at offset off[s], second rows at stride total
struct Q1Table {
  int nsplit;
  long total;
  long n[kMaxGroup];
  long off[kMaxGroup];
  long blk[kMaxGroup + 1];
  const float* xnorm[kMaxGroup];
  const float* xbn2[kMaxGroup];
  const float* xerr[kMaxGroup];
};

__global__ __launch_bounds__(256) void kmeans_refine_q1_grouped_kernel(
    const Q1Table tbl, int d, int k, const float* __restrict__ cnorm,
    const float* __restrict__ cmax, const float* __restrict__ cerr,
    const float* __restrict__ cerrmax, double pack_rel, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ cand, const float* __restrict__ score,
    const float* __restrict__ margin, uint32_t* __restrict__ qcount, ExactQ1* __restrict__ q1,
    long cap1, unsigned long long* __restrict__ stats, const float* __restrict__ dcc) {
  const long b = blockIdx.x;
  int lo = 0, hi = tbl.nsplit;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tbl.blk[mid] <= b) lo = mid; else hi = mid;
  }
  const int s = __builtin_amdgcn_readfirstlane(lo);
  const long o = tbl.off[s];
  refine_q1_block(tbl.n[s], s, b - tbl.blk[s], d, k, tbl.xnorm[s], tbl.xbn2[s], tbl.xerr[s],
                  cnorm, cmax, cerr, cerrmax, pack_rel, labels + o, cand + o, score + o,
                  margin + o, tbl.total, qcount, q1, cap1, stats, dcc);
}

// ---------------------------------------------------------------------------
// Top-3 assign with step 1 fused into its epilogue (HBMR_EXACT_FUSED_Q1, the
// default): the lane that finishes a point holds its kernel top 3 and
// margins in registers, certifies it there (q1_flagged) and appends only an
// uncertain point to the step-2 queue — one atomic per workgroup — so the
// candidate / score / margin arrays (20 B per point written, then read back
// with the labels by the step-1 scan) are never materialised.
struct FusedQ1Fin {
  const float* xnorm;
  const float* xbn2;
  const float* xerr;
  int sidx;
  int k;
  double gam, pack_rel;
  const float* cmax_p;       // max |c_j| and max |c_j - c~_j| (device, 1 float each)
  const float* cerrmax_p;
  const float* cnorm;
  const float* cerr;
  const float* dcc;
  uint32_t* qcount;
  ExactQ1* q1;
  long cap1;
  unsigned long long* stats;

  template <class AM, int PB>
  __device__ __forceinline__ void operator()(const AM (&am)[PB], int h, long p0, int col, long n,
                                             int32_t* __restrict__ labels) const {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint32_t fq_cnt[4 * PB];
    __shared__ uint32_t fq_base;
    const int shard = blockIdx.x % kQShards;
    const double inflate = 1.0 + 0x1p-20;
    const double cem = (double)cerrmax_p[0] * inflate;
    const double cm = (double)cmax_p[0] * inflate + cem;
    ExactQ1 e[PB];
    bool flag[PB];
    uint32_t rank[PB];
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      float v[3];
      int c[3];
      am[pb].top3(v[0], v[1], v[2]);
#pragma unroll
      for (int i = 0; i < 3; ++i) c[i] = am[pb].cluster(v[i], h);
      float ov[3];
      int oc[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ov[i] = __shfl_xor(v[i], 32);
        oc[i] = __shfl_xor(c[i], 32);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) insert3(v, c, ov[i], oc[i]);
      if constexpr (HasTracks<AM>::value) {
        if (((c[0] ^ c[1]) & AM::TMASK) == 0) {
          v[2] = v[0];
          c[2] = c[0];
        }
      }
      const long p = p0 + pb * 32 + col;
      flag[pb] = false;
      if (h == 0 && p < n) {
        labels[p] = c[0];
        const float bs = am[pb].score(v[0]);
        const float m2 = bs - am[pb].score(v[1]);
        ExactQ1& q = e[pb];
        q.row = (uint32_t)p;
        q.split = (uint32_t)sidx;
        q.b = c[0];
        q.s = c[1];
        q.t = c[2];
        q.sb = bs;
        q.m3 = bs - am[pb].score(v[2]);
        q.x2 = xbn2[p];
        q.xn = xnorm[p];
        q.xe = xerr[p];
        q.pad0 = q.pad1 = 0.f;
        flag[pb] = q.s < k && q1_flagged(q, m2, cnorm[q.b], cerr[q.b], k, gam, cm, cem,
                                         pack_rel, cnorm, cerr, dcc);
      }
      const unsigned long long m = __ballot(flag[pb]);
      rank[pb] = lane_rank(m);
      if (lane == 0) fq_cnt[wave * PB + pb] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t tot = 0;
#pragma unroll
      for (int i = 0; i < 4 * PB; ++i) {
        const uint32_t c = fq_cnt[i];
        fq_cnt[i] = tot;
        tot += c;
      }
      fq_base = tot ? atomicAdd(qcount + shard, tot) : 0u;
      if (tot) atomicAdd(stats + 4 * shard, (unsigned long long)tot);
    }
    __syncthreads();
    ExactQ1* out = q1 + (long)shard * cap1 + fq_base;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
      if (flag[pb]) out[fq_cnt[wave * PB + pb] + rank[pb]] = e[pb];
  }
};

// ---------------------------------------------------------------------------
// v3 of the fused exact assign (PB = 2 point blocks per wave, D <= 128).  v2
// issues ~100 VALU and ~48 SALU per 32-cluster tile and wave beside its 16
// MFMAs (PMC: MFMA pipes 51 % busy, 40 % of wave cycles issue-stalled;
// profiles/r04_exact_pipe_ab.json).  v3 trims that stream and the registers:
//  * the 16 (tile, register) codes of a tile are made once, in SGPRs, and
//    shared by both point blocks (v2 re-derived them per block: 39 s_add);
//  * -|c|^2/2 is read from LDS straight into the accumulators (v2 kept a bias
//    register set and copied it: 16 v_mov per tile);
//  * the centroid image is tiled (piece-major, hbmr_kmeans_image16_tiled): a
//    tile's DMA is lane-linear on both sides and a lane's k-step s is at a
//    fixed immediate offset (s * 1 KiB) from one base register — no
//    XOR-swizzle offsets (8 VGPRs) or per-read address VALU; 16 lanes of one
//    k-step read 256 contiguous bytes (conflict-free).
// Measured negatives, removed in round 6 (profiles/r05_exact_v3_ab.json):
// just-in-time A reads at 4 waves per SIMD, s_setprio over the MFMA chain,
// epilogue pipelining (two accumulator sets), a half-tile pipeline, two tiles
// per barrier step, a 6-slot ring and DMA reordering; so was v4, which keeps
// the centroids stationary in registers and streams the points
// (profiles/r06_exact_v4_ab.json): its per-block cross-wave merge makes it
// VALU-issue bound; and v5, which takes the barrier out by giving each wave a
// private one-tile slot refilled chunk by chunk (profiles/r06_exact_v5_ab.json):
// 4x the L2->LDS bytes and DMA issues cost more than the barrier (+13 %).
// tiled image: tile t is 32 * D * 2 contiguous bytes already in LDS order
template <int D>
__device__ __forceinline__ void stage_tile32t(char* buf, const __bf16* __restrict__ Ct,
                                              const float* __restrict__ chalf, int tile, int wave,
                                              int lane) {
  using V = AssignV2<D>;
  // wave-uniform bases + a 32-bit lane offset: the saddr form of the DMA (one
  // VGPR of address, not a 64-bit pair per instruction)
  const uint32_t loff = (uint32_t)lane * 16u;
#pragma unroll
  for (int i = 0; i < V::P; ++i) {
    const int base = (i * V::WAVES + wave) * HBMR_WAVE;
    const char* g = reinterpret_cast<const char*>(Ct) + (size_t)tile * V::TILE_BYTES +
                    (size_t)base * 16;
    __builtin_amdgcn_global_load_lds((const void*)(g + loff), (void*)(buf + base * 16), 16, 0, 0);
  }
  if (wave == 0 && lane < 32) {
    const char* g = reinterpret_cast<const char*>(chalf + (size_t)tile * 32);
    __builtin_amdgcn_global_load_lds((const void*)(g + loff / 4u), (void*)(buf + V::TILE_BYTES),
                                     4, 0, 0);
  }
}

// (tile, register) codes of tile t in SGPRs (see PackedArgMax)
__device__ __forceinline__ void tile_codes(uint32_t top, int t, uint32_t (&code)[16]) {
  const uint32_t base = top - ((uint32_t)t << 4);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    code[r] = base | (15u - r);
    asm("" : "+s"(code[r]));
  }
}

// PackedTop2x8::update with precomputed codes (pair insertion, NT tracks)
__device__ __forceinline__ void top2_insert(PackedTop2x8& am, const f32x16& acc,
                                            const uint32_t (&code)[16], uint32_t vmask) {
  constexpr int NT = PackedTop2x8::NT;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if ((r / NT) % 2) continue;
    const float u = __uint_as_float((__float_as_uint(acc[r]) & vmask) | code[r]);
    const float v = __uint_as_float((__float_as_uint(acc[r + NT]) & vmask) | code[r + NT]);
    const float m = vmed3(am.tb[r % NT], u, v);
    am.ts[r % NT] = vmax3(m, am.ts[r % NT], am.ts[r % NT]);
    am.tb[r % NT] = vmax3(am.tb[r % NT], u, v);
  }
}

template <int D, bool F16>
__device__ __forceinline__ void assign_tile_v3(const __bf16* __restrict__ X, long n,
                                               const __bf16* __restrict__ Ct,
                                               const float* __restrict__ chalf, int ntiles,
                                               int32_t* __restrict__ labels, long blk, char* smem,
                                               const FusedQ1Fin& fin) {
  static_assert(D <= 128, "v3 keeps two 32-point blocks of D <= 128 in registers");
  constexpr int PB = 2, NS = 4;
  using V = AssignV2<D, NS>;
  static_assert(V::WAVES == 4, "v3: 4 waves per workgroup");
  constexpr int KS = V::KS;
  // the bias sits right after the tile's rows whatever D is
  static_assert(V::TILE_BYTES == 32 * D * 2, "tile layout");
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / HBMR_WAVE);
  const int lane = tid & (HBMR_WAVE - 1);
  const int h = lane >> 5;
  const int col = lane & 31;
  const long p0 = blk * (V::WAVES * PB * 32) + (long)wave * PB * 32;
  // a tile buffer + rowoff: this lane's k-step s at s KiB (tiled layout)
  const int rowoff = h * 512 + col * 16;
  auto frag = [&](const char* row, int s) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8*>(row + s * 1024);
  };
  auto bias = [&](const char* buf, f32x16& acc) __attribute__((always_inline)) {
    const float* ch = reinterpret_cast<const float*>(buf + V::TILE_BYTES);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(ch + 8 * g + 4 * h);
      acc[4 * g + 0] = v[0];
      acc[4 * g + 1] = v[1];
      acc[4 * g + 2] = v[2];
      acc[4 * g + 3] = v[3];
    }
  };

#pragma unroll
  for (int i = 0; i < NS; ++i)
    if (i < ntiles) stage_tile32t<D>(smem + i * V::BUF, Ct, chalf, i, wave, lane);

  bf16x8 bfrag[PB][KS];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    long p = p0 + pb * 32 + col;
    if (p >= n) p = n - 1;
    const uint4* row = reinterpret_cast<const uint4*>(X + p * D);
#pragma unroll
    for (int s = 0; s < KS; ++s) bfrag[pb][s] = __builtin_bit_cast(bf16x8, row[2 * s + h]);
  }
  PackedTop2x8 am[PB];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) am[pb].init(ntiles);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int pb = 0; pb < PB; ++pb)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(bfrag[pb][s]));
  __syncthreads();
  const bool w0 = wave == 0;
  const uint32_t top = am[0].top;
  const uint32_t vmask = am[0].vmask;   // one copy for both blocks

  // v2's ring (tile t+1's A read during tile t), codes shared, bias into acc
  bf16x8 a[KS];
  f32x16 bz;
  {
    const char* row = smem + rowoff;
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = frag(row, s);
    bias(smem, bz);
  }
  int slot = 0;
  for (int t = 0; t < ntiles; ++t) {
    wait_tile_dmas<V::P, NS - 2>(max(0, min(NS - 2, ntiles - 2 - t)), w0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    char* rbuf = smem + slot * V::BUF;
    if (t + NS < ntiles) stage_tile32t<D>(rbuf, Ct, chalf, t + NS, wave, lane);
    slot = slot + 1 == NS ? 0 : slot + 1;
    const char* nbuf = smem + slot * V::BUF;
    const char* nrow = nbuf + rowoff;
    f32x16 acc[PB];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int pb = 0; pb < PB; ++pb)
        acc[pb] = mfma32x32x16<F16>(a[s], bfrag[pb][s], s == 0 ? bz : acc[pb]);
      a[s] = frag(nrow, s);
    }
    uint32_t code[16];
    tile_codes(top, t, code);
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) top2_insert(am[pb], acc[pb], code, vmask);
    bias(nbuf, bz);
  }
  fin(am, h, p0, col, n, labels);
}

struct TopQ1Table {       // the batch's splits, by value (X, per-point norms)
  int nsplit;
  const __bf16* X[kMaxGroup];
  const float* xnorm[kMaxGroup];
  const float* xbn2[kMaxGroup];
  const float* xerr[kMaxGroup];
  long off[kMaxGroup + 1];
  long blk[kMaxGroup + 1];
};

template <int D, bool F16>
__global__ __launch_bounds__(AssignV2<D>::THREADS, HBMR_EXACT_MINB) void
kmeans_assign_top3_q1_grouped_kernel(const TopQ1Table tbl, const __bf16* __restrict__ C,
                                     const float* __restrict__ chalf, int ntiles,
                                     int32_t* __restrict__ labels, FusedQ1Fin fin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long b = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  int lo = 0, hi = tbl.nsplit;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tbl.blk[mid] <= b) lo = mid; else hi = mid;
  }
  const int s = __builtin_amdgcn_readfirstlane(lo);
  const long o = tbl.off[s];
  fin.xnorm = tbl.xnorm[s];
  fin.xbn2 = tbl.xbn2[s];
  fin.xerr = tbl.xerr[s];
  fin.sidx = s;
  assign_tile_v2<D, 2, true, F16, false, FusedQ1Fin>(
      tbl.X[s], tbl.off[s + 1] - o, C, chalf,
                                                     ntiles, labels + o, nullptr, b - tbl.blk[s],
                                                     smem, nullptr, nullptr, -1, &fin);
}

// v3 (see assign_tile_v3): HBMR_EXACT_MINB workgroups of 4 waves per CU
template <int D, bool F16>
__global__ __launch_bounds__(256, HBMR_EXACT_MINB) void kmeans_assign_top3_q1_v3_kernel(
    const TopQ1Table tbl, const __bf16* __restrict__ Ct, const float* __restrict__ chalf,
    int ntiles, int32_t* __restrict__ labels, FusedQ1Fin fin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long b = hbmr_xcd_remap(blockIdx.x, gridDim.x);
  int lo = 0, hi = tbl.nsplit;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tbl.blk[mid] <= b) lo = mid; else hi = mid;
  }
  const int s = __builtin_amdgcn_readfirstlane(lo);
  const long o = tbl.off[s];
  fin.xnorm = tbl.xnorm[s];
  fin.xbn2 = tbl.xbn2[s];
  fin.xerr = tbl.xerr[s];
  fin.sidx = s;
  assign_tile_v3<D, F16>(tbl.X[s], tbl.off[s + 1] - o, Ct, chalf, ntiles, labels + o,
                         b - tbl.blk[s], smem, fin);
}

// 16 features of a row per lane of an 8-lane group: 128m + 32h + 4sub + (0..3)
// (0 past d; d % 4 == 0): each float4 load of the group reads 128 contiguous
// bytes of the row
template <int NM>
__device__ __forceinline__ void load_row16(const float* __restrict__ r, int d, int sub,
                                           float (&v)[16 * NM]) {
  // branch-free: every load is issued (address clamped into the row) and the
  // features past d are zeroed by a select, so all of a round's loads stay in
  // flight together (a guarded load made hipcc wait on each one in turn)
#pragma unroll
  for (int m = 0; m < NM; ++m) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int b = 128 * m + 32 * h + 4 * sub;
      const bool ok = b < d;
      const float4 a = *reinterpret_cast<const float4*>(r + (ok ? b : 0));
      float* o = v + 16 * m + 4 * h;
      o[0] = ok ? a.x : 0.f; o[1] = ok ? a.y : 0.f; o[2] = ok ? a.z : 0.f; o[3] = ok ? a.w : 0.f;
    }
  }
}

__device__ __forceinline__ float row_sum8f(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  return v;
}

__device__ __forceinline__ double row_sum8(double v) {
  v += dpp_f64<0xB1>(v);   // xor 1
  v += dpp_f64<0x4E>(v);   // xor 2
  v += dpp_f64<0x141>(v);  // row_half_mirror: the other quad of the 8-lane group
  return v;
}

template <int NM>
__global__ __launch_bounds__(256) void kmeans_refine_q2_kernel(
    const RefineTable tbl, int d, int ldx, const float* __restrict__ C32, int k,
    const float* __restrict__ cmax, const float* __restrict__ cerrmax, double pack_rel,
    const uint32_t* __restrict__ qcount, const ExactQ1* __restrict__ q1, long cap1,
    uint32_t* __restrict__ q2count, ExactQ2* __restrict__ q2, long cap2,
    unsigned long long* __restrict__ sstats) {
  // Q2 entries are staged in LDS and written out with ONE global atomic per
  // block (at the end, or when the buffer nears full): an atomic-with-return
  // per wave and round on the 8 shard counters, whose latency every spilling
  // wave waited out, was half of this kernel's time (diagnostic variant
  // without it: refine 1.71 -> 0.82 ms per 12.5M points)
  constexpr uint32_t kPerBlk = 4 * kQ2Per;        // entries per block round
  constexpr uint32_t kBuf = 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = lane / kQ2Lanes, sub = lane % kQ2Lanes;
  __shared__ ExactQ2 sbuf[kBuf];
  __shared__ uint32_t sn, sbase;
  __shared__ unsigned long long cnt[2];
  if (tid < 2) cnt[tid] = 0;
  if (tid == 0) sn = 0;
  __syncthreads();
  const double inflate = 1.0 + 0x1p-20;
  const double gam = (double)(d + 2) * 0x1p-23 * 1.01;
  const double cem = (double)cerrmax[0] * inflate;
  const double cm = (double)cmax[0] * inflate + cem;
  uint32_t c1[kQShards];
  uint32_t total = 0;
#pragma unroll
  for (int j = 0; j < kQShards; ++j) {
    c1[j] = qcount[j];
    total += c1[j];
  }
  const int shard = blockIdx.x % kQShards;
  const uint32_t stride = gridDim.x * kPerBlk;
  const uint32_t off = wave * kQ2Per + grp;
  auto flush = [&]() {            // block-uniform call sites only
    if (tid == 0) {
      sbase = atomicAdd(q2count + shard, sn);
      cnt[1] += sn;
    }
    __syncthreads();
    const uint32_t m = sn;
    for (uint32_t i = tid; i < m; i += 256) q2[(long)shard * cap2 + sbase + i] = sbuf[i];
    __syncthreads();
    if (tid == 0) sn = 0;
    __syncthreads();
  };
  uint32_t bb = blockIdx.x * kPerBlk;
  ExactQ1 e;
  if (bb < total) e = q1[shard_slot(c1, cap1, min(bb + off, total - 1))];
  for (; bb < total; bb += stride) {             // same trip count in every wave
    const ExactQ1 q = e;
    const bool have = bb + off < total;
    // prefetch the next round's entry while this round's rows are in flight
    const uint32_t nb = bb + stride;
    if (nb < total) e = q1[shard_slot(c1, cap1, min(nb + off, total - 1))];
    const bool t_real = q.t < k;
    const float* xr = tbl.x32[q.split] + (size_t)q.row * ldx;
    float xf[16 * NM], c0[16 * NM], c1r[16 * NM], c2[16 * NM];
    load_row16<NM>(xr, d, sub, xf);
    load_row16<NM>(C32 + (size_t)q.b * d, d, sub, c0);
    load_row16<NM>(C32 + (size_t)q.s * d, d, sub, c1r);
    load_row16<NM>(C32 + (size_t)(t_real ? q.t : q.b) * d, d, sub, c2);
    // fp32 distances (a third of the fp64 form's VALU work, which bound this
    // kernel): every term goes through at most 16*NM + 3 roundings (lane fma
    // chain + the 8-lane tree), so |D^ - D| <= rel * D + abs_eps; the winner is
    // decided only where the three bands do not overlap, else the point goes
    // to the neighbour scan, which restarts from w's exact fp64 distance
    float f0 = 0.f, f1 = 0.f, f2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16 * NM; ++i) {
      const float e0 = xf[i] - c0[i], e1 = xf[i] - c1r[i], e2 = xf[i] - c2[i];
      f0 = fmaf(e0, e0, f0);
      f1 = fmaf(e1, e1, f1);
      f2 = fmaf(e2, e2, f2);
    }
    f0 = row_sum8f(f0);
    f1 = row_sum8f(f1);
    f2 = row_sum8f(f2);
    const double rel = (double)(16 * NM + 8) * 0x1p-24 * 1.01, aeps = 0x1p-120;
    int w = q.b;
    double dw = f0;
    if ((double)f1 < dw || ((double)f1 == dw && q.s < w)) { w = q.s; dw = f1; }
    if (t_real && ((double)f2 < dw || ((double)f2 == dw && q.t < w))) { w = q.t; dw = f2; }
    const double whi = dw * (1.0 + rel) + aeps;            // >= D_w
    auto beats = [&](double dj) { return dj * (1.0 - rel) - aeps > whi; };
    bool separated = isfinite(whi) &&
                     (w == q.b || beats(f0)) && (w == q.s || beats(f1)) &&
                     (!t_real || w == q.t || beats(f2));
    dw = whi;
    bool certified = !t_real && separated;
    if (t_real && separated) {
      const double xn = ((double)q.xn + (double)q.xe) * inflate;
      const double x2 = (double)q.x2;
      const double amax = ((double)q.xe + cem) * inflate;
      const double st = (double)q.sb - (double)q.m3;
      double et, dl_t;
      exact_bound(st, cm, xn, x2, amax, gam, pack_rel, et, dl_t);
      certified = 0.5 * (x2 - dw) - x2 * 0x1p-23 > st + et && dl_t >= 2.0 * amax;
    }
    if (have && sub == 0 && certified && w != q.b) {
      tbl.labels[q.split][q.row] = w;
      atomicAdd(&cnt[0], 1ull);
    }
    const bool spill = have && sub == 0 && !certified;
    const unsigned long long m = __ballot(spill);
    if (m) {
      uint32_t b2 = 0;
      if (lane == 0) b2 = atomicAdd(&sn, (uint32_t)__popcll(m));    // LDS
      b2 = __shfl(b2, 0);
      if (spill) {
        ExactQ2 o;
        o.row = q.row;
        o.split = q.split;
        o.w = w;
        o.pad = 0;
        o.dw = dw;
        sbuf[b2 + lane_rank(m)] = o;
      }
    }
    __syncthreads();
    if (sn > kBuf - kPerBlk) flush();
  }
  __syncthreads();
  if (sn) flush();
  if (tid < 2 && cnt[tid]) atomicAdd(sstats + 4 * shard + 1 + tid, cnt[tid]);
}

template <int NM>
__global__ __launch_bounds__(256) void kmeans_refine_q3_kernel(
    const RefineTable tbl, int d, int ldx, const float* __restrict__ C32, int k,
    const int32_t* __restrict__ nbr_idx, const float* __restrict__ nbr_dist, int L,
    const uint32_t* __restrict__ q2count, const ExactQ2* __restrict__ q2, long cap2,
    unsigned long long* __restrict__ sstats, int nstats) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int grp = lane / kRefineGroup, sub = lane % kRefineGroup;
  __shared__ unsigned long long cnt[3];
  if (tid < 3) cnt[tid] = 0;
  __syncthreads();
  uint32_t c2[kQShards];
  uint32_t total = 0;
#pragma unroll
  for (int j = 0; j < kQShards; ++j) {
    c2[j] = q2count[j];
    total += c2[j];
  }
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t gw = blockIdx.x * 4 + (tid >> 6);
  for (uint32_t base = gw * 4; base < total; base += nwaves * 4) {
    const uint32_t idx = base + grp;
    const bool have = idx < total;
    const ExactQ2 q = q2[shard_slot(c2, cap2, have ? idx : base)];
    int32_t* lab = tbl.labels[q.split];
    const int b0 = lab[q.row];   // the MFMA pick: step 2 left it in place
    double xv[8 * NM];
    {
      float xf[8 * NM];
      load_row8<NM>(tbl.x32[q.split] + (size_t)q.row * ldx, d, sub, xf);
#pragma unroll
      for (int i = 0; i < 8 * NM; ++i) xv[i] = (double)xf[i];
    }
    const int w0 = q.w;
    int w = w0;
    // step 2 hands over its winner with an fp32 distance (an upper bound):
    // the scan starts from w0's exact fp64 distance
    double dw;
    {
      const float* c0p[1] = {C32 + (size_t)w0 * d};
      double d0[1];
      rows_dist2<NM, 1>(xv, c0p, d, sub, d0);
      dw = d0[0];
    }
    const double r0 = sqrt(dw);
    bool done = false;
    const int32_t* ni = nbr_idx + (size_t)w0 * L;
    const float* nd = nbr_dist + (size_t)w0 * L;
    const float* cw0 = C32 + (size_t)w0 * d;
    int evals = 0;
    for (int jj = 0; jj < L; jj += kElkanStep) {
      const double lim = (r0 + sqrt(dw)) * (1.0 + 0x1p-40);
      if ((double)nd[jj] > lim) {
        done = true;
        break;
      }
      int jv[kElkanStep];
      const float* cp[kElkanStep];
#pragma unroll
      for (int v = 0; v < kElkanStep; ++v) {
        const bool ok = jj + v < L && (double)nd[jj + v] <= lim;
        jv[v] = ok ? ni[jj + v] : -1;
        cp[v] = ok ? C32 + (size_t)jv[v] * d : cw0;
      }
      double dj[kElkanStep];
      rows_dist2<NM, kElkanStep>(xv, cp, d, sub, dj);
      evals += kElkanStep;
#pragma unroll
      for (int v = 0; v < kElkanStep; ++v)
        if (jv[v] >= 0 && (dj[v] < dw || (dj[v] == dw && jv[v] < w))) { w = jv[v]; dw = dj[v]; }
    }
    const bool full = !done && L < k;
    if (full) {
      for (int j = 0; j < k; j += 4) {
        const float* cp[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) cp[v] = C32 + (size_t)(j + v < k ? j + v : j) * d;
        double dj[4];
        rows_dist2<NM, 4>(xv, cp, d, sub, dj);
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (j + v < k && (dj[v] < dw || (dj[v] == dw && j + v < w))) { w = j + v; dw = dj[v]; }
      }
    }
    if (have && sub == 0) {
      atomicAdd(&cnt[1], (unsigned long long)evals);
      if (full) atomicAdd(&cnt[2], 1ull);
      if (w != b0) atomicAdd(&cnt[0], 1ull);
      lab[q.row] = w;
    }
  }
  __syncthreads();
  // sharded stats (kmeans_refine_stats_kernel folds them): word 1 of a shard
  // counts relabels; word 3 counts the scan's neighbour distances in shards
  // 0-3 and its full scans in shards 4-7
  const int sh = blockIdx.x % (kQShards / 2);
  if (tid == 0 && cnt[0]) atomicAdd(sstats + 4 * sh + 1, cnt[0]);
  if (tid == 1 && cnt[1]) atomicAdd(sstats + 4 * sh + 3, cnt[1]);
  if (tid == 2 && cnt[2]) atomicAdd(sstats + 4 * (sh + kQShards / 2) + 3, cnt[2]);
}

// stats[0..2] (+3, 4 when nstats >= 5) += the shards of a refine batch
__global__ void kmeans_refine_stats_kernel(const unsigned long long* __restrict__ ss,
                                           unsigned long long* __restrict__ stats, int nstats) {
  const int t = threadIdx.x;
  if (t >= 5 || (t >= 3 && nstats < 5)) return;
  unsigned long long v = 0;
  if (t < 3) {
    for (int j = 0; j < kQShards; ++j) v += ss[4 * j + t];
  } else {
    for (int j = 0; j < kQShards / 2; ++j) v += ss[4 * (j + (t - 3) * (kQShards / 2)) + 3];
  }
  if (v) stats[t] += v;
}

int refine_version() {
  static int v = 0;
  if (!v) {
    const char* e = getenv("HBMR_REFINE");
    v = (e && atoi(e) == 1) ? 1 : 2;
  }
  return v;
}

template <int D, bool F16>
int launch_assign_top3_grouped(int nsplit, const void* const* X, const long* n, const void* C,
                               const float* chalf, int k_pad, int32_t* labels, int32_t* cand,
                               float* scores, float* margin, hipStream_t st) {
  if constexpr (D > 128) {
    return (int)hipErrorNotSupported;      // the caller launches per split
  } else {
    if (nsplit <= 0 || nsplit > kMaxGroup || k_pad % 32) return (int)hipErrorInvalidValue;
    SplitTable t;
    memset(&t, 0, sizeof(t));
    t.nsplit = nsplit;
    constexpr int pts = AssignV2<D>::WAVES * 2 * 32;
    long total = 0, nb = 0;
    for (int i = 0; i < nsplit; ++i) {
      if (n[i] < 0) return (int)hipErrorInvalidValue;
      t.X[i] = reinterpret_cast<const __bf16*>(X[i]);
      t.n[i] = n[i];
      t.off[i] = total;
      t.blk[i] = nb;
      total += n[i];
      nb += (n[i] + pts - 1) / pts;
    }
    t.blk[nsplit] = nb;
    if (nb == 0) return 0;
    if (nb > 0x7fffffffL) return (int)hipErrorInvalidValue;
    static const bool top3 = [] {
      const char* e = getenv("HBMR_EXACT_EPI");
      return e && strcmp(e, "top3") == 0;
    }();
    auto kern = top3 ? kmeans_assign_top3_grouped_v2_kernel<D, 2, F16, true>
                     : kmeans_assign_top3_grouped_v2_kernel<D, 2, F16, false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(AssignV2<D>::THREADS),
                       AssignV2<D>::LDS_BYTES, st, t, reinterpret_cast<const __bf16*>(C), chalf,
                       k_pad / 32, labels, cand, scores, margin, total);
    return (int)hipGetLastError();
  }
}

template <int D, bool F16>
int launch_assign_top3(const void* X, long n, const void* C, const float* chalf, int k_pad,
                       int32_t* labels, int32_t* cand, float* scores, float* margin,
                       hipStream_t st) {
  if (n <= 0) return 0;
  if (k_pad % kCK) return (int)hipErrorInvalidValue;
  if constexpr (D <= 128) {
    if (assign_version(D) == 2) {
      const int pts = AssignV2<D>::WAVES * 2 * 32;
      const long nblk = (n + pts - 1) / pts;
      if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
      // HBMR_EXACT_EPI=top3: the full running top-3 epilogue (PackedTop3)
      static const bool top3 = [] {
        const char* e = getenv("HBMR_EXACT_EPI");
        return e && strcmp(e, "top3") == 0;
      }();
      auto kern = top3 ? kmeans_assign_top3_v2_kernel<D, 2, F16, true>
                       : kmeans_assign_top3_v2_kernel<D, 2, F16, false>;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk),
                         dim3(AssignV2<D>::THREADS), AssignV2<D>::LDS_BYTES, st,
                         reinterpret_cast<const __bf16*>(X), n, reinterpret_cast<const __bf16*>(C),
                         chalf, k_pad / 32, labels, cand, scores, margin);
      return (int)hipGetLastError();
    }
  }
  const long nblk = (n + AssignCfg<D>::PTS - 1) / AssignCfg<D>::PTS;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((kmeans_assign_top3_kernel<D, F16>), dim3((unsigned)nblk), dim3(kThreads),
                     AssignCfg<D>::LDS_BYTES, st, reinterpret_cast<const __bf16*>(X), n,
                     reinterpret_cast<const __bf16*>(C), chalf, k_pad / kCK, labels, cand, scores,
                     margin);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int hbmr_kmeans_assign_bf16(const void* X, long n, int dp, const void* C, const float* chalf,
                            int k_pad, int32_t* labels, float* scores, hipStream_t st) {
  switch (dp) {
    case 64: return launch_assign<64>(X, n, C, chalf, k_pad, labels, scores, st);
    case 128: return launch_assign<128>(X, n, C, chalf, k_pad, labels, scores, st);
    case 256: return launch_assign<256>(X, n, C, chalf, k_pad, labels, scores, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// Workspace of the sorted combiner: hist[k] | offsets[k+1] | cursor[k] | perm[n]
// (u32 each, regions 256-B aligned).
static size_t ws_align(size_t b) { return (b + 255) & ~(size_t)255; }

long hbmr_kmeans_accum_workspace_bytes(long n, int k) {
  return (long)(3 * ws_align(((size_t)k + 1) * 4) + ws_align((size_t)n * 4));
}

}  // extern "C"

template <typename T>
static int accum_impl(const void* X, long n, int dp, const int32_t* labels, int k,
                      long long* sums, long long* counts, int fx_shift, void* ws, long ws_bytes,
                      int mode, hipStream_t st) {
  set_lds_limits();
  const int cus = cu_count();
  const float scale = ldexpf(1.0f, fx_shift);
  if (n <= 0) return 0;
  // mode: 0 = auto, 1 = LDS-privatised (small k / chunked), 2 = sorted
  const bool small = ((size_t)k * AccCfg<128>::RS * 8 + (size_t)k * 4) <= 76 * 1024 && dp <= 128;
  const bool sorted = mode == 2 || (mode == 0 && !small && ws != nullptr &&
                                    ws_bytes >= hbmr_kmeans_accum_workspace_bytes(n, k));
  if (sorted) {
    if (ws == nullptr || ws_bytes < hbmr_kmeans_accum_workspace_bytes(n, k) || n >= (1L << 32))
      return (int)hipErrorInvalidValue;
    char* w = reinterpret_cast<char*>(ws);
    const size_t kb = ws_align(((size_t)k + 1) * 4);
    uint32_t* hist = reinterpret_cast<uint32_t*>(w);
    uint32_t* offsets = reinterpret_cast<uint32_t*>(w + kb);
    uint32_t* cursor = reinterpret_cast<uint32_t*>(w + 2 * kb);
    uint32_t* perm = reinterpret_cast<uint32_t*>(w + 3 * kb);
    HBMR_RETURN_IF_ERROR(hipMemsetAsync(hist, 0, (size_t)k * 4, st));
    const size_t hlds = (size_t)k * 4;
    long hgrid = std::min<long>((n / 4 + 255) / 256 + 1, (long)cus * 2);
    hipLaunchKernelGGL(kmeans_hist_kernel, dim3((unsigned)hgrid), dim3(256), hlds, st, labels, n,
                       k, hist);
    hipLaunchKernelGGL(kmeans_scan_kernel, dim3(1), dim3(1024), 0, st, hist, k, offsets, cursor,
                       counts);
    const long sgrid = (n + kScatterPts - 1) / kScatterPts;
    hipLaunchKernelGGL(kmeans_scatter_kernel, dim3((unsigned)sgrid), dim3(256), 2 * hlds, st,
                       labels, n, k, cursor, perm);
    // segsum: one chunk per wave, ~8 waves per CU worth of chunks at least
    // short chunks keep the per-wave dependent-load chain short for small
    // splits; long chunks amortise flush atomics for big ones
    long chunk = (n + (long)cus * 16 - 1) / ((long)cus * 16);
    chunk = std::min<long>(4096, std::max<long>(128, ((chunk + 63) / 64) * 64));
    const long nw = (n + chunk - 1) / chunk;
    const long sblocks = (nw + 3) / 4;
    switch (dp) {
#define HBMR_SEG(DD)                                                                        \
  case DD:                                                                                 \
    hipLaunchKernelGGL((kmeans_segsum_kernel<T, DD, 8>), dim3((unsigned)sblocks), dim3(256), \
                       0, st, reinterpret_cast<const T*>(X), n, perm, offsets, k, chunk,    \
                       sums, scale);                                                        \
    break;
      HBMR_SEG(64)
      HBMR_SEG(128)
      HBMR_SEG(256)
#undef HBMR_SEG
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  switch (dp) {
    case 64: return launch_accum<T, 64>(X, n, labels, k, sums, counts, scale, cus, st);
    case 128: return launch_accum<T, 128>(X, n, labels, k, sums, counts, scale, cus, st);
    case 256: return launch_accum<T, 256>(X, n, labels, k, sums, counts, scale, cus, st);
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" {

int hbmr_kmeans_accum_bf16(const void* X, long n, int dp, const int32_t* labels, int k,
                           long long* sums, long long* counts, int fx_shift, void* ws,
                           long ws_bytes, int mode, hipStream_t st) {
  return accum_impl<__bf16>(X, n, dp, labels, k, sums, counts, fx_shift, ws, ws_bytes, mode, st);
}

// Exact mode: the combiner over the fp32 points (rows of dp floats), so the
// partial sums are the int64 fixed point of the fp32 data, not of its bf16 copy.
int hbmr_kmeans_accum_f32(const float* X, long n, int dp, const int32_t* labels, int k,
                          long long* sums, long long* counts, int fx_shift, void* ws,
                          long ws_bytes, int mode, hipStream_t st) {
  return accum_impl<float>(X, n, dp, labels, k, sums, counts, fx_shift, ws, ws_bytes, mode, st);
}

int hbmr_kmeans_update(const long long* sums, const long long* counts, int fx_shift, int k, int d,
                       int dp, int k_pad, float* cen, void* cbf, float* chalf, float* shift2,
                       hipStream_t st) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(k), dim3(128), 0, st, sums, counts, k, d, dp,
                     ldexpf(1.0f, -fx_shift), cen, reinterpret_cast<__bf16*>(cbf), chalf, shift2);
  if (k_pad > k)
    hipLaunchKernelGGL(kmeans_pad_clusters_kernel, dim3(k_pad - k), dim3(64), 0, st,
                       reinterpret_cast<__bf16*>(cbf), chalf, k, k_pad, dp);
  return (int)hipGetLastError();
}

int hbmr_kmeans_padded_k(int k) { return ((k + kCK - 1) / kCK) * kCK; }

int hbmr_kmeans_padded_dim(int d) {
  for (int dp : {64, 128, 256})
    if (d <= dp) return dp;
  return -1;
}

int hbmr_f32_to_bf16_pad(const float* src, long n, int d, int dp, void* dst, hipStream_t st) {
  if (n <= 0) return 0;
  if (d > dp) return (int)hipErrorInvalidValue;
  const long total = n * dp;
  const long grid = std::min<long>((total + 255) / 256, 1L << 20);
  hipLaunchKernelGGL(f32_to_bf16_pad_kernel, dim3((unsigned)grid), dim3(256), 0, st, src, n, d,
                     dp, reinterpret_cast<uint16_t*>(dst));
  return (int)hipGetLastError();
}

// A batch of K-Means map tasks (one per split) launched from C++ in one call:
// assign + combine per split into its own output slab sums[t] / counts[t]
// (zeroed here).  Removes the per-task host overhead of the runtime's launch
// path; each task still gets its own map output (attempt isolation).
long hbmr_kmeans_batch_workspace_bytes(long total_n, int ntasks, int k) {
  return (long)(ws_align((size_t)ntasks * k * 4) * 2 + ws_align((size_t)ntasks * (k + 1) * 4) +
                ws_align((size_t)total_n * 4));
}

// Grouped path: 1 memset + 3 launches for the whole batch (assign+hist,
// scan+scatter, segmented sum).  labels must hold Σ n[t] entries.
static int map_batch_grouped(int ntasks, const void* const* X, const long* n, int dp,
                             const void* C, const float* chalf, int k_pad, int k,
                             int32_t* labels, void* ws, long long* sums, long long* counts,
                             int fx_shift, hipStream_t st, int cus) {
  SplitTable t;
  memset(&t, 0, sizeof(t));
  t.nsplit = ntasks;
  t.k = k;
  long total = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.X[i] = reinterpret_cast<const __bf16*>(X[i]);
    t.n[i] = n[i];
    t.off[i] = total;
    total += n[i];
  }
  char* w = reinterpret_cast<char*>(ws);
  const size_t hb = ws_align((size_t)ntasks * k * 4);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* cursor = reinterpret_cast<uint32_t*>(w + hb);
  uint32_t* offsets = reinterpret_cast<uint32_t*>(w + 2 * hb);
  uint32_t* perm = reinterpret_cast<uint32_t*>(w + 2 * hb + ws_align((size_t)ntasks * (k + 1) * 4));
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(hist, 0, 2 * hb, st));  // hist + cursor
  // 1. assign (+ histogram: fused atomics in the assign epilogue, or a separate
  //    LDS-binned pass over the labels; HBMR_KMEANS_FUSED_HIST=1 selects fused)
  static const bool fused = [] {
    const char* e = getenv("HBMR_KMEANS_FUSED_HIST");
    return e != nullptr && e[0] == '1';
  }();
  long nb = 0;
  int pts = 0;
  switch (dp) {
    case 64: pts = assign_pts<64>(fused); break;
    case 128: pts = assign_pts<128>(fused); break;
    case 256: pts = assign_pts<256>(fused); break;
    default: return (int)hipErrorInvalidValue;
  }
  for (int i = 0; i < ntasks; ++i) {
    t.blk[i] = nb;
    nb += (n[i] + pts - 1) / pts;
  }
  t.blk[ntasks] = nb;
  if (nb > 0) {
    switch (dp) {
#define HBMR_GA(DD)                                                                          \
  case DD:                                                                                   \
    launch_grouped_assign<DD>(nb, t, C, chalf, k_pad, labels, fused ? hist : nullptr, st);   \
    break;
      HBMR_GA(64)
      HBMR_GA(128)
      HBMR_GA(256)
#undef HBMR_GA
    }
    HBMR_RETURN_IF_ERROR(hipGetLastError());
  }
  if (!fused) {
    long hb_blocks = 0;
    for (int i = 0; i < ntasks; ++i) {
      t.blk[i] = hb_blocks;
      hb_blocks += (n[i] + kHistPts - 1) / kHistPts;
    }
    t.blk[ntasks] = hb_blocks;
    if (hb_blocks > 0) {
      hipLaunchKernelGGL(kmeans_hist_grouped_kernel, dim3((unsigned)hb_blocks), dim3(256),
                         (size_t)k * 4, st, t, labels, hist);
      HBMR_RETURN_IF_ERROR(hipGetLastError());
    }
  }
  // 2. scan + scatter (+ counts, offsets)
  nb = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.blk[i] = nb;
    nb += std::max<long>(1, (n[i] + kScatterPts - 1) / kScatterPts);
  }
  t.blk[ntasks] = nb;
  hipLaunchKernelGGL(kmeans_scatter_grouped_kernel, dim3((unsigned)nb), dim3(256),
                     (size_t)3 * k * 4, st, t, labels, hist, cursor, offsets, perm, counts);
  HBMR_RETURN_IF_ERROR(hipGetLastError());
  // 3. segmented row sums: chunks sized so the batch yields ≥ 16 waves per CU
  long chunk = (total + (long)cus * 16 - 1) / ((long)cus * 16);
  chunk = std::min<long>(4096, std::max<long>(128, ((chunk + 63) / 64) * 64));
  long nw = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.blk[i] = nw;
    nw += (n[i] + chunk - 1) / chunk;
  }
  t.blk[ntasks] = nw;
  const float scale = ldexpf(1.0f, fx_shift);
  if (nw > 0) {
    const long blocks = (nw + 3) / 4;
    switch (dp) {
#define HBMR_GS(DD)                                                                         \
  case DD:                                                                                  \
    hipLaunchKernelGGL((kmeans_segsum_grouped_kernel<DD, 8>), dim3((unsigned)blocks),       \
                       dim3(256), 0, st, t, perm, offsets, chunk, sums, scale);             \
    break;
      HBMR_GS(64)
      HBMR_GS(128)
      HBMR_GS(256)
#undef HBMR_GS
    }
  }
  return (int)hipGetLastError();
}

int hbmr_kmeans_map_batch(int ntasks, const void* const* X, const long* n, int dp,
                          const void* C, const float* chalf, int k_pad, int k, int32_t* labels,
                          void* ws, long ws_bytes, long long* sums, long long* counts,
                          int fx_shift, int zero_outputs, hipStream_t st) {
  if (ntasks <= 0) return 0;
  if (zero_outputs) {
    HBMR_RETURN_IF_ERROR(hipMemsetAsync(sums, 0, (size_t)ntasks * k * dp * 8, st));
    HBMR_RETURN_IF_ERROR(hipMemsetAsync(counts, 0, (size_t)ntasks * k * 8, st));
  }
  long total = 0;
  for (int t = 0; t < ntasks; ++t) total += n[t];
  const bool small = ((size_t)k * AccCfg<128>::RS * 8 + (size_t)k * 4) <= 76 * 1024 && dp <= 128;
  if (!small && ntasks <= kMaxGroup && k <= 8192 &&
      ws_bytes >= hbmr_kmeans_batch_workspace_bytes(total, ntasks, k)) {
    set_lds_limits();
    return map_batch_grouped(ntasks, X, n, dp, C, chalf, k_pad, k, labels, ws, sums, counts,
                             fx_shift, st, cu_count());
  }
  // every task's labels at its offset in `labels` (as the grouped path lays
  // them out): callers keep them, e.g. as the delta combiner's reference partition
  long off = 0;
  for (int t = 0; t < ntasks; ++t) {
    int rc = hbmr_kmeans_assign_bf16(X[t], n[t], dp, C, chalf, k_pad, labels + off, nullptr, st);
    if (rc) return rc;
    rc = hbmr_kmeans_accum_bf16(X[t], n[t], dp, labels + off, k, sums + (size_t)t * k * dp,
                                counts + (size_t)t * k, fx_shift, ws, ws_bytes, 0, st);
    if (rc) return rc;
    off += n[t];
  }
  return 0;
}

// ---- delta combiner (see kmeans_delta_* above) ------------------------------------
// workspace: hist[B*k] | cursor[B*k] | offsets[B*(k+1)] | mcount[B] | movers[total]
// (uint2) | perm[2*total] (u32), regions 256-B aligned.
long hbmr_kmeans_delta_workspace_bytes(long total_n, int ntasks, int k) {
  return (long)(2 * ws_align((size_t)ntasks * k * 4) + ws_align((size_t)ntasks * (k + 1) * 4) +
                ws_align((size_t)ntasks * 4) + 2 * ws_align((size_t)total_n * 8));
}

}  // extern "C"

template <typename T>
static int delta_combine_impl(int ntasks, const void* const* X, const long* n, int dp, int k,
                              const int32_t* labels, void* ws, long long* sums,
                              long long* counts, int fx_shift, int32_t* const* g,
                              const long long* const* S0, const long long* const* N0,
                              hipStream_t st) {
  SplitTable t;
  memset(&t, 0, sizeof(t));
  t.nsplit = ntasks;
  t.k = k;
  long total = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.X[i] = reinterpret_cast<const __bf16*>(X[i]);
    t.n[i] = n[i];
    t.off[i] = total;
    total += n[i];
  }
  char* w = reinterpret_cast<char*>(ws);
  const size_t hb = ws_align((size_t)ntasks * k * 4);
  const size_t ob = ws_align((size_t)ntasks * (k + 1) * 4);
  const size_t mb = ws_align((size_t)ntasks * 4);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* cursor = reinterpret_cast<uint32_t*>(w + hb);
  uint32_t* offsets = reinterpret_cast<uint32_t*>(w + 2 * hb);
  uint32_t* mcount = reinterpret_cast<uint32_t*>(w + 2 * hb + ob);
  uint2* movers = reinterpret_cast<uint2*>(w + 2 * hb + ob + mb);
  uint32_t* perm = reinterpret_cast<uint32_t*>(w + 2 * hb + ob + mb + ws_align((size_t)total * 8));
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(hist, 0, 2 * hb, st));   // hist + cursor
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(mcount, 0, mb, st));
  // 0. outputs start from the reference partition's sums and counts
  SlabTable src;
  memset(&src, 0, sizeof(src));
  for (int i = 0; i < ntasks; ++i) {
    src.s[i] = S0[i];
    src.c[i] = N0[i];
  }
  const long slab = (long)k * dp;
  const unsigned gx = (unsigned)std::max<long>(1, std::min<long>((slab / 2 + 255) / 256, 64));
  hipLaunchKernelGGL(kmeans_slab_copy_kernel, dim3(gx, (unsigned)ntasks), dim3(256), 0, st, src,
                     slab, k, sums, counts);
  HBMR_RETURN_IF_ERROR(hipGetLastError());
  // 1. movers, entry histogram, count deltas, g := labels
  long nb = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.blk[i] = nb;
    nb += (n[i] + kDiffPts - 1) / kDiffPts;
  }
  t.blk[ntasks] = nb;
  GTable gt;
  memset(&gt, 0, sizeof(gt));
  for (int i = 0; i < ntasks; ++i) gt.g[i] = g[i];
  if (nb > 0) {
    hipLaunchKernelGGL(kmeans_delta_diff_kernel, dim3((unsigned)nb), dim3(256), (size_t)2 * k * 4,
                       st, t, gt, labels, movers, mcount, hist, counts);
    HBMR_RETURN_IF_ERROR(hipGetLastError());
  }
  // 2. entries sorted by cluster (grid for the worst case, 2n entries per split)
  nb = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.blk[i] = nb;
    nb += std::max<long>(1, (2 * n[i] + kScatterPts - 1) / kScatterPts);
  }
  t.blk[ntasks] = nb;
  hipLaunchKernelGGL(kmeans_delta_scatter_kernel, dim3((unsigned)nb), dim3(256),
                     (size_t)3 * k * 4, st, t, movers, mcount, hist, cursor, offsets, perm);
  HBMR_RETURN_IF_ERROR(hipGetLastError());
  // 3. signed segmented row sums (persistent waves over the device-side counts)
  const float scale = ldexpf(1.0f, fx_shift);
  const unsigned blocks = (unsigned)cu_count() * 4;
  switch (dp) {
#define HBMR_DS(DD)                                                                          \
  case DD:                                                                                   \
    hipLaunchKernelGGL((kmeans_delta_segsum_kernel<T, DD, 8>), dim3(blocks), dim3(256), 0,   \
                       st, t, movers, mcount, perm, offsets, 256L, sums, scale);             \
    break;
    HBMR_DS(64)
    HBMR_DS(128)
    HBMR_DS(256)
#undef HBMR_DS
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

extern "C" {

int hbmr_kmeans_delta_combine(int ntasks, const void* const* X, const long* n, int dp, int x_f32,
                              int k, const int32_t* labels, void* ws, long ws_bytes,
                              long long* sums, long long* counts, int fx_shift,
                              int32_t* const* g, const long long* const* S0,
                              const long long* const* N0, hipStream_t st) {
  if (ntasks <= 0) return 0;
  if (ntasks > kMaxGroup || k <= 0 || k > 8192 || (dp != 64 && dp != 128 && dp != 256))
    return (int)hipErrorInvalidValue;
  long total = 0;
  for (int i = 0; i < ntasks; ++i) {
    if (n[i] < 0 || n[i] >= (1L << 31)) return (int)hipErrorInvalidValue;
    total += n[i];
  }
  if (ws == nullptr || ws_bytes < hbmr_kmeans_delta_workspace_bytes(total, ntasks, k))
    return (int)hipErrorInvalidValue;
  set_lds_limits();
  return x_f32 ? delta_combine_impl<float>(ntasks, X, n, dp, k, labels, ws, sums, counts,
                                           fx_shift, g, S0, N0, st)
               : delta_combine_impl<__bf16>(ntasks, X, n, dp, k, labels, ws, sums, counts,
                                            fx_shift, g, S0, N0, st);
}

// A batch of map tasks against reference partitions: grouped MFMA assign of
// every split into `labels`, then the delta combiner.
int hbmr_kmeans_map_batch_delta(int ntasks, const void* const* X, const long* n, int dp,
                                const void* C, const float* chalf, int k_pad, int k,
                                int32_t* labels, void* ws, long ws_bytes, long long* sums,
                                long long* counts, int fx_shift, int32_t* const* g,
                                const long long* const* S0, const long long* const* N0,
                                hipStream_t st) {
  if (ntasks <= 0) return 0;
  if (ntasks > kMaxGroup || k_pad % kCK) return (int)hipErrorInvalidValue;
  SplitTable t;
  memset(&t, 0, sizeof(t));
  t.nsplit = ntasks;
  t.k = k;
  int pts = 0;
  switch (dp) {
    case 64: pts = assign_pts<64>(false); break;
    case 128: pts = assign_pts<128>(false); break;
    case 256: pts = assign_pts<256>(false); break;
    default: return (int)hipErrorInvalidValue;
  }
  long total = 0, nb = 0;
  for (int i = 0; i < ntasks; ++i) {
    t.X[i] = reinterpret_cast<const __bf16*>(X[i]);
    t.n[i] = n[i];
    t.off[i] = total;
    total += n[i];
    t.blk[i] = nb;
    nb += (n[i] + pts - 1) / pts;
  }
  t.blk[ntasks] = nb;
  if (nb > 0x7fffffffL) return (int)hipErrorInvalidValue;
  if (nb > 0) {
    switch (dp) {
      case 64: launch_grouped_assign<64>(nb, t, C, chalf, k_pad, labels, nullptr, st); break;
      case 128: launch_grouped_assign<128>(nb, t, C, chalf, k_pad, labels, nullptr, st); break;
      case 256: launch_grouped_assign<256>(nb, t, C, chalf, k_pad, labels, nullptr, st); break;
    }
    HBMR_RETURN_IF_ERROR(hipGetLastError());
  }
  return hbmr_kmeans_delta_combine(ntasks, X, n, dp, 0, k, labels, ws, ws_bytes, sums, counts,
                                   fx_shift, g, S0, N0, st);
}

int hbmr_kmeans_assign_top3_bf16(const void* X, long n, int dp, const void* C, const float* chalf,
                                 int k_pad, int32_t* labels, int32_t* cand, float* scores,
                                 float* margin, hipStream_t st) {
  if (!labels || !cand || !scores || !margin) return (int)hipErrorInvalidValue;
  switch (dp) {
    case 64: return launch_assign_top3<64, false>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    case 128: return launch_assign_top3<128, false>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    case 256: return launch_assign_top3<256, false>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// exact mode's default: fp16 operands (rows of fp16 bit patterns, C the fp16
// centroid image of hbmr_kmeans_image_f16, chalf its -|c~|^2/2)
int hbmr_kmeans_assign_top3_f16(const void* X, long n, int dp, const void* C, const float* chalf,
                                int k_pad, int32_t* labels, int32_t* cand, float* scores,
                                float* margin, hipStream_t st) {
  if (!labels || !cand || !scores || !margin) return (int)hipErrorInvalidValue;
  switch (dp) {
    case 64: return launch_assign_top3<64, true>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    case 128: return launch_assign_top3<128, true>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    case 256: return launch_assign_top3<256, true>(X, n, C, chalf, k_pad, labels, cand, scores, margin, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// the top-3 assign of a batch of splits in one launch (dp <= 128; else
// hipErrorNotSupported): labels / scores [N], cand / margin [2N] of the batch,
// N = sum n, split i at offset n[0] + ... + n[i-1]
int hbmr_kmeans_assign_top3_grouped(int nsplit, const void* const* X, const long* n, int dp,
                                    int f16, const void* C, const float* chalf, int k_pad,
                                    int32_t* labels, int32_t* cand, float* scores, float* margin,
                                    hipStream_t st) {
  if (!labels || !cand || !scores || !margin) return (int)hipErrorInvalidValue;
#define HBMR_TOP3G(D)                                                                      \
  return f16 ? launch_assign_top3_grouped<D, true>(nsplit, X, n, C, chalf, k_pad, labels,  \
                                                   cand, scores, margin, st)               \
             : launch_assign_top3_grouped<D, false>(nsplit, X, n, C, chalf, k_pad, labels, \
                                                    cand, scores, margin, st)
  switch (dp) {
    case 64: HBMR_TOP3G(64);
    case 128: HBMR_TOP3G(128);
    case 256: HBMR_TOP3G(256);
    default: return (int)hipErrorInvalidValue;
  }
#undef HBMR_TOP3G
}

// Exact mode, one batch: top-3 assign with step 1 fused (FusedQ1Fin): labels
// of every point, the batch's step-2 queue and flagged count in ws (as
// hbmr_kmeans_refine_batch_q1g leaves them); dp <= 128
int hbmr_kmeans_assign_top3_q1_grouped(int nsplit, const void* const* X, const long* n, int dp,
                                       int f16, const void* C, const void* Ct,
                                       const float* chalf, int k_pad,
                                       int32_t* labels, const float* const* xnorm,
                                       const float* const* xbn2, const float* const* xerr,
                                       int d, int k, const float* cnorm, const float* cmax,
                                       const float* cerr, const float* cerrmax, void* ws,
                                       long ws_bytes, const float* dcc, hipStream_t st) {
  if (nsplit <= 0 || nsplit > kMaxGroup || k_pad % 32 || k <= 0 || k_pad < k ||
      d > kRefineMaxDp || !labels || ((uintptr_t)ws & 255) || (dp != 64 && dp != 128))
    return (int)hipErrorInvalidValue;
  TopQ1Table t;
  memset(&t, 0, sizeof(t));
  t.nsplit = nsplit;
  constexpr int pts = 4 * 2 * 32;             // AssignV2<D>::WAVES * PB * 32
  long total = 0, nb = 0;
  for (int i = 0; i < nsplit; ++i) {
    if (n[i] < 0 || n[i] > 0x7fffffffL) return (int)hipErrorInvalidValue;
    t.X[i] = reinterpret_cast<const __bf16*>(X[i]);
    t.xnorm[i] = xnorm[i];
    t.xbn2[i] = xbn2[i];
    t.xerr[i] = xerr[i];
    t.off[i] = total;
    t.blk[i] = nb;
    total += n[i];
    nb += ceil_div(n[i], pts);
  }
  t.off[nsplit] = total;
  t.blk[nsplit] = nb;
  const RefineLayout Ly = refine_layout(nsplit, n);
  if (ws_bytes < (long)Ly.bytes) return (int)hipErrorInvalidValue;
  char* w = static_cast<char*>(ws);
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(w, 0, kHdrClear, st));
  if (nb == 0) return 0;
  if (nb > 0x7fffffffL) return (int)hipErrorInvalidValue;
  int tb = 0;
  while ((1 << tb) < k_pad / 32) ++tb;
  FusedQ1Fin fin;
  memset(&fin, 0, sizeof(fin));
  fin.k = k;
  const double inflate = 1.0 + 0x1p-20;
  fin.gam = (double)(d + 2) * 0x1p-23 * 1.01;
  // cmax / cerrmax are device values: the kernel reads them through cnorm's
  // image: pass pointers and let the kernel fold them (see below)
  fin.pack_rel = ldexp(1.0, 4 + tb - 23);
  fin.cnorm = cnorm;
  fin.cerr = cerr;
  fin.dcc = dcc;
  fin.qcount = reinterpret_cast<uint32_t*>(w);
  fin.q1 = reinterpret_cast<ExactQ1*>(w + Ly.off1);
  fin.cap1 = Ly.cap1;
  fin.stats = reinterpret_cast<unsigned long long*>(w + kStatsOff);
  fin.cmax_p = cmax;
  fin.cerrmax_p = cerrmax;
  (void)inflate;
  // the v3 kernel (default; needs the tiled image Ct), or v2
  // (hbmr_kmeans_set_exact_kernel(2) / HBMR_EXACT_V3=v2, read once)
  if (exact_kernel() == 3) {
    if (!Ct) return (int)hipErrorInvalidValue;
    auto kern = dp == 64 ? (f16 ? kmeans_assign_top3_q1_v3_kernel<64, true>
                                : kmeans_assign_top3_q1_v3_kernel<64, false>)
                         : (f16 ? kmeans_assign_top3_q1_v3_kernel<128, true>
                                : kmeans_assign_top3_q1_v3_kernel<128, false>);
    const size_t lds = dp == 64 ? AssignV2<64>::LDS_BYTES : AssignV2<128>::LDS_BYTES;
    hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(256), lds, st, t,
                       reinterpret_cast<const __bf16*>(Ct), chalf, k_pad / 32, labels, fin);
    return (int)hipGetLastError();
  }
  auto kern = dp == 64 ? (f16 ? kmeans_assign_top3_q1_grouped_kernel<64, true>
                              : kmeans_assign_top3_q1_grouped_kernel<64, false>)
                       : (f16 ? kmeans_assign_top3_q1_grouped_kernel<128, true>
                              : kmeans_assign_top3_q1_grouped_kernel<128, false>);
  const size_t lds = dp == 64 ? AssignV2<64>::LDS_BYTES : AssignV2<128>::LDS_BYTES;
  hipLaunchKernelGGL(kern, dim3((unsigned)nb),
                     dim3(dp == 64 ? AssignV2<64>::THREADS : AssignV2<128>::THREADS), lds, st, t,
                     reinterpret_cast<const __bf16*>(C), chalf, k_pad / 32, labels, fin);
  return (int)hipGetLastError();
}

int hbmr_kmeans_refine_f32(const float* X32, long n, int d, int ldx, const float* xnorm,
                           const float* xbn2, const float* xerr, const float* C32, int k,
                           int k_pad, const float* cnorm, const float* cmax, const float* cerr,
                           const float* cerrmax, const int32_t* nbr_idx,
                           const float* nbr_dist, int L, int32_t* labels, const int32_t* cand,
                           const float* scores, const float* margin, unsigned long long* stats,
                           int nstats, hipStream_t st) {
  if (n <= 0) return 0;
  if (d > ldx || d > kRefineMaxDp || k <= 0 || k_pad < k || L < 1 || L > k)
    return (int)hipErrorInvalidValue;
  // packing truncation of the arg-max codes: lb = 4 + ceil(log2(k_pad / 32)) bits
  int tb = 0;
  while ((1 << tb) < k_pad / 32) ++tb;
  const double pack_rel = ldexp(1.0, 4 + tb - 23);
  const long blocks = (n + 255) / 256;
  // v2 wants whole 8-feature lane slices and 16-byte aligned rows
  const bool v2_ok = d % 8 == 0 && ldx % 4 == 0 && ((uintptr_t)X32 & 15) == 0 &&
                     ((uintptr_t)C32 & 15) == 0;
  if (v2_ok && refine_version() == 2) {
    auto kern = d <= 128 ? kmeans_refine_v2_kernel<1> : kmeans_refine_v2_kernel<2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, X32, n, d, ldx, xnorm,
                       xbn2, xerr, C32, k, cnorm, cmax, cerr, cerrmax, pack_rel, nbr_idx,
                       nbr_dist, L, labels, cand, scores, margin, stats, nstats);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(kmeans_refine_kernel, dim3((unsigned)blocks), dim3(256), 0, st, X32, n, d,
                     ldx, xnorm, xbn2, xerr, C32, k, cnorm, cmax, cerr, cerrmax, pack_rel,
                     nbr_idx, nbr_dist, L,
                     labels, cand, scores, margin, stats, nstats);
  return (int)hipGetLastError();
}


int hbmr_kmeans_exact_prep(const float* x, long n, int d, int ldx, int dp, int f16, void* x16,
                           float* xnorm, float* xn2, float* xerr, hipStream_t st) {
  if (n <= 0) return 0;
  if (d > ldx || d > dp || dp % 8 || !x16 || !xnorm || !xn2 || !xerr)
    return (int)hipErrorInvalidValue;
  const long blocks = (n + 15) / 16;
  if (blocks > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_exact_prep_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, d,
                     ldx, dp, f16, reinterpret_cast<uint16_t*>(x16), xnorm, xn2, xerr);
  return (int)hipGetLastError();
}

// the fused exact top-3 kernel: 3 (v3, the default) or 2 (v2); -1 restores the
// default (HBMR_EXACT_V3=v2 selects v2).  Returns the previous setting.
int hbmr_kmeans_set_exact_kernel(int v) {
  const int old = g_exact_kernel;
  g_exact_kernel = v == 2 || v == 3 ? v : -1;
  return old;
}

int hbmr_kmeans_image16_tiled(const void* c16, int k_pad, int dp, void* c16t, hipStream_t st) {
  if (k_pad <= 0 || k_pad % 32 || (dp != 64 && dp != 128) || !c16 || !c16t)
    return (int)hipErrorInvalidValue;
  const long pieces = (long)k_pad * dp / 8;
  hipLaunchKernelGGL(kmeans_image16_tiled_kernel, dim3((unsigned)((pieces + 255) / 256)),
                     dim3(256), 0, st, reinterpret_cast<const uint4*>(c16), k_pad, dp,
                     reinterpret_cast<uint4*>(c16t));
  return (int)hipGetLastError();
}

// maxima: float [2] = (max |c_j|, max |c_j - c~_j|), written by the kernel
int hbmr_kmeans_image16(const float* cen, int k, int d, int dp, int k_pad, int f16, void* c16,
                        float* chalf, float* cnorm, float* cerr, float* maxima, hipStream_t st) {
  if (k <= 0 || k_pad < k || d > dp) return (int)hipErrorInvalidValue;
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(maxima, 0, 2 * sizeof(float), st));
  hipLaunchKernelGGL(kmeans_image16_kernel, dim3((unsigned)k_pad), dim3(128), 0, st, cen, k, d,
                     dp, f16, reinterpret_cast<uint16_t*>(c16), chalf, cnorm, cerr,
                     reinterpret_cast<unsigned*>(maxima));
  return (int)hipGetLastError();
}


}  // extern "C"

// One workgroup per centroid a: D(a, b) = sum_i (c_ai - c_bi)^2 in fp64 — one
// rounded difference and d fused square-adds, |D~ - D| <= (d + 2) 2^-53 D —
// then the lower bound sqrt(D~ (1 - rel)) rounded DOWN to fp32 and the upper
// bound sqrt(D~ (1 + rel)) rounded UP (rel = (d + 4) 2^-53 * 1.01 also covers
// the product and sqrt roundings).  The (lower bound, b) keys of the row are
// bitonic-sorted in LDS — ties by index, i.e. a stable sort — and the L
// first kept (di, dv: the scan order and its stop rule); pd[a][b] gets the
// upper bounds.  The pairwise form (not the Gram form) bounds the error by D
// itself, so near centroids keep tight bounds.
constexpr int kNbrThreads = 256;
constexpr int kNbrMaxD = 256;
constexpr int kNbrMaxK = 8192;

__global__ __launch_bounds__(kNbrThreads) void kmeans_centroid_nbr_kernel(
    const float* __restrict__ cen, int k, int d, int L, int kp2, double rel,
    int32_t* __restrict__ di, float* __restrict__ dv, float* __restrict__ pd) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_key[];   // kp2
  __shared__ double s_ca[kNbrMaxD];
  const int a = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < d; i += kNbrThreads) s_ca[i] = (double)cen[(long)a * d + i];
  __syncthreads();
  const bool vec4 = (d & 3) == 0;
  for (int b = t; b < kp2; b += kNbrThreads) {
    unsigned long long key = ~0ull;
    if (b < k) {
      float lo_f = 0.f, hi_f = 0.f;
      if (b != a) {
        const float* cb = cen + (long)b * d;
        double acc = 0.0;
        if (vec4) {
          for (int i = 0; i < d; i += 4) {
            const float4 v = *reinterpret_cast<const float4*>(cb + i);
            double e = s_ca[i] - (double)v.x;
            acc = fma(e, e, acc);
            e = s_ca[i + 1] - (double)v.y;
            acc = fma(e, e, acc);
            e = s_ca[i + 2] - (double)v.z;
            acc = fma(e, e, acc);
            e = s_ca[i + 3] - (double)v.w;
            acc = fma(e, e, acc);
          }
        } else {
          for (int i = 0; i < d; ++i) {
            const double e = s_ca[i] - (double)cb[i];
            acc = fma(e, e, acc);
          }
        }
        const double lo = sqrt(fmax(0.0, acc * (1.0 - rel)));
        const double hi = sqrt(acc * (1.0 + rel));
        lo_f = (float)lo;
        if ((double)lo_f > lo) lo_f = nextafterf(lo_f, 0.f);
        hi_f = (float)hi;
        if ((double)hi_f < hi) hi_f = nextafterf(hi_f, __builtin_inff());
      }
      if (pd) pd[(long)a * k + b] = hi_f;
      key = ((unsigned long long)__float_as_uint(lo_f) << 32) | (unsigned)b;
    }
    s_key[b] = key;
  }
  __syncthreads();
  for (int size = 2; size <= kp2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < kp2 / 2; i += kNbrThreads) {
        const int pos = 2 * i - (i & (stride - 1));
        const int q = pos + stride;
        const bool up = (pos & size) == 0;
        const unsigned long long x = s_key[pos], y = s_key[q];
        if ((x > y) == up) {
          s_key[pos] = y;
          s_key[q] = x;
        }
      }
      __syncthreads();
    }
  }
  for (int j = t; j < L; j += kNbrThreads) {
    const unsigned long long key = s_key[j];
    di[(long)a * L + j] = (int32_t)(uint32_t)(key & 0xffffffffull);
    dv[(long)a * L + j] = __uint_as_float((uint32_t)(key >> 32));
  }
}

extern "C" {

int hbmr_kmeans_centroid_nbr(const float* cen, int k, int d, int L, int32_t* di, float* dv,
                             float* pd, hipStream_t st) {
  if (k <= 0 || k > kNbrMaxK || d <= 0 || d > kNbrMaxD || L <= 0 || L > k)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)cen & 15) != 0) return (int)hipErrorInvalidValue;
  int kp2 = 1;
  while (kp2 < k) kp2 <<= 1;
  const size_t lds = (size_t)kp2 * sizeof(unsigned long long);
  static bool lds_set = false;
  if (!lds_set) {
    HBMR_RETURN_IF_ERROR(hipFuncSetAttribute((const void*)kmeans_centroid_nbr_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)(kNbrMaxK * sizeof(unsigned long long))));
    lds_set = true;
  }
  const double rel = (double)(d + 4) * 0x1p-53 * 1.01;
  hipLaunchKernelGGL(kmeans_centroid_nbr_kernel, dim3((unsigned)k), dim3(kNbrThreads), lds, st,
                     cen, k, d, L, kp2, rel, di, dv, pd);
  return (int)hipGetLastError();
}


// Refine v3 over a batch of splits (ns[nsplit]; at most 64): per split, right
// after its top-3 assign, hbmr_kmeans_refine_batch_q1 (reset = 1 for the
// first split); then hbmr_kmeans_refine_batch_finish once.  The workspace
// holds the two sharded queues (hbmr_kmeans_refine_batch_bytes).
long hbmr_kmeans_refine_batch_bytes(int nsplit, const long* ns) {
  if (nsplit <= 0 || nsplit > kMaxGroup) return -1;
  return (long)refine_layout(nsplit, ns).bytes;
}

int hbmr_kmeans_refine_batch_q1(int nsplit, const long* ns, int s, int d, int k, int k_pad,
                                const float* xnorm, const float* xbn2, const float* xerr,
                                const float* cnorm, const float* cmax, const float* cerr,
                                const float* cerrmax, const int32_t* labels, const int32_t* cand,
                                const float* scores, const float* margin,
                                unsigned long long* stats, void* ws, long ws_bytes, int reset,
                                const float* dcc, hipStream_t st) {
  if (nsplit <= 0 || nsplit > kMaxGroup || s < 0 || s >= nsplit || k <= 0 || k_pad < k ||
      d > kRefineMaxDp || ((uintptr_t)ws & 255))
    return (int)hipErrorInvalidValue;
  for (int i = 0; i < nsplit; ++i)
    if (ns[i] < 0 || ns[i] > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const RefineLayout Ly = refine_layout(nsplit, ns);
  if (ws_bytes < (long)Ly.bytes) return (int)hipErrorInvalidValue;
  char* w = static_cast<char*>(ws);
  uint32_t* c1 = reinterpret_cast<uint32_t*>(w);
  if (reset) HBMR_RETURN_IF_ERROR(hipMemsetAsync(c1, 0, kHdrClear, st));
  const long n = ns[s];
  if (n == 0) return 0;
  int tb = 0;
  while ((1 << tb) < k_pad / 32) ++tb;
  const double pack_rel = ldexp(1.0, 4 + tb - 23);
  const long b1 = ceil_div(n, 256 * kQ1Per);
  hipLaunchKernelGGL(kmeans_refine_q1_kernel, dim3((unsigned)b1), dim3(256), 0, st, n, s, d, k,
                     xnorm, xbn2, xerr, cnorm, cmax, cerr, cerrmax, pack_rel, labels, cand,
                     scores, margin, c1, reinterpret_cast<ExactQ1*>(w + Ly.off1), Ly.cap1,
                     reinterpret_cast<unsigned long long*>(w + kStatsOff), dcc);
  return (int)hipGetLastError();
}

// step 1 of a whole batch after hbmr_kmeans_assign_top3_grouped (resets the
// batch's queues): the batch arrays as that call wrote them
int hbmr_kmeans_refine_batch_q1g(int nsplit, const long* ns, int d, int k, int k_pad,
                                 const float* const* xnorm, const float* const* xbn2,
                                 const float* const* xerr, const float* cnorm, const float* cmax,
                                 const float* cerr, const float* cerrmax, const int32_t* labels,
                                 const int32_t* cand, const float* scores, const float* margin,
                                 void* ws, long ws_bytes, const float* dcc, hipStream_t st) {
  if (nsplit <= 0 || nsplit > kMaxGroup || k <= 0 || k_pad < k || d > kRefineMaxDp ||
      ((uintptr_t)ws & 255))
    return (int)hipErrorInvalidValue;
  Q1Table t;
  memset(&t, 0, sizeof(t));
  t.nsplit = nsplit;
  long total = 0, nb = 0;
  for (int i = 0; i < nsplit; ++i) {
    if (ns[i] < 0 || ns[i] > 0x7fffffffL) return (int)hipErrorInvalidValue;
    t.n[i] = ns[i];
    t.off[i] = total;
    t.blk[i] = nb;
    t.xnorm[i] = xnorm[i];
    t.xbn2[i] = xbn2[i];
    t.xerr[i] = xerr[i];
    total += ns[i];
    nb += ceil_div(ns[i], 256 * kQ1Per);
  }
  t.blk[nsplit] = nb;
  t.total = total;
  const RefineLayout Ly = refine_layout(nsplit, ns);
  if (ws_bytes < (long)Ly.bytes) return (int)hipErrorInvalidValue;
  char* w = static_cast<char*>(ws);
  uint32_t* c1 = reinterpret_cast<uint32_t*>(w);
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(c1, 0, kHdrClear, st));
  if (nb == 0) return 0;
  int tb = 0;
  while ((1 << tb) < k_pad / 32) ++tb;
  const double pack_rel = ldexp(1.0, 4 + tb - 23);
  hipLaunchKernelGGL(kmeans_refine_q1_grouped_kernel, dim3((unsigned)nb), dim3(256), 0, st, t, d,
                     k, cnorm, cmax, cerr, cerrmax, pack_rel, labels, cand, scores, margin, c1,
                     reinterpret_cast<ExactQ1*>(w + Ly.off1), Ly.cap1,
                     reinterpret_cast<unsigned long long*>(w + kStatsOff), dcc);
  return (int)hipGetLastError();
}

int hbmr_kmeans_refine_batch_finish(int nsplit, const long* ns, const float* const* x32,
                                    int32_t* const* labels, int d, int ldx, const float* C32,
                                    int k, int k_pad, const float* cmax, const float* cerrmax,
                                    const int32_t* nbr_idx, const float* nbr_dist, int L,
                                    unsigned long long* stats, int nstats, void* ws,
                                    long ws_bytes, hipStream_t st) {
  if (nsplit <= 0 || nsplit > kMaxGroup || d > ldx || d > kRefineMaxDp || d % 8 || ldx % 4 ||
      k <= 0 || k_pad < k || L < 1 || L > k || nstats < 3 || ((uintptr_t)C32 & 15) ||
      ((uintptr_t)ws & 255))
    return (int)hipErrorInvalidValue;
  const RefineLayout Ly = refine_layout(nsplit, ns);
  if (ws_bytes < (long)Ly.bytes) return (int)hipErrorInvalidValue;
  RefineTable tbl;
  std::memset(&tbl, 0, sizeof(tbl));
  tbl.nsplit = nsplit;
  for (int i = 0; i < nsplit; ++i) {
    if ((uintptr_t)x32[i] & 15) return (int)hipErrorInvalidValue;
    tbl.x32[i] = x32[i];
    tbl.labels[i] = labels[i];
  }
  int tb = 0;
  while ((1 << tb) < k_pad / 32) ++tb;
  const double pack_rel = ldexp(1.0, 4 + tb - 23);
  char* w = static_cast<char*>(ws);
  uint32_t* c1 = reinterpret_cast<uint32_t*>(w);
  uint32_t* c2 = c1 + kQShards;
  const ExactQ1* q1 = reinterpret_cast<const ExactQ1*>(w + Ly.off1);
  ExactQ2* q2 = reinterpret_cast<ExactQ2*>(w + Ly.off2);
  unsigned long long* ss = reinterpret_cast<unsigned long long*>(w + kStatsOff);
  // (q3 walks each point's neighbours through a chain of dependent loads:
  // a full grid keeps 4x more points in flight than the quarter grid did)
  const unsigned g3 = std::max(1u, Ly.g2);
  if (d <= 128) {
    hipLaunchKernelGGL(kmeans_refine_q2_kernel<1>, dim3(Ly.g2), dim3(256), 0, st, tbl, d, ldx,
                       C32, k, cmax, cerrmax, pack_rel, c1, q1, Ly.cap1, c2, q2, Ly.cap2, ss);
    HBMR_RETURN_IF_ERROR(hipGetLastError());
    hipLaunchKernelGGL(kmeans_refine_q3_kernel<1>, dim3(g3), dim3(256), 0, st, tbl, d, ldx, C32,
                       k, nbr_idx, nbr_dist, L, c2, q2, Ly.cap2, ss, nstats);
  } else {
    hipLaunchKernelGGL(kmeans_refine_q2_kernel<2>, dim3(Ly.g2), dim3(256), 0, st, tbl, d, ldx,
                       C32, k, cmax, cerrmax, pack_rel, c1, q1, Ly.cap1, c2, q2, Ly.cap2, ss);
    HBMR_RETURN_IF_ERROR(hipGetLastError());
    hipLaunchKernelGGL(kmeans_refine_q3_kernel<2>, dim3(g3), dim3(256), 0, st, tbl, d, ldx, C32,
                       k, nbr_idx, nbr_dist, L, c2, q2, Ly.cap2, ss, nstats);
  }
  HBMR_RETURN_IF_ERROR(hipGetLastError());
  hipLaunchKernelGGL(kmeans_refine_stats_kernel, dim3(1), dim3(64), 0, st, ss, stats, nstats);
  return (int)hipGetLastError();
}

}  // extern "C"

