// GPU sort / shuffle kernels for MI355X.
//
// * LSD radix sort of (uint64 key, uint32 value) pairs, 8-bit digits — the
//   replacement for MapOutputBuffer's QuickSort over (partition, key)
//   (hadoop-1.0.3 MapTask.java:1119-1130, 1415; util/QuickSort.java:57-131).
//   Per pass: (1) per-tile digit histograms (LDS integer atomics), (2) one
//   workgroup per digit scans its column of tile counts, (3) a stable scatter:
//   each 64-lane wave ranks its keys with 8 ballots (multi-split), waves are
//   ordered through LDS counters, the tile is regrouped by digit in LDS and
//   written out in digit runs (coalesced).  Stable, so multi-word keys sort
//   by successive passes least-significant word first.
// * TeraSort pieces: teragen_kernel (Hadoop 1.0.3 TeraGen records bit for bit,
//   TeraGen.java: LCG 3141592621·s + 663896637 mod 2^32 with O(log n) jump
//   ahead instead of the reference's O(n) stepping from a seed table),
//   key extraction, 100-byte record gather by permutation, splitter search for
//   range partitioning (TeraSort.java:57-211's trie partitioner), and an
//   order check (TeraValidate).
#include <string>
#include "common.h"
#include "../include/hbmr/hbmr.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortThreads * kSortItems;  // 4096 keys per workgroup
constexpr int kRadix = 256;
constexpr int kSortWaves = kSortThreads / HBMR_WAVE;

__device__ __forceinline__ uint32_t digit_of(uint64_t k, int shift) {
  return (uint32_t)(k >> shift) & 0xFFu;
}

// Block-wide exclusive scan of one value per thread (256 threads).
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* s_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) s_w[w] = v;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; ++i) base += s_w[i];
  __syncthreads();
  return base + v - x;
}

// (2) one workgroup per digit: exclusive scan over tiles in place, column total
__global__ __launch_bounds__(1024) void radix_scan_kernel(uint32_t* __restrict__ hist, long ntiles,
                                                          uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  uint32_t* h = hist + (long)blockIdx.x * ntiles;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) s_carry = 0;
  __syncthreads();
  for (long c = 0; c < ntiles; c += 4096) {
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long idx = c + (long)t * 4 + j;
      v[j] = idx < ntiles ? h[idx] : 0u;
      sum += v[j];
    }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(x, o);
      if (lane >= o) x += u;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t wbase = s_carry;
    for (int i = 0; i < w; ++i) wbase += s_w[i];
    uint32_t run = wbase + x - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long idx = c + (long)t * 4 + j;
      if (idx < ntiles) h[idx] = run;
      run += v[j];
    }
    __syncthreads();
    if (t == 1023) s_carry = run;
    __syncthreads();
  }
  if (t == 0) totals[blockIdx.x] = s_carry;
}

// (3') stable scatter with wave-private ranking.  Each wave owns a contiguous
// 1024-key quarter of the tile (loads stay 512 B per wave instruction), ranks
// its keys among equal digits with 8 ballots and a wave-private LDS counter per
// digit — no workgroup barrier inside the per-key loop (radix_scatter_kernel
// takes three per key) — then one digit-major scan over the 4 waves' counts
// places every key.  Order (wave, item, lane) is index order, so stable.
__global__ __launch_bounds__(kSortThreads) void radix_scatter_v2_kernel(
    const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint64_t* __restrict__ kout,
    uint32_t* __restrict__ vout, long n, int shift, long ntiles, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ totals) {
  __shared__ uint64_t s_k[kSortTile];
  __shared__ uint32_t s_v[kSortTile];
  __shared__ uint32_t s_wh[kSortWaves][kRadix];  // per-wave digit counts, then wave offsets
  __shared__ uint32_t s_toff[kRadix];
  __shared__ uint32_t s_gbase[kRadix];
  __shared__ uint32_t s_w[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const long tile = blockIdx.x;
  const long base = tile * kSortTile;
  const int tile_n = (int)min((long)kSortTile, n - base);
  constexpr int kWaveSpan = kSortTile / kSortWaves;  // 1024 keys per wave

#pragma unroll
  for (int i = 0; i < kSortWaves; ++i) s_wh[i][t] = 0u;
  uint64_t k[kSortItems];
  uint32_t v[kSortItems];
  const long wbase = base + (long)w * kWaveSpan;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = wbase + i * HBMR_WAVE + lane;
    if (e < n) {
      k[i] = kin[e];
      v[i] = vin ? vin[e] : (uint32_t)e;
    }
  }
  __syncthreads();
  const uint64_t lt = __lanemask_lt();
  uint32_t rank[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const bool valid = w * kWaveSpan + i * HBMR_WAVE + lane < tile_n;
    const uint32_t d = valid ? digit_of(k[i], shift) : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t pre = __popcll(m & lt);
    uint32_t old = 0u;
    if (valid) old = s_wh[w][d];
    __builtin_amdgcn_wave_barrier();
    rank[i] = old + pre;
    if (valid && pre == 0) s_wh[w][d] = old + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // thread t = digit t: tile offset of the digit, each wave's offset within it,
  // and the digit's global start for this tile
  {
    uint32_t c[kSortWaves], cnt = 0;
#pragma unroll
    for (int i = 0; i < kSortWaves; ++i) {
      c[i] = s_wh[i][t];
      cnt += c[i];
    }
    const uint32_t gb = block_excl_scan256(totals[t], s_w);
    s_gbase[t] = gb + hist[(long)t * ntiles + tile];
    const uint32_t toff = block_excl_scan256(cnt, s_w);
    s_toff[t] = toff;
    uint32_t run = toff;
#pragma unroll
    for (int i = 0; i < kSortWaves; ++i) {
      s_wh[i][t] = run;
      run += c[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    if (w * kWaveSpan + i * HBMR_WAVE + lane < tile_n) {
      const uint32_t local = s_wh[w][digit_of(k[i], shift)] + rank[i];
      s_k[local] = k[i];
      s_v[local] = v[i];
    }
  }
  __syncthreads();
  for (int j = t; j < tile_n; j += kSortThreads) {
    const uint64_t key = s_k[j];
    const uint32_t d = digit_of(key, shift);
    const long dst = (long)s_gbase[d] + (j - (long)s_toff[d]);
    kout[dst] = key;
    vout[dst] = s_v[j];
  }
}

// (1') digit histogram per tile with one LDS add per (wave, digit) group:
// 8 ballots find the lanes sharing a digit and its leader adds their count
// (radix_hist_kernel issues one contended LDS atomic per key)
__global__ __launch_bounds__(kSortThreads) void radix_hist_v2_kernel(const uint64_t* __restrict__ keys,
                                                                     long n, int shift, long ntiles,
                                                                     uint32_t* __restrict__ hist) {
  __shared__ uint32_t s[kSortWaves][kRadix];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int i = 0; i < kSortWaves; ++i) s[i][t] = 0u;
  __syncthreads();
  constexpr int kWaveSpan = kSortTile / kSortWaves;
  const long wbase = (long)blockIdx.x * kSortTile + (long)w * kWaveSpan;
  const uint64_t lt = __lanemask_lt();
  uint64_t k[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = wbase + i * HBMR_WAVE + lane;
    k[i] = e < n ? keys[e] : 0ull;
  }
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const bool valid = wbase + i * HBMR_WAVE + lane < n;
    const uint32_t d = digit_of(k[i], shift);
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    if (valid && __popcll(m & lt) == 0) s[w][d] += (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  hist[(long)t * ntiles + blockIdx.x] = s[0][t] + s[1][t] + s[2][t] + s[3][t];
}

// ---------------------------------------------------------------- onesweep (keys only)
// LSD radix sort of uint64 keys by bits [begin, begin + 8·passes) with ONE read
// of the keys for every digit's histogram and one scatter pass per digit whose
// tile offsets come from a decoupled look-back instead of a per-pass
// histogram + scan (radix_hist_v2 + radix_scan: one more read of the keys and
// two more launches per pass).  Tiles take their index from an atomic ticket,
// so every tile a tile waits on was scheduled before it.  Status words per
// (tile, digit), 64-bit: bits 63-48 the pass's epoch, 47-46 the kind (0
// empty, 1 aggregate = this tile's count, 2 inclusive prefix through this
// tile), 31-0 the value.  A word from another epoch reads as empty, so the
// status array is zeroed once when allocated, not before every pass.
// A look-back that sees nothing for kSpinLimit polls sets *err and moves on
// (the output is then wrong and the caller's order check sees it): every wave
// reaches the kernel's end.
constexpr uint64_t kStAgg = 1ull << 46, kStInc = 2ull << 46, kStKind = 3ull << 46;
constexpr int kSpinLimit = 1 << 22;
constexpr int kMaxPasses = 8;

__global__ __launch_bounds__(kSortThreads) void radix_hist_all_kernel(
    const uint64_t* __restrict__ keys, long n, int begin, int end, int passes,
    uint32_t* __restrict__ ghist) {
  __shared__ uint32_t s[kMaxPasses][kRadix];
  const int t = threadIdx.x;
  for (int p = 0; p < passes; ++p) s[p][t] = 0u;
  __syncthreads();
  for (long base = (long)blockIdx.x * kSortTile; base < n; base += (long)gridDim.x * kSortTile) {
#pragma unroll 4
    for (int i = 0; i < kSortItems; ++i) {
      const long e = base + (long)i * kSortThreads + t;
      if (e < n) {
        const uint64_t k = keys[e];
        for (int p = 0; p < passes; ++p) {
          const int sh = begin + 8 * p;
          atomicAdd(&s[p][(uint32_t)(k >> sh) & ((1u << min(8, end - sh)) - 1u)], 1u);
        }
      }
    }
  }
  __syncthreads();
  for (int p = 0; p < passes; ++p)
    if (s[p][t]) atomicAdd(&ghist[p * kRadix + t], s[p][t]);
}

// one workgroup per pass: exclusive scan of the digit counts in place
__global__ __launch_bounds__(kSortThreads) void radix_bases_kernel(uint32_t* __restrict__ ghist) {
  __shared__ uint32_t s_w[4];
  uint32_t* h = ghist + blockIdx.x * kRadix;
  const uint32_t x = h[threadIdx.x];
  const uint32_t e = block_excl_scan256(x, s_w);
  h[threadIdx.x] = e;
}

// WAVES waves of 64 lanes, 16 keys per lane: a tile of WAVES·1024 keys.  More
// keys per tile make longer digit runs for the scatter's writes (8 waves:
// 32 keys = 256 B per digit on average) and fewer look-backs.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void radix_onesweep_kernel(
    const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout, long n, int shift,
    uint32_t dmask, const uint32_t* __restrict__ gbase, uint64_t* __restrict__ status,
    uint64_t epoch, uint32_t* __restrict__ ticket, uint32_t* __restrict__ err) {
  constexpr int kThreads = WAVES * 64;
  constexpr int kTile = kThreads * kSortItems;
  constexpr int kWaveSpan = kSortItems * 64;
  static_assert(WAVES >= 4, "one thread per digit");
  __shared__ uint64_t s_k[kTile];
  __shared__ uint32_t s_wh[WAVES][kRadix];
  __shared__ uint32_t s_cnt[kRadix];
  __shared__ uint32_t s_toff[kRadix];
  __shared__ uint32_t s_g[kRadix];
  __shared__ uint32_t s_tile;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) s_tile = atomicAdd(ticket, 1u);
  for (int i = t; i < WAVES * kRadix; i += kThreads) (&s_wh[0][0])[i] = 0u;
  __syncthreads();
  const long tile = s_tile;
  const long base = tile * kTile;
  const int tile_n = (int)min((long)kTile, n - base);
  uint64_t k[kSortItems];
  const long wbase = base + (long)w * kWaveSpan;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = wbase + i * HBMR_WAVE + lane;
    k[i] = e < n ? kin[e] : 0ull;
  }
  const uint64_t lt = __lanemask_lt();
  uint32_t rank[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const bool valid = w * kWaveSpan + i * HBMR_WAVE + lane < tile_n;
    const uint32_t d = valid ? ((uint32_t)(k[i] >> shift) & dmask) : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t pre = __popcll(m & lt);
    uint32_t old = 0u;
    if (valid) old = s_wh[w][d];
    __builtin_amdgcn_wave_barrier();
    rank[i] = old + pre;
    if (valid && pre == 0) s_wh[w][d] = old + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (t < kRadix) {
    // thread t = digit t: publish the tile's count, look back for its prefix
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) cnt += s_wh[i][t];
    uint64_t* st = status + tile * kRadix + t;
    const uint64_t ep = epoch << 48;
    uint32_t excl = 0;
    if (tile == 0) {
      __hip_atomic_store(st, ep | kStInc | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(st, ep | kStAgg | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (long p = tile - 1; p >= 0; --p) {
        const uint64_t* q = status + p * kRadix + t;
        uint64_t v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (((v >> 48) != epoch || (v & kStKind) == 0u) && ++spins < kSpinLimit) {
          __builtin_amdgcn_s_sleep(1);
          v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if ((v >> 48) != epoch || (v & kStKind) == 0u) {
          atomicOr(err, 1u);
          break;
        }
        excl += (uint32_t)v;
        if ((v & kStKind) == kStInc) break;
      }
      __hip_atomic_store(st, ep | kStInc | (excl + cnt), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    s_g[t] = gbase[t] + excl;
    s_cnt[t] = cnt;
  }
  __syncthreads();
  if (w == 0) {
    // the tile's digit offsets: exclusive scan of 256 counts, 4 per lane
    const uint32_t a0 = s_cnt[4 * lane], a1 = s_cnt[4 * lane + 1], a2 = s_cnt[4 * lane + 2],
                   a3 = s_cnt[4 * lane + 3];
    const uint32_t sum = a0 + a1 + a2 + a3;
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(x, o);
      if (lane >= o) x += u;
    }
    const uint32_t e0 = x - sum;
    s_toff[4 * lane] = e0;
    s_toff[4 * lane + 1] = e0 + a0;
    s_toff[4 * lane + 2] = e0 + a0 + a1;
    s_toff[4 * lane + 3] = e0 + a0 + a1 + a2;
  }
  __syncthreads();
  if (t < kRadix) {
    // each wave's start inside the digit's run
    uint32_t run = s_toff[t];
#pragma unroll
    for (int i = 0; i < WAVES; ++i) {
      const uint32_t c = s_wh[i][t];
      s_wh[i][t] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    if (w * kWaveSpan + i * HBMR_WAVE + lane < tile_n)
      s_k[s_wh[w][((uint32_t)(k[i] >> shift) & dmask)] + rank[i]] = k[i];
  }
  __syncthreads();
  for (int j = t; j < tile_n; j += kThreads) {
    const uint64_t key = s_k[j];
    const uint32_t d = ((uint32_t)(key >> shift) & dmask);
    kout[(long)s_g[d] + (j - (long)s_toff[d])] = key;
  }
}

// ------------------------------------------------------------------------ TeraSort
// Affine LCG x' = a x + c (mod 2^32): state after `steps` from x0 by squaring.
__device__ __forceinline__ uint32_t lcg_jump(uint64_t steps, uint32_t x) {
  uint32_t ma = 3141592621u, mc = 663896637u;  // the map for 2^i steps
  uint32_t ra = 1u, rc = 0u;                    // accumulated map
  while (steps) {
    if (steps & 1) {
      rc = ma * rc + mc;
      ra = ma * ra;
    }
    mc = ma * mc + mc;
    ma = ma * ma;
    steps >>= 1;
  }
  return ra * x + rc;
}

// Record r (100 B): 10 key bytes (3 LCG draws at iterations 3r+1..3r+3, each
// /52 then 4 base-95 printable digits), the row id right-aligned in 10 chars,
// 78 filler letters starting at 'A' + (8r mod 26), "\r\n".
__global__ __launch_bounds__(256) void teragen_kernel(long first_row, long nrows,
                                                      uint8_t* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrows) return;
  const long row = first_row + i;
  uint8_t rec[100];
  uint32_t s = lcg_jump((uint64_t)row * 3u, 0u);
  uint8_t kb[12];
  for (int q = 0; q < 3; ++q) {
    s = 3141592621u * s + 663896637u;
    uint64_t temp = (uint64_t)s / 52u;
    kb[3 + 4 * q] = (uint8_t)(' ' + temp % 95);
    temp /= 95;
    kb[2 + 4 * q] = (uint8_t)(' ' + temp % 95);
    temp /= 95;
    kb[1 + 4 * q] = (uint8_t)(' ' + temp % 95);
    temp /= 95;
    kb[4 * q] = (uint8_t)(' ' + temp % 95);
  }
  for (int j = 0; j < 10; ++j) rec[j] = kb[j];
  // row id as Java's Integer.toString((int) rowId), right-aligned in 10 chars
  int32_t rid = (int32_t)row;
  char digits[12];
  int nd = 0;
  bool neg = rid < 0;
  uint32_t u = neg ? (uint32_t)(-(int64_t)rid) : (uint32_t)rid;
  do {
    digits[nd++] = (char)('0' + u % 10);
    u /= 10;
  } while (u);
  if (neg) digits[nd++] = '-';
  const int len = nd < 10 ? nd : 10;
  for (int j = 0; j < 10 - len; ++j) rec[10 + j] = ' ';
  for (int j = 0; j < len; ++j) rec[10 + (10 - len) + j] = (uint8_t)digits[nd - 1 - j];
  const int fb = (int)((row * 8) % 26);
  for (int q = 0; q < 7; ++q)
    for (int j = 0; j < 10; ++j) rec[20 + 10 * q + j] = (uint8_t)('A' + (fb + q) % 26);
  for (int j = 0; j < 8; ++j) rec[90 + j] = (uint8_t)('A' + (fb + 7) % 26);
  rec[98] = '\r';
  rec[99] = '\n';
  uint32_t* o = reinterpret_cast<uint32_t*>(out + i * 100);
  for (int j = 0; j < 25; ++j) {
    uint32_t wv;
    __builtin_memcpy(&wv, rec + 4 * j, 4);
    o[j] = wv;
  }
}

// hi = key bytes 0..7 big-endian, lo = bytes 8..9 (unsigned lexicographic order
// of the 10-byte key == order of (hi, lo))
__global__ __launch_bounds__(256) void tera_keys_kernel(const uint8_t* __restrict__ rec, long n,
                                                        int stride, uint64_t* __restrict__ hi,
                                                        uint64_t* __restrict__ lo) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = rec + i * stride;
  uint64_t h = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) h = (h << 8) | r[j];
  hi[i] = h;
  lo[i] = ((uint64_t)r[8] << 8) | r[9];
}

__global__ __launch_bounds__(256) void gather_u64_kernel(const uint64_t* __restrict__ src,
                                                         const uint32_t* __restrict__ perm, long n,
                                                         uint64_t* __restrict__ dst) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

// dst record i = src record perm[i]; records of `words` 4-byte words
__global__ __launch_bounds__(256) void gather_records_kernel(const uint32_t* __restrict__ src,
                                                             const uint32_t* __restrict__ perm,
                                                             long n, int words,
                                                             uint32_t* __restrict__ dst) {
  const long total = n * words;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long r = e / words;
    const int w = (int)(e - r * words);
    dst[e] = src[(long)perm[r] * words + w];
  }
}

// offsets[p] = first position whose (hi, lo) >= splitter p-1 (p = 1..R-1);
// offsets[0] = 0, offsets[R] = n
__global__ void split_offsets_kernel(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                                     long n, const uint64_t* __restrict__ shi,
                                     const uint64_t* __restrict__ slo, int nparts,
                                     long* __restrict__ offsets) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > nparts) return;
  if (p == 0) {
    offsets[0] = 0;
    return;
  }
  if (p == nparts) {
    offsets[nparts] = n;
    return;
  }
  const uint64_t kh = shi[p - 1], kl = slo[p - 1];
  long a = 0, b = n;
  while (a < b) {
    const long m = (a + b) >> 1;
    const bool less = hi[m] < kh || (hi[m] == kh && lo[m] < kl);
    if (less) a = m + 1; else b = m;
  }
  offsets[p] = a;
}

__global__ __launch_bounds__(256) void check_sorted_kernel(const uint64_t* __restrict__ hi,
                                                           const uint64_t* __restrict__ lo, long n,
                                                           unsigned long long* __restrict__ bad) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x + 1;
  bool b = false;
  if (i < n) b = hi[i - 1] > hi[i] || (hi[i - 1] == hi[i] && lo[i - 1] > lo[i]);
  const uint64_t m = __ballot(b);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

// One group of the one-rank reduce, after its sort: acc[0] += the records out
// of order (against the previous record; record 0 against the previous
// group's last key *ph / *pl when given), acc[1] += sum(hi + lo) mod 2^64 (the
// order-independent key checksum) — one pass, one atomic per wave, in place
// of an order check, two reductions and the elementwise seam check.
__global__ __launch_bounds__(256) void tera_group_stats_kernel(
    const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo, long n,
    const uint64_t* __restrict__ ph, const uint64_t* __restrict__ pl,
    unsigned long long* __restrict__ parts) {
  __shared__ unsigned long long s[2][4];
  uint64_t sum = 0, bad = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint64_t h = hi[i], l = lo[i];
    sum += h + l;
    if (i > 0) {
      const uint64_t h0 = hi[i - 1], l0 = lo[i - 1];
      bad += h0 > h || (h0 == h && l0 > l);
    } else if (ph != nullptr) {
      bad += *ph > h || (*ph == h && *pl > l);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o);
    bad += __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s[0][threadIdx.x >> 6] = bad;
    s[1][threadIdx.x >> 6] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = s[0][0] + s[0][1] + s[0][2] + s[0][3];
    parts[2 * blockIdx.x + 1] = s[1][0] + s[1][1] + s[1][2] + s[1][3];
  }
}

// Key words + range partition of each record: pid = number of splitters <= key
// (partition p holds keys in [split[p-1], split[p]), as split_offsets cuts a
// sorted run).  Splitters are staged in LDS once per workgroup; each workgroup
// then walks a grid-stride slice of the records.
constexpr int kMaxSplitters = 4096;

// An order-preserving map of a key's high word to a dense integer: with every
// key byte in [m, m + R) (the job's key alphabet: the maps measure the OR of
// all key bytes, so m = 0 and R = 2^bits — 128 for printable keys),
// v(h) = the 8 bytes of h as base-R digits, and the window (v(h) - vlo) >> sh
// for a group whose keys' v lie in [vlo, vlo + span), sh chosen so the
// window fits in 32 bits.  For printable keys (R = 128) the window keeps ~30
// bits of the group's spread where the raw top 32 bits of h keep ~22 (their
// bytes use 95 of 256 codes and the group fixes most of the first one).
// R = 256, m = 0, vlo = 0 is the plain shift h >> sh.
struct KeyWindow {
  uint64_t vlo;
  uint32_t m, R;
  int sh;
};

__device__ __forceinline__ uint64_t key_window(uint64_t h, const KeyWindow& kw) {
  uint64_t v = 0;
#pragma unroll
  for (int b = 7; b >= 0; --b) v = v * kw.R + (((h >> (8 * b)) & 0xFFu) - kw.m);
  return (v - kw.vlo) >> kw.sh;
}

// running OR of a high word's bytes (folded to one byte at the flush): every
// key byte is at most the OR of all of them, so [0, 2^bits(OR)) is an
// alphabet that holds them; and the key checksum sum(hi + lo) mod 2^64 the
// map reports.  A few VALU per record: this kernel is latency bound (the
// splitter search), and a per-record byte or word min / max cost it 2.4x.
__device__ __forceinline__ void byte_range(uint64_t h, uint32_t l, uint32_t& orb, uint64_t& sum) {
  orb |= (uint32_t)h | (uint32_t)(h >> 32);
  sum += h + l;
}

// the block's (OR of key bytes, key checksum) into parts[blockIdx] — no
// global atomics on one address (across 8 XCDs they serialise at ~0.2 us
// each: 16k blocks cost the kernel 3.5 ms); reduce_pairs_kernel folds them
__device__ __forceinline__ void flush_byte_range(uint32_t orb, uint64_t sum,
                                                 unsigned long long* s_ks,
                                                 unsigned long long* parts) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    orb |= __shfl_xor(orb, o);
    sum += __shfl_xor(sum, o);
  }
  orb |= orb >> 16;
  orb |= orb >> 8;
  if ((threadIdx.x & 63) == 0) {
    atomicOr(&s_ks[0], (unsigned long long)(orb & 0xFFu));
    atomicAdd(&s_ks[1], (unsigned long long)sum);
  }
  __syncthreads();
  if (threadIdx.x == 0 && parts != nullptr) {
    parts[2 * blockIdx.x] = s_ks[0];
    parts[2 * blockIdx.x + 1] = s_ks[1];
  }
}

// one workgroup: out[0] (|= or +=, by or0) and out[1] += over nparts pairs
__global__ __launch_bounds__(256) void reduce_pairs_kernel(const unsigned long long* __restrict__ parts,
                                                           long nparts, int or0,
                                                           unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s[2][4];
  unsigned long long a = 0, b = 0;
  for (long i = threadIdx.x; i < nparts; i += 256) {
    a = or0 ? (a | parts[2 * i]) : a + parts[2 * i];
    b += parts[2 * i + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long x = __shfl_xor(a, o);
    a = or0 ? (a | x) : a + x;
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s[0][threadIdx.x >> 6] = a;
    s[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long x = out[0], y = out[1];
    for (int w = 0; w < 4; ++w) {
      x = or0 ? (x | s[0][w]) : x + s[0][w];
      y += s[1][w];
    }
    out[0] = x;
    out[1] = y;
  }
}

__global__ __launch_bounds__(256) void tera_keys_part_kernel(
    const uint8_t* __restrict__ rec, long n, int stride, const uint64_t* __restrict__ shi,
    const uint64_t* __restrict__ slo, int nsplit, uint64_t* __restrict__ hi,
    uint64_t* __restrict__ lo, uint64_t* __restrict__ pid) {
  __shared__ uint64_t s_hi[kMaxSplitters];
  __shared__ uint16_t s_lo[kMaxSplitters];
  for (int j = threadIdx.x; j < nsplit; j += 256) {
    s_hi[j] = shi[j];
    s_lo[j] = (uint16_t)slo[j];
  }
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint8_t* r = rec + i * stride;
    uint64_t h = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) h = (h << 8) | r[j];
    const uint32_t l = ((uint32_t)r[8] << 8) | r[9];
    int a = 0, b = nsplit;
    while (a < b) {
      const int m = (a + b) >> 1;
      const bool le = s_hi[m] < h || (s_hi[m] == h && s_lo[m] <= l);
      if (le) a = m + 1; else b = m;
    }
    hi[i] = h;
    lo[i] = l;
    pid[i] = (uint64_t)a;
  }
}

// Concatenate S pieces: piece s is [starts[s], starts[s] + len_s) of its split's
// (hi, lo, row) arrays, placed at [prefix[s], prefix[s+1]) of the output; the
// output also records which split each element came from.  hi/lo (in and out)
// may be null (records-only collection for the shuffle).
__global__ __launch_bounds__(256) void tera_collect_kernel(
    const uint64_t* const* __restrict__ his, const uint64_t* const* __restrict__ los,
    const uint32_t* const* __restrict__ rows, const long* __restrict__ starts,
    const long* __restrict__ prefix, int S, long n, uint64_t* __restrict__ ohi,
    uint64_t* __restrict__ olo, uint32_t* __restrict__ osplit, uint32_t* __restrict__ orow) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    int a = 0, b = S;          // largest s with prefix[s] <= i
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (prefix[m] <= i) a = m; else b = m;
    }
    const long j = starts[a] + (i - prefix[a]);
    if (ohi) ohi[i] = his[a][j];
    if (olo) olo[i] = los[a][j];
    osplit[i] = (uint32_t)a;
    orow[i] = rows[a][j];
  }
}

// Static-shape shuffle send layout (the TeraSort shuffle waves): W destination
// slots of C entries.  Entry j of slot d is element j of destination d's pieces
// — piece s is [starts[s*W + d], +len) of split s's partition-ordered rows,
// placed at [pre[d*(S+1) + s], pre[d*(S+1) + s + 1]) — while j < min(pre[d*(S+1)
// + S], C); entries past the count get split = kNoSplit (the gather skips them).
// Every offset is read on the device: no host round trip between the maps'
// partition offsets and the all-to-all that sends the slots.
constexpr uint32_t kNoSplit = 0xFFFFFFFFu;

__global__ __launch_bounds__(256) void tera_collect_slots_kernel(
    const uint32_t* const* __restrict__ rows, const long* __restrict__ starts,
    const long* __restrict__ pre, int S, int W, long C, uint32_t* __restrict__ osplit,
    uint32_t* __restrict__ orow) {
  const long n = (long)W * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int d = (int)(i / C);
    const long j = i - (long)d * C;
    const long* pd = pre + (long)d * (S + 1);
    if (j >= pd[S]) {
      osplit[i] = kNoSplit;
      orow[i] = 0u;
      continue;
    }
    int a = 0, b = S;          // largest s with pd[s] <= j
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (pd[m] <= j) a = m; else b = m;
    }
    osplit[i] = (uint32_t)a;
    orow[i] = rows[a][starts[(long)a * W + d] + (j - pd[a])];
  }
}

// ---- TeraSort map v3: partition without a sort ------------------------------
// (A) key words + partition id of every record, and the partition sizes: a
// per-workgroup LDS histogram flushed with one global add per touched bin.
__global__ __launch_bounds__(256) void tera_part_count_kernel(
    const uint8_t* __restrict__ rec, long n, int stride, const uint64_t* __restrict__ shi,
    const uint64_t* __restrict__ slo, int nsplit, uint64_t* __restrict__ hi,
    uint64_t* __restrict__ lo, uint16_t* __restrict__ pid, unsigned int* __restrict__ counts,
    unsigned long long* __restrict__ kmm) {
  __shared__ uint64_t s_hi[kMaxSplitters];
  __shared__ uint16_t s_lo[kMaxSplitters];
  __shared__ unsigned int s_cnt[kMaxSplitters + 1];
  __shared__ unsigned long long s_ks[2];
  uint32_t korb = 0u;
  uint64_t ksum = 0;
  const int nparts = nsplit + 1;
  for (int j = threadIdx.x; j < nsplit; j += 256) {
    s_hi[j] = shi[j];
    s_lo[j] = (uint16_t)slo[j];
  }
  for (int j = threadIdx.x; j < nparts; j += 256) s_cnt[j] = 0u;
  if (threadIdx.x == 0) {
    s_ks[0] = 0ull;
    s_ks[1] = 0ull;
  }
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint8_t* r = rec + i * stride;
    uint64_t h = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) h = (h << 8) | r[j];
    const uint32_t l = ((uint32_t)r[8] << 8) | r[9];
    int a = 0, b = nsplit;
    while (a < b) {
      const int m = (a + b) >> 1;
      const bool le = s_hi[m] < h || (s_hi[m] == h && s_lo[m] <= l);
      if (le) a = m + 1; else b = m;
    }
    hi[i] = h;
    lo[i] = l;
    pid[i] = (uint16_t)a;
    atomicAdd(&s_cnt[a], 1u);
    byte_range(h, l, korb, ksum);
  }
  flush_byte_range(korb, ksum, s_ks, kmm);
  for (int j = threadIdx.x; j < nparts; j += 256)
    if (s_cnt[j]) atomicAdd(&counts[j], s_cnt[j]);
}

// exclusive scan of the partition sizes (one workgroup; nparts <= 4097)
__global__ __launch_bounds__(1024) void tera_part_offsets_kernel(
    const unsigned int* __restrict__ counts, int nparts, unsigned int* __restrict__ cursor,
    long* __restrict__ offsets) {
  __shared__ long s_w[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int kPer = 5;   // 1024 * 5 >= 4097
  long v[kPer], sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int idx = t * kPer + j;
    v[j] = idx < nparts ? (long)counts[idx] : 0;
    sum += v[j];
  }
  long x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long u = __shfl_up(x, o);
    if (lane >= o) x += u;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  long run = x - sum;
  for (int i = 0; i < w; ++i) run += s_w[i];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int idx = t * kPer + j;
    if (idx < nparts) {
      offsets[idx] = run;
      cursor[idx] = (unsigned int)run;
    }
    run += v[j];
    if (idx == nparts - 1) offsets[nparts] = run;
  }
}

// (B) scatter (hi, lo, row) into partition order.  Each workgroup takes a tile
// of kSortTile records, ranks them per partition in LDS, reserves one range per
// touched partition from the global cursors, and writes.  Order inside a
// partition follows the reservation order (the reduce sorts by key anyway).
__global__ __launch_bounds__(kSortThreads) void tera_part_scatter_kernel(
    const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
    const uint16_t* __restrict__ pid, long n, int nparts, unsigned int* __restrict__ cursor,
    uint64_t* __restrict__ ohi, uint64_t* __restrict__ olo, uint32_t* __restrict__ orow) {
  __shared__ unsigned int s_cnt[kMaxSplitters + 1];
  const int t = threadIdx.x;
  const long base = (long)blockIdx.x * kSortTile;
  for (int j = t; j < nparts; j += kSortThreads) s_cnt[j] = 0u;
  __syncthreads();
  unsigned int loc[kSortItems];
  uint16_t p[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = base + (long)i * kSortThreads + t;
    if (e < n) {
      p[i] = pid[e];
      loc[i] = atomicAdd(&s_cnt[p[i]], 1u);
    }
  }
  __syncthreads();
  for (int j = t; j < nparts; j += kSortThreads) {
    const unsigned int c = s_cnt[j];
    s_cnt[j] = c ? atomicAdd(&cursor[j], c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = base + (long)i * kSortThreads + t;
    if (e < n) {
      const long d = (long)s_cnt[p[i]] + loc[i];
      ohi[d] = hi[e];
      olo[d] = lo[e];
      orow[d] = (uint32_t)e;
    }
  }
}

// (A') key / partition / count with the key read as 3 dwords (the record
// stride is a multiple of 4: bytes 0-11 of every record are 4-B aligned)
// instead of 10 byte loads per record.
__global__ __launch_bounds__(256) void tera_part_count_w_kernel(
    const uint32_t* __restrict__ rec, long n, int stride_words, const uint64_t* __restrict__ shi,
    const uint64_t* __restrict__ slo, int nsplit, uint64_t* __restrict__ hi,
    uint64_t* __restrict__ lo, uint16_t* __restrict__ pid, unsigned int* __restrict__ counts,
    unsigned long long* __restrict__ kmm) {
  // LDS sized by the splitter count (part_count_w_lds), not a static
  // 4096-entry table (56 KB: two workgroups per CU).  The kernel reads about
  // every sector of the records (a 12-byte key every 100 bytes), so it runs
  // near the copy rate; a 12-bit prefix table that spared 98 % of the
  // splitter searches measured no faster.
  extern __shared__ __align__(16) unsigned char s_dyn[];
  uint64_t* s_hi = reinterpret_cast<uint64_t*>(s_dyn);
  unsigned int* s_cnt = reinterpret_cast<unsigned int*>(s_hi + nsplit);
  uint16_t* s_lo = reinterpret_cast<uint16_t*>(s_cnt + nsplit + 1);
  __shared__ unsigned long long s_ks[2];
  uint32_t korb = 0u;
  uint64_t ksum = 0;
  const int nparts = nsplit + 1;
  for (int j = threadIdx.x; j < nsplit; j += 256) {
    s_hi[j] = shi[j];
    s_lo[j] = (uint16_t)slo[j];
  }
  for (int j = threadIdx.x; j < nparts; j += 256) s_cnt[j] = 0u;
  if (threadIdx.x == 0) {
    s_ks[0] = 0ull;
    s_ks[1] = 0ull;
  }
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint32_t* r = rec + i * stride_words;
    const uint32_t w0 = r[0], w1 = r[1], w2 = r[2];
    const uint64_t h = ((uint64_t)__builtin_bswap32(w0) << 32) | __builtin_bswap32(w1);
    const uint32_t l = ((w2 & 0xFFu) << 8) | ((w2 >> 8) & 0xFFu);
    int a = 0, b = nsplit;
    while (a < b) {
      const int m = (a + b) >> 1;
      const bool le = s_hi[m] < h || (s_hi[m] == h && s_lo[m] <= l);
      if (le) a = m + 1; else b = m;
    }
    hi[i] = h;
    lo[i] = l;
    pid[i] = (uint16_t)a;
    atomicAdd(&s_cnt[a], 1u);
    byte_range(h, l, korb, ksum);
  }
  flush_byte_range(korb, ksum, s_ks, kmm);
  for (int j = threadIdx.x; j < nparts; j += 256)
    if (s_cnt[j]) atomicAdd(&counts[j], s_cnt[j]);
}

// dst record i = record row[k] of split split[k], k = perm ? perm[i] : i, with
// U records per lane in flight: the index loads of all U records are issued,
// then their words, then the stores, so each lane keeps U independent random
// reads outstanding (the v1 loop waited on one record at a time).  Lane t
// moves word t % words of record t / words; iteration j of a block covers
// records r0 + j * stride, so the stores of every j stay coalesced.
template <int U>
__global__ __launch_bounds__(256) void gather_records_multi_v3_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ split,
    const uint32_t* __restrict__ row, const uint32_t* __restrict__ perm, long n, int words,
    uint32_t* __restrict__ dst) {
  const int rpb = 256 / words;
  const int t = threadIdx.x;
  if (t >= rpb * words) return;
  const int lr = t / words;
  const int w = t - lr * words;
  const long stride = (long)gridDim.x * rpb;
  for (long r0 = (long)blockIdx.x * rpb + lr; r0 < n; r0 += stride * U) {
    const uint32_t* src[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      src[j] = nullptr;
      if (r < n) {
        const long k = perm ? (long)perm[r] : r;
        const uint32_t sp = split[k];
        if (sp != kNoSplit) src[j] = bases[sp] + (long)row[k] * words;
      }
    }
    uint32_t v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = src[j] ? src[j][w] : 0u;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      if (src[j]) dst[r * words + w] = v[j];
    }
  }
}

// After a sort by hi only: order each run of equal hi by lo (insertion sort,
// carrying perm).  Runs are rare for TeraSort keys (8 of 10 key bytes in hi);
// a run longer than kTieRun is left alone and flagged, and the caller falls
// back to the full 80-bit sort.
constexpr int kTieRun = 64;

__global__ __launch_bounds__(256) void tera_tie_fix_kernel(const uint64_t* __restrict__ hi,
                                                           uint64_t* __restrict__ lo,
                                                           uint32_t* __restrict__ perm, long n,
                                                           unsigned int* __restrict__ flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n - 1) return;
  const uint64_t h = hi[i];
  if (hi[i + 1] != h || (i > 0 && hi[i - 1] == h)) return;   // not the start of a run
  long e = i + 1;
  while (e < n && hi[e] == h && e - i < kTieRun) ++e;
  if (e < n && hi[e] == h) {
    atomicOr(flag, 1u);
    return;
  }
  for (long a = i + 1; a < e; ++a) {
    const uint64_t kl = lo[a];
    const uint32_t kp = perm[a];
    long b = a - 1;
    while (b >= i && lo[b] > kl) {
      lo[b + 1] = lo[b];
      perm[b + 1] = perm[b];
      --b;
    }
    lo[b + 1] = kl;
    perm[b + 1] = kp;
  }
}

// ---- K8: merge of sorted runs (merge path) -----------------------------------
// Merge two sorted runs A[0,na) and B[0,nb) of (hi, lo) keys with u32 payloads
// (stable: A before B on equal keys).  Thread t owns output [t*kMergeItems,
// (t+1)*kMergeItems): it finds where that diagonal crosses the merge path by
// binary search, then merges its items sequentially.  Runs are bound by HBM
// bandwidth (each element read once, written once; the search touches
// log2(n) elements per thread).
constexpr int kMergeItems = 16;

__device__ __forceinline__ bool key_lt(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
  return ah < bh || (ah == bh && al < bl);
}

__global__ __launch_bounds__(256) void merge_path_kernel(
    const uint64_t* __restrict__ ahi, const uint64_t* __restrict__ alo,
    const uint32_t* __restrict__ av, long na, const uint64_t* __restrict__ bhi,
    const uint64_t* __restrict__ blo, const uint32_t* __restrict__ bv, long nb,
    uint64_t* __restrict__ ohi, uint64_t* __restrict__ olo, uint32_t* __restrict__ ov) {
  const long n = na + nb;
  const long d = ((long)blockIdx.x * 256 + threadIdx.x) * kMergeItems;
  if (d >= n) return;
  // largest i in [max(0, d-nb), min(d, na)] with A[i-1] <= B[d-i] (A wins ties)
  long lo_i = d > nb ? d - nb : 0, hi_i = d < na ? d : na;
  while (lo_i < hi_i) {
    const long i = (lo_i + hi_i + 1) >> 1;
    const long j = d - i;
    // i is feasible iff A[i-1] <= B[j] (j < nb) — i.e. not B[j] < A[i-1]
    if (j >= nb || !key_lt(bhi[j], blo[j], ahi[i - 1], alo[i - 1])) lo_i = i;
    else hi_i = i - 1;
  }
  long i = lo_i, j = d - lo_i;
  const long end = d + kMergeItems < n ? d + kMergeItems : n;
  for (long o = d; o < end; ++o) {
    bool take_a;
    if (i >= na) take_a = false;
    else if (j >= nb) take_a = true;
    else take_a = !key_lt(bhi[j], blo[j], ahi[i], alo[i]);
    if (take_a) {
      ohi[o] = ahi[i];
      olo[o] = alo[i];
      ov[o] = av[i];
      ++i;
    } else {
      ohi[o] = bhi[j];
      olo[o] = blo[j];
      ov[o] = bv[j];
      ++j;
    }
  }
}

// ---- TeraSort reduce v4: packed record ids ------------------------------------
// A group's records are named by a 32-bit gid = split << 24 | row (splits < 256,
// rows < 2^24): the key sort carries the gid itself, so the record gather makes
// ONE dependent index load per record (v3: perm, then split and row).
__global__ __launch_bounds__(256) void tera_collect_gid_kernel(
    const uint64_t* const* __restrict__ his, const uint32_t* const* __restrict__ rows,
    const long* __restrict__ starts, const long* __restrict__ prefix, int S, long n, int pack,
    KeyWindow kw, uint64_t* __restrict__ ohi, uint32_t* __restrict__ ogid) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    int a = 0, b = S;          // largest s with prefix[s] <= i
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (prefix[m] <= i) a = m; else b = m;
    }
    const long j = starts[a] + (i - prefix[a]);
    const uint32_t g = ((uint32_t)a << 24) | rows[a][j];
    if (pack) {
      // one sortable word: the key's 32-bit window above the record id
      ohi[i] = ((key_window(his[a][j], kw) & 0xFFFFFFFFull) << 32) | g;
    } else {
      ohi[i] = his[a][j];
      ogid[i] = g;
    }
  }
}

// (with key outputs: the lanes holding words 0-2 of a record also store its
// key — hi as two byte-swapped halves, lo from word 2 — so the sorted keys
// need no second pass over the gathered records)
template <int U>
__global__ __launch_bounds__(256) void gather_records_gid_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ gid,
    const uint64_t* packed, long n,
    int words, uint32_t* __restrict__ dst, uint32_t* __restrict__ khi,
    uint64_t* __restrict__ klo, uint32_t* __restrict__ kwin) {
  const int rpb = 256 / words;
  const int t = threadIdx.x;
  if (t >= rpb * words) return;
  const int lr = t / words;
  const int w = t - lr * words;
  const long stride = (long)gridDim.x * rpb;
  for (long r0 = (long)blockIdx.x * rpb + lr; r0 < n; r0 += stride * U) {
    const uint32_t* src[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      src[j] = nullptr;
      if (r < n) {
        const uint32_t g = packed ? (uint32_t)packed[r] : gid[r];
        src[j] = bases[g >> 24] + (long)(g & 0xFFFFFFu) * words;
      }
    }
    uint32_t v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = src[j] ? src[j][w] : 0u;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      if (r < n) {
        dst[r * words + w] = v[j];
      }
    }
    if (khi != nullptr && w < 3) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const long r = r0 + j * stride;
        if (r >= n) continue;
        if (w < 2) {
          khi[2 * r + 1 - w] = __builtin_bswap32(v[j]);  // hi = bytes 0-7, big-endian
        } else {
          klo[r] = ((uint64_t)(v[j] & 0xFFu) << 8) | ((v[j] >> 8) & 0xFFu);  // bytes 8-9
        }
      }
    }
  }
}

// The record gather in 16-B pieces (v2, default): a record of W words is
// moved by L = ceil(W / 4) lanes, lane c the 16 B at word 4c (the last lane
// the remaining 1-4 words) — 7 lanes per 100-B TeraSort record instead of 25,
// so a wave keeps 9 records x U in flight per round instead of 2.5 x U, with
// 16-B loads/stores at the record's 4-B alignment (global memory takes
// dword-aligned vector accesses).  The lane holding words 0-3 also writes the
// record's key (hi byte-swapped from words 0-1, lo from word 2's bytes 8-9).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef u32x4_t __attribute__((aligned(4))) u32x4_a4;
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef u32x2_t __attribute__((aligned(4))) u32x2_a4;

template <int U>
__global__ __launch_bounds__(256) void gather_records_gid16_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ gid,
    const uint64_t* packed, long n,
    int words, uint32_t* __restrict__ dst, uint32_t* __restrict__ khi,
    uint64_t* __restrict__ klo, uint32_t* __restrict__ kwin) {
  const int L = (words + 3) >> 2;            // lanes per record
  const int rpw = HBMR_WAVE / L;             // records per wave
  const int lane = threadIdx.x & (HBMR_WAVE - 1), wave = threadIdx.x / HBMR_WAVE;
  if (lane >= rpw * L) return;               // (no barrier in this kernel)
  const int lr = lane / L;
  const int c = lane - lr * L;
  const int w0 = 4 * c;                      // first word of this lane's piece
  const int nw = words - w0 < 4 ? words - w0 : 4;
  const long rpb = (long)rpw * (256 / HBMR_WAVE);
  const long stride = (long)gridDim.x * rpb;
  for (long r0 = (long)blockIdx.x * rpb + wave * rpw + lr; r0 < n; r0 += stride * U) {
    const uint32_t* src[U];
    uint32_t win[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      src[j] = nullptr;
      win[j] = 0u;
      if (r < n) {
        uint32_t g;
        if (packed) {
          const uint64_t pk = packed[r];
          g = (uint32_t)pk;
          win[j] = (uint32_t)(pk >> 32);
        } else {
          g = gid[r];
        }
        src[j] = bases[g >> 24] + (long)(g & 0xFFFFFFu) * words + w0;
      }
    }
    u32x4_t v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      v[j] = u32x4_t{0u, 0u, 0u, 0u};
      if (!src[j]) continue;
      if (nw == 4) {
        v[j] = *reinterpret_cast<const u32x4_a4*>(src[j]);
      } else if (nw == 2) {
        const u32x2_t t = *reinterpret_cast<const u32x2_a4*>(src[j]);
        v[j].x = t.x;
        v[j].y = t.y;
      } else {
        v[j].x = src[j][0];
        if (nw > 1) v[j].y = src[j][1];
        if (nw > 2) v[j].z = src[j][2];
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      if (r >= n) continue;
      uint32_t* d = dst + r * words + w0;
      if (nw == 4) {
        *reinterpret_cast<u32x4_a4*>(d) = v[j];
      } else if (nw == 2) {
        *reinterpret_cast<u32x2_a4*>(d) = u32x2_t{v[j].x, v[j].y};
      } else {
        d[0] = v[j].x;
        if (nw > 1) d[1] = v[j].y;
        if (nw > 2) d[2] = v[j].z;
      }
      if (khi != nullptr && c == 0) {
        khi[2 * r + 1] = __builtin_bswap32(v[j].x);   // hi = bytes 0-7, big-endian
        khi[2 * r] = __builtin_bswap32(v[j].y);
        klo[r] = ((uint64_t)(v[j].z & 0xFFu) << 8) | ((v[j].z >> 8) & 0xFFu);   // bytes 8-9
        if (kwin != nullptr) kwin[r] = win[j];    // the sort window, for the tie fix
      }
    }
  }
}

// After the sort on a window of the high key word and the record gather:
// order each run of an equal sorted prefix (hi >> shift) by the full key
// (hi, lo), moving hi, lo and the (already gathered) records themselves.
// Two passes, one thread per record: (1) a record in a run ranks itself
// among the run's members by (hi, lo, position) and, if its place changes,
// copies itself to a compact scratch slot with its destination; (2) every
// scratch slot is written to its destination.  Runs longer than kTieRun (or
// more moved records than the scratch holds) are flagged for the full-key
// path.  A 32-bit window over ~12M keys leaves equal prefixes on a few
// percent of them, in pairs and triples.
__global__ __launch_bounds__(256) void tera_tie_rank_kernel(
    const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
    const uint32_t* __restrict__ rec, long n, int words, KeyWindow kw,
    const uint32_t* __restrict__ win, long cap, unsigned int* __restrict__ cnt,
    uint32_t* __restrict__ sdst, uint64_t* __restrict__ shi, uint64_t* __restrict__ slo,
    uint32_t* __restrict__ srec, unsigned int* __restrict__ flag) {
  const long j = (long)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  // the records' windows: as the gather stored them, else recomputed from hi
  auto wnd = [&](long x) -> uint64_t { return win ? (uint64_t)win[x] : key_window(hi[x], kw); };
  const uint64_t h = wnd(j);
  const bool prev = j > 0 && wnd(j - 1) == h;
  const bool next = j + 1 < n && wnd(j + 1) == h;
  if (!prev && !next) return;
  const uint64_t hj = hi[j], lj = lo[j];
  long s0 = j, e = j + 1;
  while (s0 > 0 && wnd(s0 - 1) == h && j - s0 < kTieRun) --s0;
  while (e < n && wnd(e) == h && e - j < kTieRun) ++e;
  if ((s0 > 0 && wnd(s0 - 1) == h) || (e < n && wnd(e) == h) || e - s0 > kTieRun) {
    atomicOr(flag, 1u);
    return;
  }
  long rank = 0;
  for (long k = s0; k < e; ++k) {
    const uint64_t hk = hi[k], lk = lo[k];
    rank += hk < hj || (hk == hj && (lk < lj || (lk == lj && k < j)));
  }
  const long d = s0 + rank;
  if (d == j) return;
  const unsigned int slot = atomicAdd(cnt, 1u);
  if ((long)slot >= cap) {
    atomicOr(flag, 1u);
    return;
  }
  sdst[slot] = (uint32_t)d;
  shi[slot] = hj;
  slo[slot] = lj;
  for (int w = 0; w < words; ++w) srec[(long)slot * words + w] = rec[j * words + w];
}

__global__ __launch_bounds__(256) void tera_tie_move_kernel(
    uint64_t* __restrict__ hi, uint64_t* __restrict__ lo, uint32_t* __restrict__ rec, int words,
    long cap, const unsigned int* __restrict__ cnt, const uint32_t* __restrict__ sdst,
    const uint64_t* __restrict__ shi, const uint64_t* __restrict__ slo,
    const uint32_t* __restrict__ srec) {
  const long m = min((long)*cnt, cap);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    const long d = sdst[i];
    hi[d] = shi[i];
    lo[d] = slo[i];
    for (int w = 0; w < words; ++w) rec[d * words + w] = srec[i * words + w];
  }
}

inline long ceil_div(long a, long b) { return (a + b - 1) / b; }

int g_onesweep_waves = 8;  // waves per onesweep tile (hbmr_radix_set_onesweep_waves, A/B)
int g_gather_unroll = 2;   // records in flight per lane group (hbmr_gather_set_unroll, A/B)

}  // namespace

extern "C" {

long hbmr_radix_sort_workspace_bytes(long n) {
  const long ntiles = std::max(1L, ceil_div(n, kSortTile));
  return (long)(kRadix * ntiles + kRadix) * 4;
}

// Sort (keys, vals) by key bits [begin_bit, end_bit) (8-bit digits, LSD, stable).
// keys/vals hold the input and receive the output; tkeys/tvals are scratch of
// the same size.  vals == nullptr sorts (key, original index) into tvals-free
// mode is not supported: pass a values array (e.g. iota) — see hbmr.ops.sort.
int hbmr_radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t* tkeys, uint32_t* tvals,
                              long n, int begin_bit, int end_bit, void* ws, long ws_bytes,
                              hipStream_t st) {
  if (n <= 1) return 0;
  if (n >= (1L << 32) || begin_bit < 0 || end_bit > 64 || begin_bit >= end_bit)
    return (int)hipErrorInvalidValue;
  const long ntiles = ceil_div(n, kSortTile);
  if (ws_bytes < hbmr_radix_sort_workspace_bytes(n)) return (int)hipErrorInvalidValue;
  uint32_t* hist = reinterpret_cast<uint32_t*>(ws);
  uint32_t* totals = hist + (long)kRadix * ntiles;
  uint64_t* ka = keys;
  uint32_t* va = vals;
  uint64_t* kb = tkeys;
  uint32_t* vb = tvals;
  int passes = 0;
  for (int shift = begin_bit; shift < end_bit; shift += 8, ++passes) {
    hipLaunchKernelGGL(radix_hist_v2_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st,
                       ka, n, shift, ntiles, hist);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(kRadix), dim3(1024), 0, st, hist, ntiles, totals);
    hipLaunchKernelGGL(radix_scatter_v2_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st,
                       ka, va, kb, vb, n, shift, ntiles, hist, totals);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  if (passes & 1) {
    HBMR_RETURN_IF_ERROR(hipMemcpyAsync(keys, ka, n * 8, hipMemcpyDeviceToDevice, st));
    HBMR_RETURN_IF_ERROR(hipMemcpyAsync(vals, va, n * 4, hipMemcpyDeviceToDevice, st));
  }
  return (int)hipGetLastError();
}

long hbmr_radix_onesweep_workspace_bytes(long n) {
  return (long)(kMaxPasses * kRadix + kMaxPasses + 1) * 4;
}

long hbmr_radix_onesweep_status_bytes(long n) {
  return std::max(1L, ceil_div(n, kSortTile)) * kRadix * 8;   // tiles of >= 4096 keys
}

// Sort uint64 keys by bits [begin_bit, end_bit) (8-bit digits, LSD, stable),
// keys only, onesweep: one histogram read for all digits, then per digit one
// look-back scatter.  keys holds the input and receives the output; tkeys is
// scratch of the same size; *err (device) is set if a look-back timed out.
// status (hbmr_radix_onesweep_status_bytes) is reused across calls on one
// stream: each pass tags its words with a fresh epoch from *epoch (a host
// counter; at 0 or 0xFFFF the status is zeroed first and the count restarts).
// copy_back = 0 leaves an odd pass count's result in tkeys.
int hbmr_radix_sort_keys_u64(uint64_t* keys, uint64_t* tkeys, long n, int begin_bit, int end_bit,
                             void* ws, long ws_bytes, void* status, long status_bytes,
                             unsigned int* epoch, uint32_t* err, int copy_back, hipStream_t st) {
  if (n <= 1) return 0;
  const int passes = (end_bit - begin_bit + 7) / 8;
  if (n >= (1L << 30) || begin_bit < 0 || end_bit > 64 || begin_bit >= end_bit ||
      passes > kMaxPasses || epoch == nullptr)
    return (int)hipErrorInvalidValue;
  if (ws_bytes < hbmr_radix_onesweep_workspace_bytes(n) ||
      status_bytes < hbmr_radix_onesweep_status_bytes(n))
    return (int)hipErrorInvalidValue;
  const long ntiles = ceil_div(n, kSortTile);
  uint32_t* ghist = reinterpret_cast<uint32_t*>(ws);
  uint32_t* tickets = ghist + kMaxPasses * kRadix;
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(ghist, 0, (kMaxPasses * kRadix + kMaxPasses) * 4, st));
  const long hgrid = std::min<long>(ntiles, 2048);
  hipLaunchKernelGGL(radix_hist_all_kernel, dim3((unsigned)hgrid), dim3(kSortThreads), 0, st,
                     keys, n, begin_bit, end_bit, passes, ghist);
  hipLaunchKernelGGL(radix_bases_kernel, dim3((unsigned)passes), dim3(kSortThreads), 0, st, ghist);
  uint64_t* ka = keys;
  uint64_t* kb = tkeys;
  const int waves = g_onesweep_waves;
  const long tiles = ceil_div(n, (long)waves * 64 * kSortItems);
  for (int p = 0; p < passes; ++p) {
    if (*epoch == 0 || *epoch >= 0xFFFFu) {
      HBMR_RETURN_IF_ERROR(hipMemsetAsync(status, 0, status_bytes, st));
      *epoch = 0;
    }
    const uint64_t ep = ++*epoch;
    const int sh = begin_bit + 8 * p;
    const uint32_t dm = (1u << std::min(8, end_bit - begin_bit - 8 * p)) - 1u;
    if (waves == 16)
      hipLaunchKernelGGL(radix_onesweep_kernel<16>, dim3((unsigned)tiles), dim3(1024), 0, st, ka,
                         kb, n, sh, dm, ghist + p * kRadix, reinterpret_cast<uint64_t*>(status),
                         ep, tickets + p, err);
    else if (waves == 8)
      hipLaunchKernelGGL(radix_onesweep_kernel<8>, dim3((unsigned)tiles), dim3(512), 0, st, ka, kb,
                         n, sh, dm, ghist + p * kRadix, reinterpret_cast<uint64_t*>(status), ep,
                         tickets + p, err);
    else
      hipLaunchKernelGGL(radix_onesweep_kernel<4>, dim3((unsigned)tiles), dim3(256), 0, st, ka, kb,
                         n, sh, dm, ghist + p * kRadix, reinterpret_cast<uint64_t*>(status), ep,
                         tickets + p, err);
    std::swap(ka, kb);
  }
  if ((passes & 1) && copy_back)
    HBMR_RETURN_IF_ERROR(hipMemcpyAsync(keys, ka, n * 8, hipMemcpyDeviceToDevice, st));
  return (int)hipGetLastError();
}

int hbmr_teragen(long first_row, long nrows, void* out, hipStream_t st) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(teragen_kernel, dim3((unsigned)ceil_div(nrows, 256)), dim3(256), 0, st,
                     first_row, nrows, reinterpret_cast<uint8_t*>(out));
  return (int)hipGetLastError();
}

int hbmr_tera_keys(const void* records, long n, int stride, uint64_t* hi, uint64_t* lo,
                   hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(tera_keys_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint8_t*>(records), n, stride, hi, lo);
  return (int)hipGetLastError();
}

int hbmr_gather_u64(const uint64_t* src, const uint32_t* perm, long n, uint64_t* dst,
                    hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_u64_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, src,
                     perm, n, dst);
  return (int)hipGetLastError();
}

int hbmr_gather_records(const void* src, const uint32_t* perm, long n, int record_bytes, void* dst,
                        hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4) return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  const long grid = std::min<long>(ceil_div(n * words, 256), 1L << 20);
  hipLaunchKernelGGL(gather_records_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t*>(src), perm, n, words,
                     reinterpret_cast<uint32_t*>(dst));
  return (int)hipGetLastError();
}

int hbmr_split_offsets(const uint64_t* hi, const uint64_t* lo, long n, const uint64_t* shi,
                       const uint64_t* slo, int nparts, long* offsets, hipStream_t st) {
  hipLaunchKernelGGL(split_offsets_kernel, dim3((unsigned)ceil_div(nparts + 1, 256)), dim3(256), 0,
                     st, hi, lo, n, shi, slo, nparts, offsets);
  return (int)hipGetLastError();
}

int hbmr_check_sorted(const uint64_t* hi, const uint64_t* lo, long n, unsigned long long* bad,
                      hipStream_t st) {
  if (n <= 1) return 0;
  hipLaunchKernelGGL(check_sorted_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, hi,
                     lo, n, bad);
  return (int)hipGetLastError();
}

// acc: device u64[2 + 2 * 1024]: (out of order, checksum) accumulators, then
// the per-block partials
int hbmr_tera_group_stats(const uint64_t* hi, const uint64_t* lo, long n, const uint64_t* ph,
                          const uint64_t* pl, unsigned long long* acc, hipStream_t st) {
  if (n <= 0) return 0;
  if ((ph == nullptr) != (pl == nullptr)) return (int)hipErrorInvalidValue;
  const long grid = std::min<long>(ceil_div(n, 256 * 4), 1024);
  hipLaunchKernelGGL(tera_group_stats_kernel, dim3((unsigned)grid), dim3(256), 0, st, hi, lo, n,
                     ph, pl, acc + 2);
  hipLaunchKernelGGL(reduce_pairs_kernel, dim3(1), dim3(256), 0, st, acc + 2, grid, 0, acc);
  return (int)hipGetLastError();
}

int hbmr_tera_keys_part(const void* records, long n, int stride, const uint64_t* shi,
                        const uint64_t* slo, int nsplit, uint64_t* hi, uint64_t* lo,
                        uint64_t* pid, hipStream_t st) {
  if (n <= 0) return 0;
  if (nsplit < 0 || nsplit > kMaxSplitters) return (int)hipErrorInvalidValue;
  const long grid = std::min<long>(ceil_div(n, 256), 256L * 64);
  hipLaunchKernelGGL(tera_keys_part_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint8_t*>(records), n, stride, shi, slo, nsplit, hi,
                     lo, pid);
  return (int)hipGetLastError();
}

int hbmr_tera_collect_slots(const uint32_t* const* rows, const long* starts, const long* pre,
                            int S, int W, long C, uint32_t* osplit, uint32_t* orow,
                            hipStream_t st) {
  if (W <= 0 || C <= 0) return 0;
  if (S <= 0) return (int)hipErrorInvalidValue;
  const long grid = std::min<long>(ceil_div((long)W * C, 256), 256L * 256);
  hipLaunchKernelGGL(tera_collect_slots_kernel, dim3((unsigned)grid), dim3(256), 0, st, rows,
                     starts, pre, S, W, C, osplit, orow);
  return (int)hipGetLastError();
}

int hbmr_tera_collect(const uint64_t* const* his, const uint64_t* const* los,
                      const uint32_t* const* rows, const long* starts, const long* prefix, int S,
                      long n, uint64_t* ohi, uint64_t* olo, uint32_t* osplit, uint32_t* orow,
                      hipStream_t st) {
  if (n <= 0) return 0;
  if (S <= 0) return (int)hipErrorInvalidValue;
  const long grid = std::min<long>(ceil_div(n, 256), 256L * 256);
  hipLaunchKernelGGL(tera_collect_kernel, dim3((unsigned)grid), dim3(256), 0, st, his, los, rows,
                     starts, prefix, S, n, ohi, olo, osplit, orow);
  return (int)hipGetLastError();
}

// TeraSort map v3: (hi, lo, row) of n records in partition order and the
// partition boundaries offsets[0..nparts] (int64, device).  ws: device scratch
// of hbmr_tera_partition_workspace_bytes(n, nparts) bytes.
constexpr long kPartGridMax = 256L * 64;

inline size_t part_count_w_lds(int nsplit) {
  return (size_t)nsplit * 8 + (size_t)(nsplit + 1) * 4 + (size_t)nsplit * 2 + 16;
}

long hbmr_tera_partition_workspace_bytes(long n, int nparts) {
  return n * 8 * 2 + n * 2 + 2L * (nparts + 1) * 4 + 64 + kPartGridMax * 16;
}

// kst (nullable, device uint64[2] the caller zeroes): [0] |= every key's
// high-word bytes, [1] += sum(hi + lo) over the split (its key checksum)
int hbmr_tera_partition(const void* records, long n, int stride, const uint64_t* shi,
                        const uint64_t* slo, int nsplit, uint64_t* ohi, uint64_t* olo,
                        uint32_t* orow, long* offsets, unsigned long long* kmm, void* ws,
                        long ws_bytes, hipStream_t st) {
  const int nparts = nsplit + 1;
  if (nsplit < 0 || nsplit > kMaxSplitters) return (int)hipErrorInvalidValue;
  if (n < 0 || n >= (1L << 32)) return (int)hipErrorInvalidValue;
  if (ws_bytes < hbmr_tera_partition_workspace_bytes(n, nparts)) return (int)hipErrorInvalidValue;
  uint8_t* p = reinterpret_cast<uint8_t*>(ws);
  uint64_t* hi = reinterpret_cast<uint64_t*>(p);
  uint64_t* lo = hi + n;
  uint16_t* pid = reinterpret_cast<uint16_t*>(lo + n);
  unsigned int* counts = reinterpret_cast<unsigned int*>(
      (reinterpret_cast<uintptr_t>(pid + n) + 15) & ~uintptr_t(15));
  unsigned int* cursor = counts + (nparts + 1);
  unsigned long long* kparts = reinterpret_cast<unsigned long long*>(
      (reinterpret_cast<uintptr_t>(cursor + (nparts + 1)) + 15) & ~uintptr_t(15));
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(counts, 0, (size_t)(nparts + 1) * 4, st));
  // word loads of the key when the records allow them, else byte loads
  const bool words = stride % 4 == 0 && stride >= 12 &&
                     reinterpret_cast<uintptr_t>(records) % 4 == 0;
  if (n > 0) {
    const long grid = std::min<long>(ceil_div(n, 256), kPartGridMax);
    unsigned long long* kp = kmm != nullptr ? kparts : nullptr;
    if (words)
      hipLaunchKernelGGL(tera_part_count_w_kernel, dim3((unsigned)grid), dim3(256),
                         part_count_w_lds(nsplit), st,
                         reinterpret_cast<const uint32_t*>(records), n, stride / 4, shi, slo,
                         nsplit, hi, lo, pid, counts, kp);
    else
      hipLaunchKernelGGL(tera_part_count_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                         reinterpret_cast<const uint8_t*>(records), n, stride, shi, slo, nsplit,
                         hi, lo, pid, counts, kp);
    if (kmm != nullptr)
      hipLaunchKernelGGL(reduce_pairs_kernel, dim3(1), dim3(256), 0, st, kparts, grid, 1, kmm);
  }
  hipLaunchKernelGGL(tera_part_offsets_kernel, dim3(1), dim3(1024), 0, st, counts, nparts, cursor,
                     offsets);
  // (an LDS-staged scatter writing contiguous per-partition runs measured 2.4x
  // slower than this item-wise one: 19.1 vs 8.1 ms per 20 GB, twice the tiles'
  // scans, barriers and cursor atomics for writes that were already
  // ~85-record runs per partition and tile)
  if (n > 0)
    hipLaunchKernelGGL(tera_part_scatter_kernel, dim3((unsigned)ceil_div(n, kSortTile)),
                       dim3(kSortThreads), 0, st, hi, lo, pid, n, nparts, cursor, ohi, olo, orow);
  return (int)hipGetLastError();
}

int hbmr_tera_tie_fix(const uint64_t* hi, uint64_t* lo, uint32_t* perm, long n,
                      unsigned int* flag, hipStream_t st) {
  if (n <= 1) return 0;
  hipLaunchKernelGGL(tera_tie_fix_kernel, dim3((unsigned)ceil_div(n - 1, 256)), dim3(256), 0, st,
                     hi, lo, perm, n, flag);
  return (int)hipGetLastError();
}

int hbmr_merge_path(const uint64_t* ahi, const uint64_t* alo, const uint32_t* av, long na,
                    const uint64_t* bhi, const uint64_t* blo, const uint32_t* bv, long nb,
                    uint64_t* ohi, uint64_t* olo, uint32_t* ov, hipStream_t st) {
  const long n = na + nb;
  if (n <= 0) return 0;
  if (na < 0 || nb < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_path_kernel, dim3((unsigned)ceil_div(ceil_div(n, kMergeItems), 256)),
                     dim3(256), 0, st, ahi, alo, av, na, bhi, blo, bv, nb, ohi, olo, ov);
  return (int)hipGetLastError();
}

// pack != 0: ohi = window << 32 | gid with the window of key_window(vlo, m,
// R, sh) (< 2^32 for the group's keys), ogid unused
int hbmr_tera_collect_gid(const uint64_t* const* his, const uint32_t* const* rows,
                          const long* starts, const long* prefix, int S, long n, int pack,
                          uint64_t vlo, unsigned int m, unsigned int R, int sh, uint64_t* ohi,
                          uint32_t* ogid, hipStream_t st) {
  if (n <= 0) return 0;
  if (S <= 0 || S > 256 || (!pack && ogid == nullptr) || R < 2 || R > 256 || m + R > 256 ||
      sh < 0 || sh > 63)
    return (int)hipErrorInvalidValue;
  const KeyWindow kw{vlo, m, R, sh};
  const long grid = std::min<long>(ceil_div(n, 256), 256L * 256);
  hipLaunchKernelGGL(tera_collect_gid_kernel, dim3((unsigned)grid), dim3(256), 0, st, his, rows,
                     starts, prefix, S, n, pack, kw, ohi, ogid);
  return (int)hipGetLastError();
}

// gid: the record ids (split << 24 | row), or nullptr and packed: sorted keys
// whose low 32 bits are the ids (hi may be packed itself: each record's id is
// read before its key is written over it, by the same lanes)
int hbmr_gather_records_gid(const void* const* bases, const uint32_t* gid, const uint64_t* packed,
                            long n, int record_bytes, void* dst, uint64_t* hi, uint64_t* lo,
                            uint32_t* win, hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 64 || (gid == nullptr) == (packed == nullptr))
    return (int)hipErrorInvalidValue;
  if ((hi == nullptr) != (lo == nullptr) || (hi != nullptr && record_bytes < 12))
    return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  constexpr int U = 4;
  if (words >= 3) {
    const int u = g_gather_unroll;
    const long rpb = (long)(HBMR_WAVE / ((words + 3) / 4)) * (256 / HBMR_WAVE);
    const long grid16 = std::min<long>(ceil_div(n, rpb * u), 1L << 18);
    auto k = u == 1 ? gather_records_gid16_kernel<1>
           : u == 4 ? gather_records_gid16_kernel<4>
           : u == 8 ? gather_records_gid16_kernel<8> : gather_records_gid16_kernel<2>;
    hipLaunchKernelGGL(k, dim3((unsigned)grid16), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t* const*>(bases), gid, packed, n, words,
                       reinterpret_cast<uint32_t*>(dst), reinterpret_cast<uint32_t*>(hi), lo,
                       packed != nullptr ? win : nullptr);
    return (int)hipGetLastError();
  }
  const long grid = std::min<long>(ceil_div(n, (256 / words) * U), 1L << 18);
  hipLaunchKernelGGL(gather_records_gid_kernel<U>, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t* const*>(bases), gid, packed, n, words,
                     reinterpret_cast<uint32_t*>(dst), reinterpret_cast<uint32_t*>(hi), lo,
                     nullptr);
  return (int)hipGetLastError();
}

// waves per onesweep scatter tile: 4 (4096 keys), 8 (default: 80M keys in
// 2.02 ms against 2.54 for 4 — longer digit runs per write, fewer look-backs)
// or 16 (1.98 ms, one workgroup per CU);
// returns the previous setting
int hbmr_radix_set_onesweep_waves(int w) {
  const int old = g_onesweep_waves;
  g_onesweep_waves = w == 4 || w == 16 ? w : 8;
  return old;
}

// records each lane group of the packed-id gather keeps in flight: 1, 2
// (default: 0.81 ms per 12.5M records against 0.91 for 4 and 1.39 for 8 —
// more random lines in flight per CU thrash it), 4 or 8; returns the previous
// setting
int hbmr_gather_set_unroll(int u) {
  const int old = g_gather_unroll;
  g_gather_unroll = u == 1 || u == 4 || u == 8 ? u : 2;
  return old;
}

long hbmr_tera_tie_fix_scratch_bytes(long cap, int record_bytes) {
  return 16 + cap * (4 + 8 + 8 + (long)record_bytes);
}

// scratch: hbmr_tera_tie_fix_scratch_bytes(cap, record_bytes) for at most cap
// moved records (more are flagged)
// runs: equal key_window(vlo, m, R, sh) of hi (m = 0, R = 256, vlo = 0: hi >> sh),
// read from win (the gather's copy of each record's window) when given
int hbmr_tera_tie_fix_records(uint64_t* hi, uint64_t* lo, void* rec, long n, int record_bytes,
                              uint64_t vlo, unsigned int m, unsigned int R, int sh,
                              const uint32_t* win, unsigned int* flag, void* scratch, long cap,
                              hipStream_t st) {
  if (n <= 1) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 64 || sh < 0 || sh > 63 || cap < 1 ||
      n >= (1L << 32) || R < 2 || R > 256 || m + R > 256)
    return (int)hipErrorInvalidValue;
  const KeyWindow kw{vlo, m, R, sh};
  char* sc = reinterpret_cast<char*>(scratch);
  unsigned int* cnt = reinterpret_cast<unsigned int*>(sc);
  uint64_t* shi = reinterpret_cast<uint64_t*>(sc + 16);
  uint64_t* slo = shi + cap;
  uint32_t* sdst = reinterpret_cast<uint32_t*>(slo + cap);
  uint32_t* srec = sdst + cap;
  const int words = record_bytes / 4;
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(cnt, 0, 4, st));
  hipLaunchKernelGGL(tera_tie_rank_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, hi,
                     lo, reinterpret_cast<const uint32_t*>(rec), n, words, kw, win, cap, cnt, sdst,
                     shi, slo, srec, flag);
  const long grid = std::min<long>(ceil_div(cap, 256), 4096);
  hipLaunchKernelGGL(tera_tie_move_kernel, dim3((unsigned)grid), dim3(256), 0, st, hi, lo,
                     reinterpret_cast<uint32_t*>(rec), words, cap, cnt, sdst, shi, slo, srec);
  return (int)hipGetLastError();
}

int hbmr_gather_records_multi(const void* const* bases, const uint32_t* split, const uint32_t* row,
                              const uint32_t* perm, long n, int record_bytes, void* dst,
                              hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 256) return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  constexpr int U = 4;
  const long grid = std::min<long>(ceil_div(n, (256 / words) * U), 1L << 18);
  hipLaunchKernelGGL(gather_records_multi_v3_kernel<U>, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t* const*>(bases), split, row, perm, n, words,
                     reinterpret_cast<uint32_t*>(dst));
  return (int)hipGetLastError();
}

}  // extern "C"
