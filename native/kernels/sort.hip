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

// (1) digit histogram per tile, digit-major: hist[d * ntiles + tile]
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const uint64_t* __restrict__ keys,
                                                                  long n, int shift, long ntiles,
                                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t s[kSortWaves][kRadix];  // per-wave bins: 4x less same-address contention
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kSortWaves * kRadix; i += kSortThreads) (&s[0][0])[i] = 0u;
  __syncthreads();
  const long base = (long)blockIdx.x * kSortTile;
#pragma unroll 4
  for (int i = 0; i < kSortItems; ++i) {
    const long e = base + (long)i * kSortThreads + threadIdx.x;
    if (e < n) atomicAdd(&s[w][digit_of(keys[e], shift)], 1u);
  }
  __syncthreads();
  const int d = threadIdx.x;
  hist[(long)d * ntiles + blockIdx.x] = s[0][d] + s[1][d] + s[2][d] + s[3][d];
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

// (3) stable scatter of one tile
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint64_t* __restrict__ kout,
    uint32_t* __restrict__ vout, long n, int shift, long ntiles, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ totals) {
  __shared__ uint64_t s_k[kSortTile];
  __shared__ uint32_t s_v[kSortTile];
  __shared__ uint32_t s_wc[kSortWaves][kRadix];
  __shared__ uint32_t s_run[kRadix];
  __shared__ uint32_t s_toff[kRadix];
  __shared__ uint32_t s_gbase[kRadix];
  __shared__ uint32_t s_w[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const long tile = blockIdx.x;
  const long base = tile * kSortTile;
  const int tile_n = (int)min((long)kSortTile, n - base);

  // global start of digit t for this tile, and the tile's own digit offsets
  const uint32_t hd = hist[(long)t * ntiles + tile];
  const uint32_t cnt = (tile + 1 < ntiles ? hist[(long)t * ntiles + tile + 1] : totals[t]) - hd;
  const uint32_t gb = block_excl_scan256(totals[t], s_w);
  s_gbase[t] = gb + hd;
  const uint32_t toff = block_excl_scan256(cnt, s_w);
  s_toff[t] = toff;
  s_run[t] = 0u;
#pragma unroll
  for (int i = 0; i < kSortWaves; ++i) s_wc[i][t] = 0u;

  uint64_t k[kSortItems];
  uint32_t v[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const long e = base + (long)i * kSortThreads + t;
    if (e < n) {
      k[i] = kin[e];
      v[i] = vin ? vin[e] : (uint32_t)e;
    }
  }
  __syncthreads();
  const uint64_t lt = __lanemask_lt();
#pragma unroll 1
  for (int i = 0; i < kSortItems; ++i) {
    const bool valid = i * kSortThreads + t < tile_n;
    const uint32_t d = valid ? digit_of(k[i], shift) : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t pre = __popcll(m & lt);
    if (valid && pre == 0) s_wc[w][d] = __popcll(m);
    __syncthreads();
    if (valid) {
      uint32_t off = s_run[d] + pre;
      for (int ww = 0; ww < w; ++ww) off += s_wc[ww][d];
      const uint32_t local = s_toff[d] + off;
      s_k[local] = k[i];
      s_v[local] = v[i];
    }
    __syncthreads();
    {
      uint32_t sum = 0;
#pragma unroll
      for (int ww = 0; ww < kSortWaves; ++ww) {
        sum += s_wc[ww][t];
        s_wc[ww][t] = 0u;
      }
      s_run[t] += sum;
    }
    __syncthreads();
  }
  // the tile is grouped by digit in LDS: write each digit run to its place
  for (int j = t; j < tile_n; j += kSortThreads) {
    const uint64_t key = s_k[j];
    const uint32_t d = digit_of(key, shift);
    const long dst = (long)s_gbase[d] + (j - (long)s_toff[d]);
    kout[dst] = key;
    vout[dst] = s_v[j];
  }
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

// Key words + range partition of each record: pid = number of splitters <= key
// (partition p holds keys in [split[p-1], split[p]), as split_offsets cuts a
// sorted run).  Splitters are staged in LDS once per workgroup; each workgroup
// then walks a grid-stride slice of the records.
constexpr int kMaxSplitters = 4096;

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

// dst record i = record row[k] of split split[k], k = perm ? perm[i] : i
// (split kNoSplit: record i is left unwritten); records
// of `words` 4-byte words, one word per lane (25 lanes cover a 100-byte record)
// A workgroup copies 256 / words whole records per step: lane t moves word
// t % words of record t / words (one 32-bit division per thread, not one
// 64-bit division per word), so each record's index loads are shared by its
// lanes and its words are read and written as one contiguous run.
__global__ __launch_bounds__(256) void gather_records_multi_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ split,
    const uint32_t* __restrict__ row, const uint32_t* __restrict__ perm, long n, int words,
    uint32_t* __restrict__ dst) {
  const int rpb = 256 / words;
  const int t = threadIdx.x;
  if (t >= rpb * words) return;
  const int lr = t / words;
  const int w = t - lr * words;
  for (long r = (long)blockIdx.x * rpb + lr; r < n; r += (long)gridDim.x * rpb) {
    const long k = perm ? (long)perm[r] : r;
    const uint32_t sp = split[k];
    if (sp != kNoSplit) dst[r * words + w] = bases[sp][(long)row[k] * words + w];
  }
}

// ---- TeraSort map v3: partition without a sort ------------------------------
// (A) key words + partition id of every record, and the partition sizes: a
// per-workgroup LDS histogram flushed with one global add per touched bin.
__global__ __launch_bounds__(256) void tera_part_count_kernel(
    const uint8_t* __restrict__ rec, long n, int stride, const uint64_t* __restrict__ shi,
    const uint64_t* __restrict__ slo, int nsplit, uint64_t* __restrict__ hi,
    uint64_t* __restrict__ lo, uint16_t* __restrict__ pid, unsigned int* __restrict__ counts) {
  __shared__ uint64_t s_hi[kMaxSplitters];
  __shared__ uint16_t s_lo[kMaxSplitters];
  __shared__ unsigned int s_cnt[kMaxSplitters + 1];
  const int nparts = nsplit + 1;
  for (int j = threadIdx.x; j < nsplit; j += 256) {
    s_hi[j] = shi[j];
    s_lo[j] = (uint16_t)slo[j];
  }
  for (int j = threadIdx.x; j < nparts; j += 256) s_cnt[j] = 0u;
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
  }
  __syncthreads();
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
    uint64_t* __restrict__ lo, uint16_t* __restrict__ pid, unsigned int* __restrict__ counts) {
  __shared__ uint64_t s_hi[kMaxSplitters];
  __shared__ uint16_t s_lo[kMaxSplitters];
  __shared__ unsigned int s_cnt[kMaxSplitters + 1];
  const int nparts = nsplit + 1;
  for (int j = threadIdx.x; j < nsplit; j += 256) {
    s_hi[j] = shi[j];
    s_lo[j] = (uint16_t)slo[j];
  }
  for (int j = threadIdx.x; j < nparts; j += 256) s_cnt[j] = 0u;
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
  }
  __syncthreads();
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
    const long* __restrict__ starts, const long* __restrict__ prefix, int S, long n,
    uint64_t* __restrict__ ohi, uint32_t* __restrict__ ogid) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    int a = 0, b = S;          // largest s with prefix[s] <= i
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (prefix[m] <= i) a = m; else b = m;
    }
    const long j = starts[a] + (i - prefix[a]);
    ohi[i] = his[a][j];
    ogid[i] = ((uint32_t)a << 24) | rows[a][j];
  }
}

// (with key outputs: the lanes holding words 0-2 of a record also store its
// key — hi as two byte-swapped halves, lo from word 2 — so the sorted keys
// need no second pass over the gathered records)
template <int U, bool NT = false>
__global__ __launch_bounds__(256) void gather_records_gid_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ gid, long n,
    int words, uint32_t* __restrict__ dst, uint32_t* __restrict__ khi,
    uint64_t* __restrict__ klo) {
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
        const uint32_t g = gid[r];
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
        if constexpr (NT)
          __builtin_nontemporal_store(v[j], dst + r * words + w);  // streamed: no L2 reuse
        else
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

template <int U, bool NT>
__global__ __launch_bounds__(256) void gather_records_gid16_kernel(
    const uint32_t* const* __restrict__ bases, const uint32_t* __restrict__ gid, long n,
    int words, uint32_t* __restrict__ dst, uint32_t* __restrict__ khi,
    uint64_t* __restrict__ klo) {
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
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long r = r0 + j * stride;
      src[j] = nullptr;
      if (r < n) {
        const uint32_t g = gid[r];
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
        if constexpr (NT)
          __builtin_nontemporal_store(v[j], reinterpret_cast<u32x4_a4*>(d));
        else
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
      }
    }
  }
}

// After the sort on the high key word's top 64 - shift bits and the record
// gather: order each run of an equal sorted prefix (hi >> shift) by the full
// key (hi, lo), moving hi, lo and the (already gathered) records themselves;
// runs longer than kTieRun are flagged for the full-key path.  shift = 16
// saves two of eight radix passes: among the ~10^8 keys of a group, equal
// 48-bit prefixes come in a few dozen pairs.
__global__ __launch_bounds__(256) void tera_tie_fix_records_kernel(
    uint64_t* __restrict__ hi, uint64_t* __restrict__ lo, uint32_t* __restrict__ rec,
    long n, int words, int shift, unsigned int* __restrict__ flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n - 1) return;
  const uint64_t h = hi[i] >> shift;
  if ((hi[i + 1] >> shift) != h || (i > 0 && (hi[i - 1] >> shift) == h)) return;
  long e = i + 1;
  while (e < n && (hi[e] >> shift) == h && e - i < kTieRun) ++e;
  if (e < n && (hi[e] >> shift) == h) {
    atomicOr(flag, 1u);
    return;
  }
  // insertion sort by adjacent swaps (no per-lane record buffer)
  for (long a = i + 1; a < e; ++a) {
    for (long b = a - 1;
         b >= i && (hi[b] > hi[b + 1] || (hi[b] == hi[b + 1] && lo[b] > lo[b + 1])); --b) {
      const uint64_t th = hi[b];
      hi[b] = hi[b + 1];
      hi[b + 1] = th;
      const uint64_t t = lo[b];
      lo[b] = lo[b + 1];
      lo[b + 1] = t;
      for (int w = 0; w < words; ++w) {
        const uint32_t x = rec[b * words + w];
        rec[b * words + w] = rec[(b + 1) * words + w];
        rec[(b + 1) * words + w] = x;
      }
    }
  }
}

inline long ceil_div(long a, long b) { return (a + b - 1) / b; }

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
  // HBMR_RADIX_V1=1: the round-1 kernels (per-key atomics, 3 barriers per key), for A/B
  static const bool v1 = [] {
    const char* e = getenv("HBMR_RADIX_V1");
    return e && *e == '1';
  }();
  int passes = 0;
  for (int shift = begin_bit; shift < end_bit; shift += 8, ++passes) {
    if (v1)
      hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st, ka,
                         n, shift, ntiles, hist);
    else
      hipLaunchKernelGGL(radix_hist_v2_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st,
                         ka, n, shift, ntiles, hist);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(kRadix), dim3(1024), 0, st, hist, ntiles, totals);
    if (v1)
      hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st,
                         ka, va, kb, vb, n, shift, ntiles, hist, totals);
    else
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
long hbmr_tera_partition_workspace_bytes(long n, int nparts) {
  return n * 8 * 2 + n * 2 + 2L * (nparts + 1) * 4 + 64;
}

int hbmr_tera_partition(const void* records, long n, int stride, const uint64_t* shi,
                        const uint64_t* slo, int nsplit, uint64_t* ohi, uint64_t* olo,
                        uint32_t* orow, long* offsets, void* ws, long ws_bytes, hipStream_t st) {
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
  HBMR_RETURN_IF_ERROR(hipMemsetAsync(counts, 0, (size_t)(nparts + 1) * 4, st));
  // HBMR_TERA_PART=v1: the byte-load count (rounds 3-4)
  static const bool v1 = [] {
    const char* e = getenv("HBMR_TERA_PART");
    return e && std::string(e) == "v1";
  }();
  const bool words = !v1 && stride % 4 == 0 && stride >= 12 &&
                     reinterpret_cast<uintptr_t>(records) % 4 == 0;
  if (n > 0) {
    const long grid = std::min<long>(ceil_div(n, 256), 256L * 64);
    if (words)
      hipLaunchKernelGGL(tera_part_count_w_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                         reinterpret_cast<const uint32_t*>(records), n, stride / 4, shi, slo,
                         nsplit, hi, lo, pid, counts);
    else
      hipLaunchKernelGGL(tera_part_count_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                         reinterpret_cast<const uint8_t*>(records), n, stride, shi, slo, nsplit,
                         hi, lo, pid, counts);
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

int hbmr_tera_collect_gid(const uint64_t* const* his, const uint32_t* const* rows,
                          const long* starts, const long* prefix, int S, long n, uint64_t* ohi,
                          uint32_t* ogid, hipStream_t st) {
  if (n <= 0) return 0;
  if (S <= 0 || S > 256) return (int)hipErrorInvalidValue;
  const long grid = std::min<long>(ceil_div(n, 256), 256L * 256);
  hipLaunchKernelGGL(tera_collect_gid_kernel, dim3((unsigned)grid), dim3(256), 0, st, his, rows,
                     starts, prefix, S, n, ohi, ogid);
  return (int)hipGetLastError();
}

int hbmr_gather_records_gid(const void* const* bases, const uint32_t* gid, long n,
                            int record_bytes, void* dst, uint64_t* hi, uint64_t* lo,
                            hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 64) return (int)hipErrorInvalidValue;
  if ((hi == nullptr) != (lo == nullptr) || (hi != nullptr && record_bytes < 12))
    return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  // HBMR_GATHER=u8 / nt / u8nt: 8 records in flight per lane and/or streamed
  // (non-temporal) stores of the gathered records, for A/B
  static const int mode = [] {
    const char* e = getenv("HBMR_GATHER");
    if (!e) return 0;
    const std::string m(e);
    return (m.find("u8") != std::string::npos ? 1 : 0) | (m.find("nt") != std::string::npos ? 2 : 0);
  }();
  const int U = (mode & 1) ? 8 : 4;
  // HBMR_GATHER=w1...: the word-per-lane kernel (round 3-4) for A/B
  static const bool word_lanes = [] {
    const char* e = getenv("HBMR_GATHER");
    return e && std::string(e).find("w1") != std::string::npos;
  }();
  if (!word_lanes && words >= 3) {
    auto k16 = mode == 0 ? gather_records_gid16_kernel<4, false>
             : mode == 1 ? gather_records_gid16_kernel<8, false>
             : mode == 2 ? gather_records_gid16_kernel<4, true>
                         : gather_records_gid16_kernel<8, true>;
    const long rpb = (long)(HBMR_WAVE / ((words + 3) / 4)) * (256 / HBMR_WAVE);
    const long grid16 = std::min<long>(ceil_div(n, rpb * U), 1L << 18);
    hipLaunchKernelGGL(k16, dim3((unsigned)grid16), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t* const*>(bases), gid, n, words,
                       reinterpret_cast<uint32_t*>(dst), reinterpret_cast<uint32_t*>(hi), lo);
    return (int)hipGetLastError();
  }
  auto kern = mode == 0 ? gather_records_gid_kernel<4, false>
            : mode == 1 ? gather_records_gid_kernel<8, false>
            : mode == 2 ? gather_records_gid_kernel<4, true>
                        : gather_records_gid_kernel<8, true>;
  const long grid = std::min<long>(ceil_div(n, (256 / words) * U), 1L << 18);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t* const*>(bases), gid, n, words,
                     reinterpret_cast<uint32_t*>(dst), reinterpret_cast<uint32_t*>(hi), lo);
  return (int)hipGetLastError();
}

int hbmr_tera_tie_fix_records(uint64_t* hi, uint64_t* lo, void* rec, long n,
                              int record_bytes, int shift, unsigned int* flag, hipStream_t st) {
  if (n <= 1) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 64 || shift < 0 || shift > 63)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tera_tie_fix_records_kernel, dim3((unsigned)ceil_div(n - 1, 256)), dim3(256),
                     0, st, hi, lo, reinterpret_cast<uint32_t*>(rec), n, record_bytes / 4, shift,
                     flag);
  return (int)hipGetLastError();
}

int hbmr_gather_records_multi(const void* const* bases, const uint32_t* split, const uint32_t* row,
                              const uint32_t* perm, long n, int record_bytes, void* dst,
                              hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 256) return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  static const bool v1 = [] {
    const char* e = getenv("HBMR_GATHER_V1");
    return e && *e == '1';
  }();
  if (v1) {
    const long grid = std::min<long>(ceil_div(n, 256 / words), 1L << 20);
    hipLaunchKernelGGL(gather_records_multi_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t* const*>(bases), split, row, perm, n, words,
                       reinterpret_cast<uint32_t*>(dst));
  } else {
    constexpr int U = 4;
    const long grid = std::min<long>(ceil_div(n, (256 / words) * U), 1L << 18);
    hipLaunchKernelGGL(gather_records_multi_v3_kernel<U>, dim3((unsigned)grid), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t* const*>(bases), split, row, perm, n, words,
                       reinterpret_cast<uint32_t*>(dst));
  }
  return (int)hipGetLastError();
}

}  // extern "C"
