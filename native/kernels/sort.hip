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

// dst record i = record row[k] of split split[k], k = perm ? perm[i] : i; records
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
    dst[r * words + w] = bases[split[k]][(long)row[k] * words + w];
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

int hbmr_gather_records_multi(const void* const* bases, const uint32_t* split, const uint32_t* row,
                              const uint32_t* perm, long n, int record_bytes, void* dst,
                              hipStream_t st) {
  if (n <= 0) return 0;
  if (record_bytes % 4 || record_bytes > 4 * 256) return (int)hipErrorInvalidValue;
  const int words = record_bytes / 4;
  const long grid = std::min<long>(ceil_div(n, 256 / words), 1L << 20);
  hipLaunchKernelGGL(gather_records_multi_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t* const*>(bases), split, row, perm, n, words,
                     reinterpret_cast<uint32_t*>(dst));
  return (int)hipGetLastError();
}

}  // extern "C"
