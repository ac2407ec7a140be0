// Text map kernels: tokenize → exact hash-aggregate
// (the fused combiner) → Java-hash partition → pack, for GPU WordCount.
//
// The reference's WordCount map (src/examples/.../WordCount.java and the Pipes
// wordcount-simple.cc:34-41) emits (word, 1) per token, and the combiner /
// reducer sums per word after a sort by key.  On the GPU a split is one byte
// buffer in HBM:
//
//  1. wc_tokenize_count / wc_tokenize_write: word starts (a non-space byte
//     whose predecessor is a space or the buffer start; spaces are the ASCII
//     whitespace set of the CPU mapper) compacted in order by a per-tile count,
//     a scan of tile counts and a per-tile rewrite.  Each lane owns 16
//     consecutive bytes read as one 16-byte vector load.
//  2. wc_insert: open-addressing tables of 64-bit keys (32-bit hash tag |
//     representative start + 1) claimed by 64-bit CAS; a tag match is
//     confirmed by comparing the bytes of the representative occurrence, so
//     the aggregation is exact (no hash-only merging).  Each workgroup folds
//     its words into an LDS table first and inserts every distinct word once
//     into the global (HBM) table.  Counts are 64-bit atomics; an optional
//     weight per word makes the same kernel merge partial (word, count) tables.
//  3. wc_compact: occupied slots → (start, len, count, partition), partition =
//     (Text.hashCode() & INT_MAX) % R with hashCode = WritableComparator.
//     hashBytes (31·h + signed byte, h0 = 1), i.e. Hadoop's HashPartitioner.
//  4. wc_pack: words (in a given order) → "word\n" blob for the shuffle.
#include "common.h"
#include "../include/hbmr/hbmr.h"

namespace {

constexpr int kTokThreads = 256;
constexpr int kTokBytes = 16;                    // per lane
constexpr int kTokTile = kTokThreads * kTokBytes;  // 4096 bytes per workgroup

__device__ __forceinline__ bool is_space(uint8_t c) {
  // bytes.split(): space, \t, \n, \v, \f, \r
  return c == ' ' || (c >= 9 && c <= 13);
}

__device__ __forceinline__ void load16(const uint8_t* __restrict__ buf, long n, long i0,
                                       uint8_t b[kTokBytes]) {
  if (i0 + kTokBytes <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(buf + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < kTokBytes; ++j) b[j] = (uint8_t)(w[j >> 2] >> ((j & 3) * 8));
  } else {
#pragma unroll
    for (int j = 0; j < kTokBytes; ++j) b[j] = (i0 + j < n) ? buf[i0 + j] : (uint8_t)' ';
  }
}

// start-of-word bit mask of this lane's 16 bytes
__device__ __forceinline__ uint32_t start_mask(const uint8_t* __restrict__ buf, long n, long i0) {
  uint8_t b[kTokBytes];
  load16(buf, n, i0, b);
  bool prev_space = (i0 == 0) ? true : (i0 - 1 < n ? is_space(buf[i0 - 1]) : true);
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < kTokBytes; ++j) {
    const bool sp = is_space(b[j]);
    if (!sp && prev_space && i0 + j < n) m |= 1u << j;
    prev_space = sp;
  }
  return m;
}

__device__ __forceinline__ uint32_t block_reduce_add(uint32_t v, uint32_t* s_w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int i = 0; i < kTokThreads / HBMR_WAVE; ++i) t += s_w[i];
  return t;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w) {
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
  return base + v - x;
}

__global__ __launch_bounds__(kTokThreads) void wc_tokenize_count_kernel(
    const uint8_t* __restrict__ buf, long n, uint32_t* __restrict__ tile_counts) {
  __shared__ uint32_t s_w[kTokThreads / HBMR_WAVE];
  const long i0 = (long)blockIdx.x * kTokTile + (long)threadIdx.x * kTokBytes;
  const uint32_t c = i0 < n ? (uint32_t)__popc(start_mask(buf, n, i0)) : 0u;
  const uint32_t t = block_reduce_add(c, s_w);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = t;
}

__global__ __launch_bounds__(kTokThreads) void wc_tokenize_write_kernel(
    const uint8_t* __restrict__ buf, long n, const long* __restrict__ tile_base,
    uint32_t* __restrict__ starts, uint32_t* __restrict__ lens) {
  __shared__ uint32_t s_w[kTokThreads / HBMR_WAVE];
  const long i0 = (long)blockIdx.x * kTokTile + (long)threadIdx.x * kTokBytes;
  uint32_t m = i0 < n ? start_mask(buf, n, i0) : 0u;
  const uint32_t off = block_excl_scan((uint32_t)__popc(m), s_w);
  long o = tile_base[blockIdx.x] + off;
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    const long s = i0 + j;
    long e = s + 1;
    while (e < n && !is_space(buf[e])) ++e;
    starts[o] = (uint32_t)s;
    lens[o] = (uint32_t)(e - s);
    ++o;
  }
}

__device__ __forceinline__ uint64_t word_hash64(const uint8_t* p, uint32_t len) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (uint32_t i = 0; i < len; ++i) h = (h ^ p[i]) * 1099511628211ull;
  h ^= h >> 33;                          // murmur3 fmix64
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

// bytes of the word at p (len) equal the whitespace-delimited word at rs?
__device__ __forceinline__ bool same_word(const uint8_t* __restrict__ buf, long n, uint32_t rs,
                                          const uint8_t* p, uint32_t len) {
  for (uint32_t i = 0; i < len; ++i)
    if ((long)rs + i >= n || buf[rs + i] != p[i]) return false;
  return !((long)rs + len < n && !is_space(buf[rs + len]));
}

// insert (key = tag | start+1) with weight into the global table
__device__ __forceinline__ bool global_insert(const uint8_t* __restrict__ buf, long n,
                                              uint64_t h, unsigned long long key, uint32_t s,
                                              uint32_t len, unsigned long long wt,
                                              unsigned long long* __restrict__ tkeys,
                                              unsigned long long* __restrict__ tcounts,
                                              unsigned long long mask) {
  const uint8_t* p = buf + s;
  unsigned long long slot = h & mask;
  // a probe run this long means the table is too full: report overflow and let
  // the host retry with a larger table instead of crawling
  const unsigned long long max_probe = mask < 4096ull ? mask : 4096ull;
  for (unsigned long long probe = 0; probe <= max_probe; ++probe) {
    unsigned long long cur = tkeys[slot];
    if (cur == 0ull) {
      cur = atomicCAS(&tkeys[slot], 0ull, key);
      if (cur == 0ull) {
        atomicAdd(&tcounts[slot], wt);
        return true;
      }
    }
    if ((cur >> 32) == (key >> 32) &&
        same_word(buf, n, (uint32_t)(cur & 0xffffffffull) - 1u, p, len)) {
      atomicAdd(&tcounts[slot], wt);
      return true;
    }
    slot = (slot + 1) & mask;
  }
  return false;
}

constexpr int kInsThreads = 256;
constexpr int kInsWordsPerThread = 16;
constexpr int kInsWords = kInsThreads * kInsWordsPerThread;  // words per workgroup
constexpr int kLdsSlots = 2048;                              // 32 KiB of LDS
constexpr int kLdsProbes = 32;

// Two-level aggregation: a workgroup first folds its 4096 words into an LDS
// table (hot words — the Zipf head of natural text — collapse there instead
// of hammering one global counter), then inserts each distinct word once into
// the global table with its local count.  Words that find no LDS slot within
// kLdsProbes go straight to the global table.
__global__ __launch_bounds__(kInsThreads) void wc_insert_kernel(
    const uint8_t* __restrict__ buf, long n, const uint32_t* __restrict__ starts,
    const uint32_t* __restrict__ lens, const int64_t* __restrict__ weights, long nwords,
    unsigned long long* __restrict__ tkeys, unsigned long long* __restrict__ tcounts,
    unsigned long long mask, int* __restrict__ overflow) {
  __shared__ unsigned long long s_keys[kLdsSlots];
  __shared__ unsigned long long s_cnt[kLdsSlots];
  for (int i = threadIdx.x; i < kLdsSlots; i += kInsThreads) {
    s_keys[i] = 0ull;
    s_cnt[i] = 0ull;
  }
  __syncthreads();
  const long w0 = (long)blockIdx.x * kInsWords;
  bool ovf = false;
#pragma unroll 1
  for (int j = 0; j < kInsWordsPerThread; ++j) {
    const long w = w0 + (long)j * kInsThreads + threadIdx.x;
    if (w >= nwords) break;
    const uint32_t s = starts[w], len = lens[w];
    const uint8_t* p = buf + s;
    const uint64_t h = word_hash64(p, len);
    const unsigned long long key = ((h >> 32) << 32) | (unsigned long long)(s + 1u);
    const unsigned long long wt = weights ? (unsigned long long)weights[w] : 1ull;
    uint32_t slot = (uint32_t)(h >> 7) & (kLdsSlots - 1);
    bool done = false;
    for (int probe = 0; probe < kLdsProbes && !done; ++probe) {
      unsigned long long cur = s_keys[slot];
      if (cur == 0ull) {
        cur = atomicCAS(&s_keys[slot], 0ull, key);
        if (cur == 0ull) {
          atomicAdd(&s_cnt[slot], wt);
          done = true;
          break;
        }
      }
      if ((cur >> 32) == (key >> 32) &&
          same_word(buf, n, (uint32_t)(cur & 0xffffffffull) - 1u, p, len)) {
        atomicAdd(&s_cnt[slot], wt);
        done = true;
        break;
      }
      slot = (slot + 1) & (kLdsSlots - 1);
    }
    if (!done && !global_insert(buf, n, h, key, s, len, wt, tkeys, tcounts, mask)) ovf = true;
  }
  __syncthreads();
  // flush: each distinct word of this workgroup once into the global table
  for (int i = threadIdx.x; i < kLdsSlots; i += kInsThreads) {
    const unsigned long long key = s_keys[i];
    if (key == 0ull) continue;
    const uint32_t s = (uint32_t)(key & 0xffffffffull) - 1u;
    uint32_t len = 0;
    while ((long)s + len < n && !is_space(buf[s + len])) ++len;
    const uint64_t h = word_hash64(buf + s, len);
    if (!global_insert(buf, n, h, key, s, len, s_cnt[i], tkeys, tcounts, mask)) ovf = true;
  }
  if (ovf) atomicExch(overflow, 1);
}

__global__ __launch_bounds__(256) void wc_compact_kernel(
    const uint8_t* __restrict__ buf, long n, const unsigned long long* __restrict__ tkeys,
    const unsigned long long* __restrict__ tcounts, long cap, int R,
    uint32_t* __restrict__ ustart, uint32_t* __restrict__ ulen, int64_t* __restrict__ ucount,
    int32_t* __restrict__ upart, unsigned int* __restrict__ counter) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const unsigned long long k = tkeys[i];
  if (k == 0ull) return;
  const uint32_t s = (uint32_t)(k & 0xffffffffull) - 1u;
  long e = s;
  uint32_t jh = 1u;
  while (e < n && !is_space(buf[e])) {
    jh = 31u * jh + (uint32_t)(int32_t)(int8_t)buf[e];
    ++e;
  }
  const unsigned int o = atomicAdd(counter, 1u);
  ustart[o] = s;
  ulen[o] = (uint32_t)(e - s);
  ucount[o] = (int64_t)tcounts[i];
  upart[o] = (int32_t)(((int32_t)jh & 0x7fffffff) % R);
}

__global__ __launch_bounds__(256) void wc_pack_kernel(
    const uint8_t* __restrict__ buf, const uint32_t* __restrict__ ustart,
    const uint32_t* __restrict__ ulen, const int64_t* __restrict__ order, long nu,
    const int64_t* __restrict__ out_off, uint8_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nu) return;
  const long u = order ? order[i] : i;
  const uint8_t* src = buf + ustart[u];
  const uint32_t len = ulen[u];
  uint8_t* dst = out + out_off[i];
  for (uint32_t j = 0; j < len; ++j) dst[j] = src[j];
  dst[len] = '\n';
}

inline int grid_for(long n, int per) { return (int)((n + per - 1) / per); }

}  // namespace

extern "C" {

long hbmr_wc_tiles(long n) { return (n + kTokTile - 1) / kTokTile; }

int hbmr_wc_tokenize_count(const uint8_t* buf, long n, uint32_t* tile_counts,
                           hipStream_t stream) {
  const long tiles = hbmr_wc_tiles(n);
  if (tiles == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(buf) & 15u) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wc_tokenize_count_kernel, dim3((unsigned)tiles), dim3(kTokThreads), 0,
                     stream, buf, n, tile_counts);
  return (int)hipGetLastError();
}

int hbmr_wc_tokenize_write(const uint8_t* buf, long n, const long* tile_base, uint32_t* starts,
                           uint32_t* lens, hipStream_t stream) {
  const long tiles = hbmr_wc_tiles(n);
  if (tiles == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(buf) & 15u) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wc_tokenize_write_kernel, dim3((unsigned)tiles), dim3(kTokThreads), 0,
                     stream, buf, n, tile_base, starts, lens);
  return (int)hipGetLastError();
}

// cap must be a power of two; tkeys/tcounts zeroed by the caller
int hbmr_wc_insert(const uint8_t* buf, long n, const uint32_t* starts, const uint32_t* lens,
                   const int64_t* weights, long nwords, uint64_t* tkeys, uint64_t* tcounts,
                   long cap, int* overflow, hipStream_t stream) {
  if (nwords == 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || n >= 0xffffffffl) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wc_insert_kernel, dim3(grid_for(nwords, kInsWords)), dim3(kInsThreads), 0,
                     stream, buf, n,
                     starts, lens, weights, nwords,
                     reinterpret_cast<unsigned long long*>(tkeys),
                     reinterpret_cast<unsigned long long*>(tcounts),
                     (unsigned long long)(cap - 1), overflow);
  return (int)hipGetLastError();
}

int hbmr_wc_compact(const uint8_t* buf, long n, const uint64_t* tkeys, const uint64_t* tcounts,
                    long cap, int R, uint32_t* ustart, uint32_t* ulen, int64_t* ucount,
                    int32_t* upart, unsigned int* counter, hipStream_t stream) {
  if (cap == 0) return 0;
  if (R <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wc_compact_kernel, dim3(grid_for(cap, 256)), dim3(256), 0, stream, buf, n,
                     reinterpret_cast<const unsigned long long*>(tkeys),
                     reinterpret_cast<const unsigned long long*>(tcounts), cap, R, ustart, ulen,
                     ucount, upart, counter);
  return (int)hipGetLastError();
}

int hbmr_wc_pack(const uint8_t* buf, const uint32_t* ustart, const uint32_t* ulen,
                 const int64_t* order, long nu, const int64_t* out_off, uint8_t* out,
                 hipStream_t stream) {
  if (nu == 0) return 0;
  hipLaunchKernelGGL(wc_pack_kernel, dim3(grid_for(nu, 256)), dim3(256), 0, stream, buf, ustart,
                     ulen, order, nu, out_off, out);
  return (int)hipGetLastError();
}

}  // extern "C"
