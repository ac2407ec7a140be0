// CPU WordCount map kernel (BASELINE config 1): whitespace tokenisation and
// per-split word counting for hbmr.models.wordcount's native map runner.
//
// The reference's WordCount mapper (examples/WordCount.java) emits (word, 1)
// per StringTokenizer token and relies on the combiner; here a split's text
// is counted in one open-addressing table (word bytes in an arena, 64-bit
// hash, linear probing) and each distinct word is emitted once with its count
// — the in-mapper combining of hbmr.wordcount.inmapper.combine, without a
// Python object per token.  Tokens are maximal runs of bytes other than
// ASCII whitespace (space, \t, \n, \v, \f, \r), as Python's bytes.split().
#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <algorithm>
#include <vector>

namespace {

struct Entry {
  uint64_t hash;   // 0 = empty slot
  uint64_t w0, w1; // the word's first 16 bytes, zero-padded (compare without the arena)
  int64_t off;     // word bytes in the arena
  int32_t len;
  int64_t count;
};

// ASCII whitespace as a table (one load per byte instead of a compare chain)
struct SpaceTable {
  bool t[256];
  SpaceTable() {
    for (int c = 0; c < 256; ++c) t[c] = c == ' ' || (c >= '\t' && c <= '\r');
  }
};
const SpaceTable kSpace;

inline bool is_space(unsigned char c) { return kSpace.t[c]; }

// whitespace bits of 64 bytes (AVX2): ' ' or 9..13
__attribute__((target("avx2"))) inline uint64_t space_mask64(const unsigned char* p) {
  const __m256i sp = _mm256_set1_epi8(' '), nine = _mm256_set1_epi8(9),
                four = _mm256_set1_epi8(4);
  const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
  const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 32));
  const __m256i ta = _mm256_sub_epi8(a, nine), tb = _mm256_sub_epi8(b, nine);
  const __m256i wa = _mm256_or_si256(_mm256_cmpeq_epi8(a, sp),
                                     _mm256_cmpeq_epi8(_mm256_min_epu8(ta, four), ta));
  const __m256i wb = _mm256_or_si256(_mm256_cmpeq_epi8(b, sp),
                                     _mm256_cmpeq_epi8(_mm256_min_epu8(tb, four), tb));
  return (uint64_t)(uint32_t)_mm256_movemask_epi8(wa) |
         (uint64_t)(uint32_t)_mm256_movemask_epi8(wb) << 32;
}

inline uint64_t mix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h | 1;   // never 0 (the empty marker)
}

inline uint64_t load64(const unsigned char* p) {
  uint64_t w;
  std::memcpy(&w, p, 8);    // constant size: one unaligned load
  return w;
}

inline uint64_t low_bytes(uint64_t w, int64_t n) {   // the first n < 8 bytes of w
  return w & ((1ULL << (8 * n)) - 1);
}

// the first 16 bytes of a word, zero-padded (n bytes readable at p; `end` is
// the buffer's end: with 16 bytes to spare the bytes come from two masked
// loads, not a variable-length memcpy call per token)
inline void prefix16(const unsigned char* p, int64_t n, const unsigned char* end, uint64_t& w0,
                     uint64_t& w1) {
  if (p + 16 <= end) {
    const uint64_t a = load64(p), b = load64(p + 8);
    if (n < 8) {
      w0 = low_bytes(a, n);
      w1 = 0;
    } else if (n < 16) {
      w0 = a;
      w1 = n == 8 ? 0 : low_bytes(b, n - 8);
    } else {
      w0 = a;
      w1 = b;
    }
    return;
  }
  w0 = w1 = 0;
  if (n >= 16) {
    std::memcpy(&w0, p, 8);
    std::memcpy(&w1, p + 8, 8);
  } else if (n > 8) {
    std::memcpy(&w0, p, 8);
    std::memcpy(&w1, p + 8, (size_t)(n - 8));
  } else {
    std::memcpy(&w0, p, (size_t)n);
  }
}

inline uint64_t hash_word(const unsigned char* p, int64_t n, uint64_t w0, uint64_t w1) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)n;
  h = (h ^ w0) * 0x100000001B3ULL;
  h ^= h >> 29;
  h = (h ^ w1) * 0x100000001B3ULL;
  for (int64_t i = 16; i < n; i += 8) {     // long words: the rest in 8-byte steps
    uint64_t w = 0;
    std::memcpy(&w, p + i, (size_t)std::min<int64_t>(8, n - i));
    h = (h ^ w) * 0x100000001B3ULL;
    h ^= h >> 29;
  }
  return mix(h);
}

struct Table {
  std::vector<Entry> slots;
  std::vector<unsigned char> arena;
  int64_t used = 0;
  int64_t tokens = 0;
  int64_t newlines = 0;

  Table() : slots(1 << 12) {}   // grows at 3/4 load; small stays cache-resident

  void grow() {
    std::vector<Entry> old;
    old.swap(slots);
    slots.assign(old.size() * 2, Entry{0, 0, 0, 0, 0, 0});
    const uint64_t mask = slots.size() - 1;
    for (const Entry& e : old) {
      if (!e.hash) continue;
      uint64_t i = e.hash & mask;
      while (slots[i].hash) i = (i + 1) & mask;
      slots[i] = e;
    }
  }

  void add(const unsigned char* w, int64_t n, const unsigned char* end) {
    ++tokens;
    uint64_t w0, w1;
    prefix16(w, n, end, w0, w1);
    const uint64_t h = hash_word(w, n, w0, w1);
    uint64_t mask = slots.size() - 1;
    uint64_t i = h & mask;
    for (;;) {
      Entry& e = slots[i];
      if (!e.hash) break;
      if (e.hash == h && e.len == n && e.w0 == w0 && e.w1 == w1 &&
          (n <= 16 || std::memcmp(arena.data() + e.off + 16, w + 16, (size_t)(n - 16)) == 0)) {
        ++e.count;
        return;
      }
      i = (i + 1) & mask;
    }
    if ((used + 1) * 4 > (int64_t)slots.size() * 3) {   // load factor 0.75
      grow();
      mask = slots.size() - 1;
      i = h & mask;
      while (slots[i].hash) i = (i + 1) & mask;
    }
    Entry& e = slots[i];
    e.hash = h;
    e.w0 = w0;
    e.w1 = w1;
    e.off = (int64_t)arena.size();
    e.len = (int32_t)n;
    e.count = 1;
    arena.insert(arena.end(), w, w + n);
    ++used;
  }
};

// 64 bytes at a time: token starts / ends from the whitespace bitmask (a
// token open across chunks carries over in `open`); returns the first byte
// not scanned (the tail goes byte by byte)
__attribute__((target("avx2"))) int64_t scan_avx2(Table* t, const unsigned char* p, int64_t n,
                                                  const unsigned char* end, int64_t& open) {
  int64_t i = 0;
  uint64_t prev = 0;                 // bit 63: byte i-1 was a token byte
  for (; i + 64 <= n; i += 64) {
    const uint64_t nonsp = ~space_mask64(p + i);
    const uint64_t shifted = (nonsp << 1) | (prev >> 63);
    uint64_t starts = nonsp & ~shifted;
    uint64_t ends = ~nonsp & shifted;
    for (;;) {
      if (open >= 0) {
        if (!ends) break;            // the token runs on into the next chunk
        const int e = __builtin_ctzll(ends);
        ends &= ends - 1;
        t->add(p + open, i + e - open, end);
        open = -1;
      }
      if (!starts) break;
      open = i + __builtin_ctzll(starts);
      starts &= starts - 1;
    }
    prev = nonsp;
  }
  return i;
}

const bool kAvx2 = __builtin_cpu_supports("avx2");

}  // namespace

extern "C" {

void* hbmr_wc_cpu_new() { return new Table(); }

void hbmr_wc_cpu_free(void* h) { delete static_cast<Table*>(h); }

// Count the tokens of buf[0, n); returns the number of distinct words so far.
int64_t hbmr_wc_cpu_add(void* h, const void* buf, int64_t n) {
  Table* t = static_cast<Table*>(h);
  const unsigned char* p = static_cast<const unsigned char*>(buf);
  const unsigned char* end = p + n;
  int64_t i = 0, nl = 0;
  int64_t open = -1;
  if (kAvx2) i = scan_avx2(t, p, n, end, open);
  for (; i < n; ++i) {               // the tail (or no AVX2), byte by byte
    if (is_space(p[i])) {
      if (open >= 0) t->add(p + open, i - open, end);
      open = -1;
    } else if (open < 0) {
      open = i;
    }
  }
  if (open >= 0) t->add(p + open, n - open, end);
  // newlines (the map's input records) by memchr, outside the token loop
  for (const void* q = p; (q = std::memchr(q, '\n', (size_t)(end - (const unsigned char*)q)));
       q = (const unsigned char*)q + 1)
    ++nl;
  t->newlines += nl;
  return t->used;
}

// newlines seen by hbmr_wc_cpu_add so far (the map's input records)
int64_t hbmr_wc_cpu_newlines(void* h) { return static_cast<Table*>(h)->newlines; }

int64_t hbmr_wc_cpu_words(void* h) { return static_cast<Table*>(h)->used; }

int64_t hbmr_wc_cpu_tokens(void* h) { return static_cast<Table*>(h)->tokens; }

int64_t hbmr_wc_cpu_bytes(void* h) { return (int64_t) static_cast<Table*>(h)->arena.size(); }

// Distinct words in first-seen order: their bytes concatenated into `words`
// (hbmr_wc_cpu_bytes of them), offsets[0..w] and counts[0..w-1]; then clears
// the table for the next batch.
void hbmr_wc_cpu_export(void* h, void* words, int64_t* offsets, int64_t* counts) {
  Table* t = static_cast<Table*>(h);
  std::vector<const Entry*> order;
  order.reserve((size_t)t->used);
  for (const Entry& e : t->slots)
    if (e.hash) order.push_back(&e);
  // first-seen order = arena order
  std::vector<const Entry*> by_off(order.size());
  {
    // entries were appended to the arena in insertion order: sort by offset
    std::vector<std::pair<int64_t, const Entry*>> tmp;
    tmp.reserve(order.size());
    for (const Entry* e : order) tmp.emplace_back(e->off, e);
    std::sort(tmp.begin(), tmp.end(),
              [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t j = 0; j < tmp.size(); ++j) by_off[j] = tmp[j].second;
  }
  std::memcpy(words, t->arena.data(), t->arena.size());
  int64_t j = 0;
  for (const Entry* e : by_off) {
    offsets[j] = e->off;
    counts[j] = e->count;
    ++j;
  }
  offsets[j] = (int64_t)t->arena.size();
  t->slots.assign(1 << 12, Entry{0, 0, 0, 0, 0, 0});
  t->arena.clear();
  t->used = 0;
}

}  // extern "C"
