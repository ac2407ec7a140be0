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
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <vector>

namespace {

struct Entry {
  uint64_t hash;   // 0 = empty slot
  int64_t off;     // word bytes in the arena
  int32_t len;
  int64_t count;
};

inline bool is_space(unsigned char c) {
  return c == ' ' || (c >= '\t' && c <= '\r');
}

inline uint64_t mix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h | 1;   // never 0 (the empty marker)
}

inline uint64_t hash_bytes(const unsigned char* p, int64_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)n;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x100000001B3ULL;
    h ^= h >> 29;
  }
  uint64_t w = 0;
  std::memcpy(&w, p + i, (size_t)(n - i));
  h = (h ^ w) * 0x100000001B3ULL;
  return mix(h);
}

struct Table {
  std::vector<Entry> slots;
  std::vector<unsigned char> arena;
  int64_t used = 0;
  int64_t tokens = 0;

  Table() : slots(1 << 16) {}

  void grow() {
    std::vector<Entry> old;
    old.swap(slots);
    slots.assign(old.size() * 2, Entry{0, 0, 0, 0});
    const uint64_t mask = slots.size() - 1;
    for (const Entry& e : old) {
      if (!e.hash) continue;
      uint64_t i = e.hash & mask;
      while (slots[i].hash) i = (i + 1) & mask;
      slots[i] = e;
    }
  }

  void add(const unsigned char* w, int64_t n) {
    ++tokens;
    const uint64_t h = hash_bytes(w, n);
    uint64_t mask = slots.size() - 1;
    uint64_t i = h & mask;
    for (;;) {
      Entry& e = slots[i];
      if (!e.hash) break;
      if (e.hash == h && e.len == n && std::memcmp(arena.data() + e.off, w, (size_t)n) == 0) {
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
    e.off = (int64_t)arena.size();
    e.len = (int32_t)n;
    e.count = 1;
    arena.insert(arena.end(), w, w + n);
    ++used;
  }
};

}  // namespace

extern "C" {

void* hbmr_wc_cpu_new() { return new Table(); }

void hbmr_wc_cpu_free(void* h) { delete static_cast<Table*>(h); }

// Count the tokens of buf[0, n); returns the number of distinct words so far.
int64_t hbmr_wc_cpu_add(void* h, const void* buf, int64_t n) {
  Table* t = static_cast<Table*>(h);
  const unsigned char* p = static_cast<const unsigned char*>(buf);
  int64_t i = 0;
  while (i < n) {
    while (i < n && is_space(p[i])) ++i;
    const int64_t s = i;
    while (i < n && !is_space(p[i])) ++i;
    if (i > s) t->add(p + s, i - s);
  }
  return t->used;
}

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
  t->slots.assign(1 << 16, Entry{0, 0, 0, 0});
  t->arena.clear();
  t->used = 0;
}

}  // extern "C"
