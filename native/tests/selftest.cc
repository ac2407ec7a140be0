// Host self-test of the native runtime pieces, built under ASAN+UBSAN and TSAN
// by `python native/build.py sanitize asan|tsan` (tests/test_sanitizers.py):
// map-output sort/partition/IFile kernels, SequenceFile write/read/split read,
// VInt codec, and the multi-threaded CPU K-Means map.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "hbmr/hbmr.h"
#include "../io/sequencefile.h"

extern "C" {
void hbmr_hash_partition(int kind, const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                         int64_t n, int R, int32_t* part);
void hbmr_sort_records(int kind, const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                       int64_t n, const int32_t* part, int64_t* perm);
int64_t hbmr_group_runs(int kind, const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                        const int64_t* perm, int64_t lo, int64_t hi, int64_t* ends);
int64_t hbmr_ifile_encode(const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                          const uint8_t* vbuf, const int64_t* vpos, const int64_t* vlen,
                          const int64_t* perm, int64_t lo, int64_t hi, uint8_t* out);
int64_t hbmr_ifile_decode(const uint8_t* buf, int64_t n, int64_t cap, int64_t* kpos,
                          int64_t* klen, int64_t* vpos, int64_t* vlen);
}

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "selftest: check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

static int test_mapout() {
  std::mt19937 rng(7);
  const int n = 5000, R = 7;
  std::string kbuf, vbuf;
  std::vector<int64_t> kpos, klen, vpos, vlen;
  for (int i = 0; i < n; ++i) {
    const int len = 1 + rng() % 12;
    std::string w;
    for (int j = 0; j < len; ++j) w.push_back(char('a' + rng() % 6));
    kpos.push_back((int64_t)kbuf.size());
    kbuf.push_back((char)len);  // Text: one-byte VInt length
    kbuf += w;
    klen.push_back(len + 1);
    vpos.push_back((int64_t)vbuf.size());
    vbuf += std::string("\x00\x00\x00\x01", 4);
    vlen.push_back(4);
  }
  std::vector<int32_t> part(n);
  hbmr_hash_partition(0, (const uint8_t*)kbuf.data(), kpos.data(), klen.data(), n, R, part.data());
  for (int i = 0; i < n; ++i) CHECK(part[i] >= 0 && part[i] < R);
  std::vector<int64_t> perm(n);
  hbmr_sort_records(0, (const uint8_t*)kbuf.data(), kpos.data(), klen.data(), n, part.data(),
                    perm.data());
  for (int i = 1; i < n; ++i) {
    const int64_t a = perm[i - 1], b = perm[i];
    CHECK(part[a] <= part[b]);
    if (part[a] == part[b]) {
      const std::string ka = kbuf.substr(kpos[a] + 1, klen[a] - 1);
      const std::string kb = kbuf.substr(kpos[b] + 1, klen[b] - 1);
      CHECK(ka <= kb);
    }
  }
  std::vector<int64_t> ends(n);
  const int64_t runs = hbmr_group_runs(0, (const uint8_t*)kbuf.data(), kpos.data(), klen.data(),
                                       perm.data(), 0, n, ends.data());
  CHECK(runs > 0 && ends[runs - 1] == n);
  std::vector<uint8_t> out(kbuf.size() + vbuf.size() + 10 * n + 4);
  const int64_t bytes = hbmr_ifile_encode((const uint8_t*)kbuf.data(), kpos.data(), klen.data(),
                                          (const uint8_t*)vbuf.data(), vpos.data(), vlen.data(),
                                          perm.data(), 0, n, out.data());
  CHECK(bytes > 0 && bytes <= (int64_t)out.size());
  std::vector<int64_t> dk(n), dkl(n), dv(n), dvl(n);
  const int64_t nr = hbmr_ifile_decode(out.data(), bytes, n, dk.data(), dkl.data(), dv.data(),
                                       dvl.data());
  CHECK(nr == n);
  for (int i = 0; i < n; ++i) {
    const int64_t r = perm[i];
    CHECK(dkl[i] == klen[r] && std::memcmp(out.data() + dk[i], kbuf.data() + kpos[r], klen[r]) == 0);
    CHECK(dvl[i] == 4);
  }
  CHECK(hbmr_ifile_decode(out.data(), bytes - 3, n, dk.data(), dkl.data(), dv.data(),
                          dvl.data()) < n);
  return 0;
}

static int test_seqfile(const std::string& dir) {
  using namespace hbmr::io;
  const std::string path = dir + "/selftest.seq";
  const int n = 3000;
  {
    SeqWriter w(path, "org.apache.hadoop.io.Text", "org.apache.hadoop.io.IntWritable");
    for (int i = 0; i < n; ++i) {
      std::string k;
      const std::string s = "key" + std::to_string(i);
      write_vlong(k, (int64_t)s.size());
      k += s;
      w.append(k, encode_int_writable(i));
    }
    w.close();
  }
  {
    SeqReader r(path);
    std::string k, v;
    int i = 0;
    while (r.next(k, v)) {
      CHECK(decode_int_writable(v) == i);
      ++i;
    }
    CHECK(i == n);
  }
  // splits cover every record exactly once
  FILE* f = std::fopen(path.c_str(), "rb");
  std::fseek(f, 0, SEEK_END);
  const int64_t len = std::ftell(f);
  std::fclose(f);
  int total = 0;
  for (int64_t s = 0; s < len; s += 4096) {
    SeqSplitReader sr(path, s, std::min<int64_t>(4096, len - s));
    std::string k, v;
    while (sr.next(k, v)) ++total;
  }
  CHECK(total == n);
  std::string enc;
  for (int64_t x : {0LL, 1LL, -1LL, 127LL, -112LL, -113LL, 128LL, 1LL << 40, -(1LL << 40)}) {
    enc.clear();
    write_vlong(enc, x);
    const uint8_t* p = (const uint8_t*)enc.data();
    CHECK(read_vlong(p, p + enc.size()) == x);
  }
  return 0;
}

static int test_kmeans_cpu() {
  const long n = 4000;
  const int d = 16, k = 8;
  std::vector<float> X(n * d), C(k * d);
  std::mt19937 rng(3);
  std::normal_distribution<float> g;
  for (auto& x : X) x = g(rng);
  for (int j = 0; j < k * d; ++j) C[j] = X[j];
  std::vector<int32_t> labels(n);
  std::vector<long long> sums(k * d), counts(k);
  double cost = 0;
  CHECK(hbmr_kmeans_map_cpu_f32(X.data(), n, d, C.data(), k, labels.data(), sums.data(),
                                counts.data(), &cost, 24, 4) == 0);
  long long tot = 0;
  for (auto c : counts) tot += c;
  CHECK(tot == n);
  return 0;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  if (test_mapout() || test_seqfile(dir) || test_kmeans_cpu()) return 1;
  std::printf("selftest ok\n");
  return 0;
}
