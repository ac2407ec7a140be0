// C ABI over the C++ SequenceFile reader/writer for dense float-vector data
// (SequenceFile<LongWritable, FloatVectorWritable>, the K-Means input format):
//
//   hbmr_seq_write_points  — n points as one SequenceFile (K-Means inputs and
//                            tests; the Python writer does ~100K records/s)
//   hbmr_seq_count_points  — records of a FileSplit (the exact split boundary
//                            rule of SequenceFileRecordReader)
//   hbmr_seq_read_points   — a FileSplit's vectors decoded straight into a
//                            caller buffer (pinned host memory on the GPU path,
//                            so the split goes to HBM in one hipMemcpyAsync)
//
// The file→HBM loader of SURVEY.md §2.6 (NativeIO row): no per-record Python.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "sequencefile.h"

namespace {

inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

thread_local std::string g_err;

}  // namespace

extern "C" {

const char* hbmr_seq_last_error() { return g_err.c_str(); }

// points: [n, d] fp32 (host order); keys first_id, first_id + 1, ...
int hbmr_seq_write_points(const char* path, const float* points, long n, int d, long first_id) {
  try {
    hbmr::io::SeqWriter w(path, "org.apache.hadoop.io.LongWritable",
                          "org.apache.hadoop.io.FloatVectorWritable");
    std::string key(8, '\0'), val(4 + 4 * (size_t)d, '\0');
    uint8_t* vp = reinterpret_cast<uint8_t*>(&val[0]);
    vp[0] = (uint8_t)(d >> 24);
    vp[1] = (uint8_t)(d >> 16);
    vp[2] = (uint8_t)(d >> 8);
    vp[3] = (uint8_t)d;
    for (long i = 0; i < n; ++i) {
      const uint64_t id = (uint64_t)(first_id + i);
      for (int b = 0; b < 8; ++b) key[b] = (char)(id >> (56 - 8 * b));
      const float* x = points + (size_t)i * d;
      for (int j = 0; j < d; ++j) {
        uint32_t u;
        memcpy(&u, x + j, 4);
        uint8_t* q = vp + 4 + 4 * j;
        q[0] = (uint8_t)(u >> 24);
        q[1] = (uint8_t)(u >> 16);
        q[2] = (uint8_t)(u >> 8);
        q[3] = (uint8_t)u;
      }
      w.append(key, val);
    }
    w.close();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
}

long hbmr_seq_count_points(const char* path, long start, long length) {
  try {
    hbmr::io::SeqSplitReader rr(path, start, length);
    std::string k, v;
    long n = 0;
    while (rr.next(k, v)) ++n;
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"

namespace {

// Uncompressed files: parse the records in place from a populated read-only
// mapping of the split's bytes (no per-record stdio reads or string copies) and
// byte-swap each vector straight into `out` (the loop vectorises to vpshufb).
// Same boundary rule as SeqSplitReader: after syncing to the first marker at
// or after `start`, records are taken until one that starts at or past the
// split end is preceded by a sync marker.
long read_points_mapped(hbmr::io::SeqReader& r, long start, long length, int d, float* out,
                        long cap) {
  const int64_t flen = r.file_length();
  const int64_t end = start + length;
  if (start > r.position()) r.sync_to(start);
  const int64_t pos0 = r.position();
  if (pos0 >= end || pos0 >= flen) return 0;
  const long page = sysconf(_SC_PAGESIZE);
  const int64_t map_off = pos0 / page * page;
  const int fd = open(r.path().c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + r.path());
  struct Map {
    int fd;
    void* p = MAP_FAILED;
    size_t n = 0;
    ~Map() {
      if (p != MAP_FAILED) munmap(p, n);
      close(fd);
    }
  } m{fd};
  // the split's bytes (+1 MiB for the records up to the next sync marker past
  // its end) populated in one go; the rest of the file only if the parse runs on
  int64_t mapped = std::min<int64_t>(flen - map_off, end - map_off + (1 << 20));
  m.n = (size_t)mapped;
  m.p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, map_off);
  if (m.p == MAP_FAILED) throw std::runtime_error("mmap failed for " + r.path());
  const uint8_t* b = static_cast<const uint8_t*>(m.p) - map_off;  // b[file offset]
  auto need = [&](int64_t upto) {  // bytes [.., upto) must be mapped
    if (upto <= map_off + mapped) return;
    munmap(m.p, m.n);
    mapped = flen - map_off;
    m.n = (size_t)mapped;
    m.p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, fd, map_off);
    if (m.p == MAP_FAILED) throw std::runtime_error("mmap failed for " + r.path());
    b = static_cast<const uint8_t*>(m.p) - map_off;
  };
  const uint8_t* sync = r.sync_bytes();
  const size_t rec_val = 4 + 4 * (size_t)d;
  int64_t pos = pos0;
  long n = 0;
  while (n < cap && pos + 4 <= flen) {
    const int64_t rec_pos = pos;
    bool sync_seen = false;
    need(pos + 4);
    int32_t len = (int32_t)be32(b + pos);
    if (len == -1) {
      if (pos + 4 + 16 > flen) throw std::runtime_error(r.path() + ": sync check failure");
      need(pos + 24);
      if (memcmp(b + pos + 4, sync, 16) != 0)
        throw std::runtime_error(r.path() + ": sync check failure");
      sync_seen = true;
      pos += 20;
      if (pos + 4 > flen) break;
      len = (int32_t)be32(b + pos);
    }
    if (rec_pos >= end && sync_seen) break;
    if (pos + 8 > flen) throw std::runtime_error("truncated record");
    const int32_t klen = (int32_t)be32(b + pos + 4);
    if (klen < 0 || klen > len || pos + 8 + len > flen) throw std::runtime_error("corrupt record");
    need(pos + 8 + len);
    const uint8_t* v = b + pos + 8 + klen;
    if ((size_t)(len - klen) < rec_val || (int)be32(v) != d)
      throw std::runtime_error("point of wrong dimension");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(v + 4);
    uint32_t* dst = reinterpret_cast<uint32_t*>(out + (size_t)n * d);
    for (int j = 0; j < d; ++j) {
      uint32_t u;
      memcpy(&u, src + j, 4);
      dst[j] = __builtin_bswap32(u);
    }
    pos += 8 + len;
    ++n;
  }
  return n;
}

}  // namespace

extern "C" {

// Decode up to `cap` records of the split into out[cap, d] (fp32); returns the
// count, or -1 on error (wrong dimension, I/O).
long hbmr_seq_read_points(const char* path, long start, long length, int d, float* out,
                          long cap) {
  try {
    {
      hbmr::io::SeqReader r(path);
      if (r.compression() == hbmr::io::Compression::NONE &&
          getenv("HBMR_SEQ_NO_MMAP") == nullptr)
        return read_points_mapped(r, start, length, d, out, cap);
    }
    hbmr::io::SeqSplitReader rr(path, start, length);
    std::string k, v;
    long n = 0;
    while (n < cap && rr.next(k, v)) {
      if (v.size() < 4) throw std::runtime_error("bad FloatVectorWritable");
      const uint8_t* p = reinterpret_cast<const uint8_t*>(v.data());
      if ((int)be32(p) != d || v.size() < 4 + 4 * (size_t)d)
        throw std::runtime_error("point of wrong dimension");
      float* o = out + (size_t)n * d;
      for (int j = 0; j < d; ++j) {
        const uint32_t u = be32(p + 4 + 4 * j);
        memcpy(o + j, &u, 4);
      }
      ++n;
    }
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"
