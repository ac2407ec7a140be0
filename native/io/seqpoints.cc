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
#include <cstdint>
#include <cstring>
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

// Decode up to `cap` records of the split into out[cap, d] (fp32); returns the
// count, or -1 on error (wrong dimension, I/O).
long hbmr_seq_read_points(const char* path, long start, long length, int d, float* out,
                          long cap) {
  try {
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
