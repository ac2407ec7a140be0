// K-Means Pipes task binaries (BASELINE config 2: hybrid Pipes job with a CPU
// binary and a GPU binary, as the fork's users ran K-Means — one Lloyd
// iteration per job, centroids side-loaded from a file).
//
// Shared by kmeans_cpu.cc (CPU slots) and kmeans_gpu.hip (GPU slots):
//   * SplitPointsReader — C++ RecordReader: reads the task's FileSplit of a
//     SequenceFile<LongWritable, FloatVectorWritable> and hands the WHOLE split
//     to map() as one record (value = n×d native fp32), so a GPU map is one
//     H2D + a few kernels instead of the reference's per-record MAP_ITEM
//     messages (SURVEY.md §2.9 "Pipes socket");
//   * partial encoding — key = cluster id (decimal), value = int64 count +
//     d int64 fixed-point sums (Σ round(x·2^fx)), so partials combine exactly
//     whatever CPU/GPU mix produced them;
//   * KMeansReducer — sums the partials of a cluster and emits the new centroid
//     as comma-separated floats (key = cluster id);
//   * block mode (hbmr.kmeans.pipes.block): a map emits ONE record, key "*",
//     whose value packs every non-empty cluster's (int32 id, int64 count,
//     d int64 sums) — in-mapper combining: one frame per map through the
//     parent instead of k (k = 1024 at the headline shape) — and the reducer,
//     given the "*" group, sums the blocks and emits the same per-cluster
//     centroid lines.  Same int64 partials, so the result is bit-identical.
//
// Job keys: hbmr.kmeans.k, hbmr.kmeans.dims, hbmr.kmeans.centroids.file
// (SequenceFile<IntWritable, FloatVectorWritable>), hbmr.kmeans.fx.shift (24),
// hbmr.kmeans.pipes.block (false).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../io/sequencefile.h"
#include "hadoop/Pipes.hh"
#include "hadoop/StringUtils.hh"

namespace kmp {

constexpr const char* kBlockKey = "*";

struct Params {
  int k = 0, d = 0, fx = 24;
  bool block = false, binary = false;
  std::string centroids;
  explicit Params(const HadoopPipes::JobConf* conf) {
    k = conf->getInt("hbmr.kmeans.k");
    d = conf->getInt("hbmr.kmeans.dims");
    if (conf->hasKey("hbmr.kmeans.fx.shift")) fx = conf->getInt("hbmr.kmeans.fx.shift");
    block = conf->hasKey("hbmr.kmeans.pipes.block") && conf->getBoolean("hbmr.kmeans.pipes.block");
    binary = conf->hasKey("hbmr.kmeans.pipes.binary.output") &&
             conf->getBoolean("hbmr.kmeans.pipes.binary.output");
    centroids = conf->get("hbmr.kmeans.centroids.file");
    if (centroids.rfind("file:", 0) == 0) centroids = centroids.substr(5);
  }
};

// [k, d] fp32 centroids from SequenceFile<IntWritable, FloatVectorWritable>.
inline std::vector<float> load_centroids(const std::string& path, int k, int d) {
  std::vector<float> c((size_t)k * d, 0.f);
  hbmr::io::SeqReader r(path);
  std::string kb, vb;
  std::vector<float> v;
  int seen = 0;
  while (r.next(kb, vb)) {
    const int j = hbmr::io::decode_int_writable(kb);
    hbmr::io::decode_float_vector(vb, v);
    if (j < 0 || j >= k || (int)v.size() != d) throw std::runtime_error("bad centroid record");
    memcpy(&c[(size_t)j * d], v.data(), sizeof(float) * d);
    ++seen;
  }
  if (seen != k) throw std::runtime_error("centroid file has " + std::to_string(seen) + " of " +
                                          std::to_string(k) + " centroids");
  return c;
}

class SplitPointsReader : public HadoopPipes::RecordReader {
 public:
  explicit SplitPointsReader(HadoopPipes::MapContext& ctx) : done_(false) {
    const Params p(ctx.getJobConf());
    const hbmr::io::FileSplitDesc s = hbmr::io::parse_file_split(ctx.getInputSplit());
    key_ = s.path + ":" + std::to_string(s.start);
    hbmr::io::SeqSplitReader rr(s.path, s.start, s.length);
    std::string kb, vb;
    std::vector<float> v;
    while (rr.next(kb, vb)) {
      hbmr::io::decode_float_vector(vb, v);
      if ((int)v.size() != p.d) throw std::runtime_error("point of wrong dimension");
      data_.append(reinterpret_cast<const char*>(v.data()), sizeof(float) * v.size());
    }
  }
  bool next(std::string& key, std::string& value) override {
    if (done_) return false;
    key = key_;
    value.swap(data_);
    done_ = true;
    return true;
  }
  float getProgress() override { return done_ ? 1.f : 0.f; }

 private:
  bool done_;
  std::string key_, data_;
};

inline std::string encode_partial(int64_t count, const int64_t* sums, int d) {
  std::string v(8 * (size_t)(d + 1), '\0');
  memcpy(&v[0], &count, 8);
  memcpy(&v[8], sums, 8 * (size_t)d);
  return v;
}

// ``buf``: a block-mode buffer the caller keeps across maps (its capacity is
// reused: no allocation and zero-fill of ~1 MB per map at k = 1024)
inline void emit_partials(HadoopPipes::MapContext& ctx, const Params& p, const int64_t* sums,
                          int sums_stride, const int64_t* counts,
                          std::string* buf = nullptr) {
  const int k = p.k, d = p.d;
  if (!p.block) {
    for (int j = 0; j < k; ++j)
      if (counts[j] > 0)
        ctx.emit(HadoopUtils::toString(j),
                 encode_partial(counts[j], sums + (size_t)j * sums_stride, d));
    return;
  }
  const size_t rec = 4 + 8 * (size_t)(d + 1);
  int used = 0;
  for (int j = 0; j < k; ++j) used += counts[j] > 0;
  std::string local;
  std::string& v = buf ? *buf : local;
  v.resize(rec * (size_t)used);
  char* o = &v[0];
  for (int j = 0; j < k; ++j) {
    if (counts[j] <= 0) continue;
    const int32_t id = j;
    memcpy(o, &id, 4);
    memcpy(o + 4, &counts[j], 8);
    memcpy(o + 12, sums + (size_t)j * sums_stride, 8 * (size_t)d);
    o += rec;
  }
  ctx.emit(kBlockKey, v);
}

inline std::string centroid_text(const int64_t* s, int64_t cnt, int d, int fx) {
  std::string out;
  char buf[32];
  const double inv = std::ldexp(1.0, -fx) / (double)cnt;
  for (int i = 0; i < d; ++i) {
    snprintf(buf, sizeof(buf), i ? ",%.9g" : "%.9g", (float)((double)s[i] * inv));
    out += buf;
  }
  return out;
}

// A new centroid as the reducer's output value: comma-separated %.9g floats
// (text; every fp32 round-trips), or (hbmr.kmeans.pipes.binary.output) the d
// fp32 values as little-endian bytes — the same floats without 131k snprintf
// calls in the reducer and as many parses in the driver at k = 1024
inline std::string centroid_value(const int64_t* s, int64_t cnt, int d, int fx, bool binary) {
  const double inv = std::ldexp(1.0, -fx) / (double)cnt;
  if (binary) {
    std::string out(4 * (size_t)d, '\0');
    for (int i = 0; i < d; ++i) {
      const float f = (float)((double)s[i] * inv);
      memcpy(&out[4 * (size_t)i], &f, 4);
    }
    return out;
  }
  return centroid_text(s, cnt, d, fx);
}

class KMeansReducer : public HadoopPipes::Reducer {
 public:
  explicit KMeansReducer(HadoopPipes::TaskContext& ctx) : p_(ctx.getJobConf()) {}
  void reduce(HadoopPipes::ReduceContext& ctx) override {
    if (ctx.getInputKey() == kBlockKey) {
      reduce_blocks(ctx);
      return;
    }
    int64_t cnt = 0;
    std::vector<int64_t> s((size_t)p_.d, 0), part((size_t)p_.d);
    while (ctx.nextValue()) {
      const std::string& v = ctx.getInputValue();
      if (v.size() != 8 * (size_t)(p_.d + 1)) throw std::runtime_error("bad partial");
      int64_t c;
      memcpy(&c, v.data(), 8);
      memcpy(part.data(), v.data() + 8, 8 * (size_t)p_.d);
      cnt += c;
      for (int i = 0; i < p_.d; ++i) s[i] += part[i];
    }
    ctx.emit(ctx.getInputKey(), centroid_value(s.data(), cnt, p_.d, p_.fx, p_.binary));
  }

  // every map's block (block mode): per-cluster sums over all of them, then
  // one centroid line per non-empty cluster, in cluster order
  void reduce_blocks(HadoopPipes::ReduceContext& ctx) {
    const int k = p_.k, d = p_.d;
    const size_t rec = 4 + 8 * (size_t)(d + 1);
    std::vector<int64_t> cnt((size_t)k, 0), s((size_t)k * d, 0), part((size_t)d);
    while (ctx.nextValue()) {
      const std::string& v = ctx.getInputValue();
      if (v.size() % rec) throw std::runtime_error("bad partials block");
      for (const char* o = v.data(); o < v.data() + v.size(); o += rec) {
        int32_t j;
        int64_t c;
        memcpy(&j, o, 4);
        memcpy(&c, o + 4, 8);
        if (j < 0 || j >= k) throw std::runtime_error("bad cluster id in partials block");
        memcpy(part.data(), o + 12, 8 * (size_t)d);
        cnt[j] += c;
        int64_t* sj = &s[(size_t)j * d];
        for (int i = 0; i < d; ++i) sj[i] += part[i];
      }
    }
    for (int j = 0; j < k; ++j)
      if (cnt[j] > 0)
        ctx.emit(HadoopUtils::toString(j),
                 centroid_value(&s[(size_t)j * d], cnt[j], d, p_.fx, p_.binary));
  }

 private:
  Params p_;
};

}  // namespace kmp
