// K-Means Pipes GPU task binary (the GPU half of a hybrid K-Means job; see
// kmeans_pipes.h).  Runs on the device the scheduler chose — argv[1] /
// HadoopPipes::getGPUDeviceId(), which the fork never delivered.
//
// A long-lived child (hbmr.pipes.child.reuse; hbmr/pipes/mux.py keeps one per
// device and streams RUN_MAPs into it with several in flight), so everything
// expensive happens once per process or once per job, not per task:
//   * device state (stream, workspaces) is allocated on first use and grown;
//   * a split is read from its SequenceFile once (C++ reader, decoded into a
//     pinned staging buffer, one H2D) and kept resident in HBM keyed by the
//     split; later iterations skip the file (hbmr.pipes.split.cache.mb);
//   * the centroid image of a job (its centroid file, keyed by path, size and
//     mtime) is built once and shared by every map of the job.
//
// Two modes, chosen by the job's hbmr.kmeans.exact (as the framework's split
// job does):
//   * exact (default of the K-Means Pipes driver): labels are the fp64 arg-min
//     over the fp32 points — fp16 MFMA top-3 with step 1 of the certification
//     fused in, step 2 and the Elkan neighbour scan in fp64 (the library's
//     exact pipeline: hbmr_kmeans_exact_prep / image16 / centroid_nbr /
//     assign_top3_q1_grouped / refine_batch_finish) — and the partial sums are
//     the int64 fixed point of the fp32 rows (hbmr_kmeans_accum_f32).  The CPU
//     binary (kmeans_cpu.cc, hbmr_kmeans_map_cpu_f32_ex in exact mode) gives
//     the same labels and bit-identical partials, so a hybrid job's centroids
//     do not depend on which slots ran its maps;
//   * bf16: MFMA assign with a fused arg-max on padded bf16 rows and the
//     combiner over the bf16 copy (the round-3 binary).
#include <hip/hip_runtime.h>

#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <stdexcept>

#include "hbmr/hbmr.h"
#include "hadoop/TemplateFactory.hh"
#include "kmeans_pipes.h"

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " +             \
                                                   hipGetErrorString(e_));               \
  } while (0)

#define LIB_OK(x)                                                                        \
  do {                                                                                   \
    int r_ = (x);                                                                        \
    if (r_) throw std::runtime_error(std::string(#x) + " failed: " + std::to_string(r_)); \
  } while (0)

namespace {

constexpr int kNbrL = 256;     // exact mode's neighbour lists (hbmr.ops.kmeans.NBR_L)

// HBMR_PIPES_TRACE=<file>: "<wall seconds> <event>" lines appended per map
// phase (tools/trace_config2.py merges them into the tracker's timeline)
void tmark(const char* what) {
  static FILE* f = [] {
    const char* p = std::getenv("HBMR_PIPES_TRACE");
    return p && *p ? std::fopen(p, "a") : nullptr;
  }();
  if (!f) return;
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  std::fprintf(f, "%lld.%09ld child.%s\n", (long long)ts.tv_sec, ts.tv_nsec, what);
  std::fflush(f);
}

// A device buffer that only grows.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t bytes) {
    if (bytes > cap) {
      if (p) HIP_OK(hipFree(p));
      HIP_OK(hipMalloc(&p, bytes));
      cap = bytes;
    }
    return p;
  }
};

void* dalloc(size_t bytes) {
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, bytes ? bytes : 256));
  return p;
}

// A split resident in HBM: bf16 mode keeps the padded bf16 rows; exact mode
// the fp32 rows (padded to dp), their fp16 copy and the per-point norms.
struct CachedSplit {
  long n = 0;
  void* xb = nullptr;        // bf16 [n, dp]            (bf16 mode)
  float* x32 = nullptr;      // fp32 [n, dp]            (exact)
  void* x16 = nullptr;       // fp16 [n, dp]            (exact)
  float *xnorm = nullptr, *xbn2 = nullptr, *xerr = nullptr;
  size_t bytes = 0;
  void release() {
    for (void* p : {xb, (void*)x32, x16, (void*)xnorm, (void*)xbn2, (void*)xerr})
      if (p) HIP_OK(hipFree(p));
    *this = CachedSplit();
  }
};

// The centroid-side state of one job (one centroid file).
struct CentroidImage {
  std::string key;
  int k = 0, d = 0, dp = 0, kpad = 0, L = 0;
  bool exact = false;
  float* cen = nullptr;       // fp32 [k, d]
  void* cbf = nullptr;        // bf16 [kpad, dp] + chalf (bf16 mode)
  void *c16 = nullptr, *c16t = nullptr;   // fp16 [kpad, dp], tiled copy (exact)
  float *chalf = nullptr, *cnorm = nullptr, *cerr = nullptr, *maxima = nullptr;
  int32_t* nbr_i = nullptr;
  float *nbr_d = nullptr, *pd = nullptr;
  void release() {
    for (void* p : {(void*)cen, cbf, c16, c16t, (void*)chalf, (void*)cnorm, (void*)cerr,
                    (void*)maxima, (void*)nbr_i, (void*)nbr_d, (void*)pd})
      if (p) HIP_OK(hipFree(p));
    *this = CentroidImage();
  }
};

// Process-lifetime device state of this child.
struct DeviceState {
  int device = -1;
  hipStream_t st = nullptr;
  DevBuf x32stage, lab, sums, counts, ws, rws, stats;
  float* pinned = nullptr;
  size_t pinned_cap = 0;
  // a map's partials come back into pinned memory (a pageable 1 MB D2H at
  // k = 1024 is staged by the runtime) and are emitted from a block buffer
  // kept across maps (no 1 MB allocation and zero-fill per map)
  long long* hpart = nullptr;
  size_t hpart_cap = 0;
  std::string block;
  std::map<std::string, CachedSplit> splits;
  size_t cached_bytes = 0, cache_cap = 0;
  CentroidImage img;

  void init(int dev) {
    if (device >= 0) return;
    device = dev;
    HIP_OK(hipSetDevice(dev));
    HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const char* mb = getenv("HBMR_PIPES_SPLIT_CACHE_MB");
    cache_cap = (size_t)(mb ? atol(mb) : 65536) << 20;
  }

  long long* partials(size_t n) {
    if (n > hpart_cap) {
      if (hpart) HIP_OK(hipHostFree(hpart));
      HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&hpart), 8 * n));
      hpart_cap = n;
    }
    return hpart;
  }

  float* staging(size_t bytes) {
    if (bytes > pinned_cap) {
      if (pinned) HIP_OK(hipHostFree(pinned));
      HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&pinned), bytes));
      pinned_cap = bytes;
    }
    return pinned;
  }
};

DeviceState& state() {
  static DeviceState s;
  return s;
}

// path|size|mtime of a centroid file: a new file (the next iteration's) or a
// rewritten one gets a new image
std::string file_key(const std::string& path) {
  struct stat sb;
  if (stat(path.c_str(), &sb) != 0) throw std::runtime_error("cannot stat " + path);
  return path + "|" + std::to_string((long long)sb.st_size) + "|" +
         std::to_string((long long)sb.st_mtim.tv_sec) + "." +
         std::to_string((long long)sb.st_mtim.tv_nsec);
}

// Hands map() one record per split whose key is the raw FileSplit and whose
// value is empty: the mapper loads (or finds resident) the split itself.
class SplitDescReader : public HadoopPipes::RecordReader {
 public:
  explicit SplitDescReader(HadoopPipes::MapContext& ctx) : split_(ctx.getInputSplit()) {}
  bool next(std::string& key, std::string& value) override {
    if (done_) return false;
    key = split_;
    value.clear();
    done_ = true;
    return true;
  }
  float getProgress() override { return done_ ? 1.f : 0.f; }

 private:
  std::string split_;
  bool done_ = false;
};

}  // namespace

class KMeansGpuMapper : public HadoopPipes::Mapper {
 public:
  explicit KMeansGpuMapper(HadoopPipes::TaskContext& ctx) : p_(ctx.getJobConf()) {
    tmark("mapper.ctor");
    int device = HadoopPipes::getGPUDeviceId();
    if (device < 0) device = 0;
    DeviceState& S = state();
    S.init(device);
    const HadoopPipes::JobConf* conf = ctx.getJobConf();
    exact_ = conf->hasKey("hbmr.kmeans.exact") && conf->getBoolean("hbmr.kmeans.exact");
    dp_ = hbmr_kmeans_padded_dim(p_.d);
    if (dp_ < 0) throw std::runtime_error("dimension not supported by the MFMA kernel");
    if (exact_ && (dp_ > 128 || p_.d % 8))
      throw std::runtime_error("exact mode wants d % 8 == 0 and d <= 128");
    kpad_ = hbmr_kmeans_padded_k(p_.k);
    image(S);
    tmark("mapper.ready");
    points_ = ctx.getCounter("KMEANS", "POINTS");
    gpu_ = ctx.getCounter("KMEANS", "GPU_MAPS");
    hits_ = ctx.getCounter("KMEANS", "GPU_SPLIT_CACHE_HITS");
    flagged_ = ctx.getCounter("KMEANS", "EXACT_FLAGGED_POINTS");
    relabelled_ = ctx.getCounter("KMEANS", "EXACT_RELABELLED_POINTS");
  }

  // The job's centroid image, built on the first map of the job — into the
  // previous job's buffers when the shapes match (an iteration chain): a
  // hipFree synchronises the device, and freeing and re-allocating the eleven
  // buffers per job cost milliseconds before the job's first map
  void image(DeviceState& S) {
    const std::string key = file_key(p_.centroids) + (exact_ ? "|x" : "|b");
    CentroidImage& I = S.img;
    if (I.key == key) return;
    const std::vector<float> c = kmp::load_centroids(p_.centroids, p_.k, p_.d);
    tmark("image.loaded");
    const bool reuse = I.cen != nullptr && I.k == p_.k && I.d == p_.d && I.dp == dp_ &&
                       I.kpad == kpad_ && I.exact == exact_;
    if (!reuse) {
      I.release();
      I.k = p_.k;
      I.d = p_.d;
      I.dp = dp_;
      I.kpad = kpad_;
      I.exact = exact_;
      I.cen = static_cast<float*>(dalloc(sizeof(float) * c.size()));
      I.chalf = static_cast<float*>(dalloc(sizeof(float) * kpad_));
      if (!exact_) {
        I.cbf = dalloc(2 * (size_t)kpad_ * dp_);
      } else {
        I.c16 = dalloc(2 * (size_t)kpad_ * dp_);
        I.c16t = dalloc(2 * (size_t)kpad_ * dp_);
        I.cnorm = static_cast<float*>(dalloc(sizeof(float) * p_.k));
        I.cerr = static_cast<float*>(dalloc(sizeof(float) * p_.k));
        I.maxima = static_cast<float*>(dalloc(sizeof(float) * 2));
        I.L = std::min(kNbrL, p_.k);
        I.nbr_i = static_cast<int32_t*>(dalloc(sizeof(int32_t) * (size_t)p_.k * I.L));
        I.nbr_d = static_cast<float*>(dalloc(sizeof(float) * (size_t)p_.k * I.L));
        I.pd = static_cast<float*>(dalloc(sizeof(float) * (size_t)p_.k * p_.k));
      }
    }
    I.key.clear();
    HIP_OK(hipMemcpyAsync(I.cen, c.data(), sizeof(float) * c.size(), hipMemcpyHostToDevice, S.st));
    if (!exact_) {
      HIP_OK(hipMemsetAsync(I.cbf, 0, 2 * (size_t)kpad_ * dp_, S.st));
      // sums/counts == NULL: rebuild the bf16 image and -|c|²/2 from cen
      LIB_OK(hbmr_kmeans_update(nullptr, nullptr, p_.fx, p_.k, p_.d, dp_, kpad_, I.cen, I.cbf,
                                I.chalf, nullptr, S.st));
    } else {
      LIB_OK(hbmr_kmeans_image16(I.cen, p_.k, p_.d, dp_, kpad_, 1, I.c16, I.chalf, I.cnorm,
                                 I.cerr, I.maxima, S.st));
      LIB_OK(hbmr_kmeans_image16_tiled(I.c16, kpad_, dp_, I.c16t, S.st));
      LIB_OK(hbmr_kmeans_centroid_nbr(I.cen, p_.k, p_.d, I.L, I.nbr_i, I.nbr_d, I.pd, S.st));
    }
    // (the host vector c dies at return: the copy must have left it)
    HIP_OK(hipStreamSynchronize(S.st));
    I.key = key;
  }

  // The split in HBM: resident from an earlier task, or read now.
  const CachedSplit& split(const std::string& raw) {
    DeviceState& S = state();
    const std::string ckey = raw + (exact_ ? "|x" : "|b");
    auto it = S.splits.find(ckey);
    if (it != S.splits.end()) {
      cache_hit_ = true;
      return it->second;
    }
    cache_hit_ = false;
    const hbmr::io::FileSplitDesc desc = hbmr::io::parse_file_split(raw);
    hbmr::io::SeqSplitReader rr(desc.path, desc.start, desc.length);
    std::string kb, vb;
    std::vector<float> v;
    std::vector<float> host;
    long n = 0;
    while (rr.next(kb, vb)) {
      hbmr::io::decode_float_vector(vb, v);
      if ((int)v.size() != p_.d) throw std::runtime_error("point of wrong dimension");
      host.insert(host.end(), v.begin(), v.end());
      if (dp_ > p_.d) host.resize(host.size() + (dp_ - p_.d), 0.f);   // rows padded to dp
      ++n;
    }
    CachedSplit cs;
    cs.n = n;
    if (n > 0) {
      const size_t bytes = sizeof(float) * host.size();     // n * dp floats
      float* pin = S.staging(bytes);
      memcpy(pin, host.data(), bytes);
      if (exact_) {
        cs.x32 = static_cast<float*>(dalloc(bytes));
        HIP_OK(hipMemcpyAsync(cs.x32, pin, bytes, hipMemcpyHostToDevice, S.st));
        cs.x16 = dalloc(2 * (size_t)n * dp_);
        cs.xnorm = static_cast<float*>(dalloc(sizeof(float) * n));
        cs.xbn2 = static_cast<float*>(dalloc(sizeof(float) * n));
        cs.xerr = static_cast<float*>(dalloc(sizeof(float) * n));
        LIB_OK(hbmr_kmeans_exact_prep(cs.x32, n, p_.d, dp_, dp_, 1, cs.x16, cs.xnorm, cs.xbn2,
                                      cs.xerr, S.st));
        cs.bytes = bytes + 2 * (size_t)n * dp_ + 12 * (size_t)n;
      } else {
        float* x32 = static_cast<float*>(S.x32stage.get(bytes));
        HIP_OK(hipMemcpyAsync(x32, pin, bytes, hipMemcpyHostToDevice, S.st));
        cs.xb = dalloc(2 * (size_t)n * dp_);
        LIB_OK(hbmr_f32_to_bf16_pad(x32, n, dp_, dp_, cs.xb, S.st));
        cs.bytes = 2 * (size_t)n * dp_;
      }
      HIP_OK(hipStreamSynchronize(S.st));  // the staging buffer is reused next time
    }
    if (S.cached_bytes + cs.bytes > S.cache_cap) {
      tmp_ = cs;                            // over the cap: for this task only
      return tmp_;
    }
    S.cached_bytes += cs.bytes;
    return S.splits.emplace(ckey, cs).first->second;
  }

  void map(HadoopPipes::MapContext& ctx) override {
    DeviceState& S = state();
    const CentroidImage& I = S.img;
    tmark("map.start");
    const CachedSplit& cs = split(ctx.getInputKey());
    const long n = cs.n;
    const size_t nsums = (size_t)p_.k * dp_;
    long long* sums = S.partials(nsums + (size_t)p_.k);
    long long* counts = sums + nsums;
    unsigned long long st[5] = {0, 0, 0, 0, 0};
    if (n > 0) {
      const long wsb = hbmr_kmeans_accum_workspace_bytes(n, p_.k);
      int32_t* lab = static_cast<int32_t*>(S.lab.get(4 * (size_t)n));
      long long* dsums = static_cast<long long*>(S.sums.get(8 * nsums));
      long long* dcounts = static_cast<long long*>(S.counts.get(8 * (size_t)p_.k));
      void* ws = S.ws.get((size_t)wsb);
      HIP_OK(hipMemsetAsync(dsums, 0, 8 * nsums, S.st));
      HIP_OK(hipMemsetAsync(dcounts, 0, 8 * (size_t)p_.k, S.st));
      if (exact_) {
        auto* dstats = static_cast<unsigned long long*>(S.stats.get(sizeof(st)));
        HIP_OK(hipMemsetAsync(dstats, 0, sizeof(st), S.st));
        const long ns[1] = {n};
        const long rwb = hbmr_kmeans_refine_batch_bytes(1, ns);
        if (rwb < 0) throw std::runtime_error("refine workspace");
        void* rws = S.rws.get((size_t)rwb);
        const void* xs[1] = {cs.x16};
        const float* xn[1] = {cs.xnorm};
        const float* xb2[1] = {cs.xbn2};
        const float* xe[1] = {cs.xerr};
        // top-3 f16 MFMA assign with step 1 of the certification fused in
        LIB_OK(hbmr_kmeans_assign_top3_q1_grouped(1, xs, ns, dp_, 1, I.c16, I.c16t, I.chalf,
                                                  kpad_, lab, xn, xb2, xe, p_.d, p_.k, I.cnorm,
                                                  I.maxima, I.cerr, I.maxima + 1, rws, rwb, I.pd,
                                                  S.st));
        // step 2 (fp64 re-score of the flagged points) and the neighbour scan
        const float* x32s[1] = {cs.x32};
        int32_t* labs[1] = {lab};
        LIB_OK(hbmr_kmeans_refine_batch_finish(1, ns, x32s, labs, p_.d, dp_, I.cen, p_.k, kpad_,
                                               I.maxima, I.maxima + 1, I.nbr_i, I.nbr_d, I.L,
                                               dstats, 5, rws, rwb, S.st));
        // fixed point of the fp32 rows: the CPU binary's partials, bit for bit
        LIB_OK(hbmr_kmeans_accum_f32(cs.x32, n, dp_, lab, p_.k, dsums, dcounts, p_.fx, ws, wsb,
                                     0, S.st));
        HIP_OK(hipMemcpyAsync(st, dstats, sizeof(st), hipMemcpyDeviceToHost, S.st));
      } else {
        LIB_OK(hbmr_kmeans_assign_bf16(cs.xb, n, dp_, I.cbf, I.chalf, kpad_, lab, nullptr, S.st));
        LIB_OK(hbmr_kmeans_accum_bf16(cs.xb, n, dp_, lab, p_.k, dsums, dcounts, p_.fx, ws, wsb, 0,
                                      S.st));
      }
      HIP_OK(hipMemcpyAsync(sums, dsums, 8 * nsums, hipMemcpyDeviceToHost, S.st));
      HIP_OK(hipMemcpyAsync(counts, dcounts, 8 * (size_t)p_.k, hipMemcpyDeviceToHost, S.st));
      HIP_OK(hipStreamSynchronize(S.st));
    } else {
      std::memset(sums, 0, 8 * (nsums + (size_t)p_.k));
    }
    tmark("map.device_done");
    if (tmp_.n || tmp_.xb || tmp_.x32) tmp_.release();   // an uncached split
    kmp::emit_partials(ctx, p_, reinterpret_cast<const int64_t*>(sums), dp_,
                       reinterpret_cast<const int64_t*>(counts), &S.block);
    ctx.incrementCounter(points_, (uint64_t)n);
    ctx.incrementCounter(gpu_, 1);
    if (cache_hit_) ctx.incrementCounter(hits_, 1);
    if (exact_) {
      ctx.incrementCounter(flagged_, st[0]);
      ctx.incrementCounter(relabelled_, st[1]);
    }
  }

 private:
  kmp::Params p_;
  bool exact_ = false;
  int dp_ = 0, kpad_ = 0;
  bool cache_hit_ = false;
  CachedSplit tmp_;
  HadoopPipes::TaskContext::Counter* points_;
  HadoopPipes::TaskContext::Counter* gpu_;
  HadoopPipes::TaskContext::Counter* hits_;
  HadoopPipes::TaskContext::Counter* flagged_;
  HadoopPipes::TaskContext::Counter* relabelled_;
};

int main(int argc, char** argv) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<KMeansGpuMapper, kmp::KMeansReducer, void, void,
                                          SplitDescReader>())
             ? 0
             : 1;
}
