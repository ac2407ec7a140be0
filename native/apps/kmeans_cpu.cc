// K-Means Pipes CPU task binary (the CPU half of a hybrid K-Means job; see
// kmeans_pipes.h).  The map runs the native multi-threaded fp32 assignment
// (exact mode: certified, uncertain points re-scored in fp64) + int64
// fixed-point combiner of native/cpu/kmeans_cpu.cc over the whole split.
#include <stdexcept>
#include <thread>

#include "hbmr/hbmr.h"
#include "hadoop/TemplateFactory.hh"
#include "kmeans_pipes.h"

class KMeansCpuMapper : public HadoopPipes::Mapper {
 public:
  explicit KMeansCpuMapper(HadoopPipes::TaskContext& ctx) : p_(ctx.getJobConf()) {
    cen_ = kmp::load_centroids(p_.centroids, p_.k, p_.d);
    const HadoopPipes::JobConf* conf = ctx.getJobConf();
    threads_ = conf->hasKey("hbmr.cpu.threads.per.slot") ? conf->getInt("hbmr.cpu.threads.per.slot")
                                                          : 1;
    // exact mode (hbmr.kmeans.exact): fp32 scores certified against their
    // error bound, uncertain points re-scored in fp64 — the fp64 arg-min the
    // GPU binary's exact pipeline also gives, so both emit the same partials
    exact_ = conf->hasKey("hbmr.kmeans.exact") && conf->getBoolean("hbmr.kmeans.exact");
    points_ = ctx.getCounter("KMEANS", "POINTS");
    cpu_ = ctx.getCounter("KMEANS", "CPU_MAPS");
  }
  void map(HadoopPipes::MapContext& ctx) override {
    const std::string& v = ctx.getInputValue();
    const long n = (long)(v.size() / (sizeof(float) * p_.d));
    std::vector<int32_t> labels((size_t)n);
    std::vector<long long> sums((size_t)p_.k * p_.d, 0), counts((size_t)p_.k, 0);
    double cost = 0;
    long rescored = 0;
    const int rc = hbmr_kmeans_map_cpu_f32_ex(reinterpret_cast<const float*>(v.data()), n, p_.d,
                                              cen_.data(), p_.k, labels.data(), sums.data(),
                                              counts.data(), &cost, p_.fx, threads_,
                                              exact_ ? 1 : 0, &rescored);
    if (rc) throw std::runtime_error("hbmr_kmeans_map_cpu_f32_ex failed");
    ctx.incrementCounter(cpu_, 1);
    kmp::emit_partials(ctx, p_, reinterpret_cast<const int64_t*>(sums.data()), p_.d,
                       reinterpret_cast<const int64_t*>(counts.data()));
    ctx.incrementCounter(points_, (uint64_t)n);
  }

 private:
  kmp::Params p_;
  std::vector<float> cen_;
  int threads_ = 1;
  bool exact_ = false;
  HadoopPipes::TaskContext::Counter* points_;
  HadoopPipes::TaskContext::Counter* cpu_;
};

int main(int argc, char** argv) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<KMeansCpuMapper, kmp::KMeansReducer, void, void,
                                          kmp::SplitPointsReader>())
             ? 0
             : 1;
}
