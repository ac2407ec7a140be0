// K-Means Pipes GPU task binary (the GPU half of a hybrid K-Means job; see
// kmeans_pipes.h).  Runs on the device the scheduler chose — argv[1] /
// HadoopPipes::getGPUDeviceId(), which the fork never delivered.
// The whole split goes to HBM in one copy: fp32 → bf16 (padded), MFMA assign
// with fused arg-max, sorted int64 fixed-point combiner (libhbmr kernels), and
// only the k×(d+1) partials come back.
#include <hip/hip_runtime.h>

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

class KMeansGpuMapper : public HadoopPipes::Mapper {
 public:
  explicit KMeansGpuMapper(HadoopPipes::TaskContext& ctx) : p_(ctx.getJobConf()) {
    device_ = HadoopPipes::getGPUDeviceId();
    if (device_ < 0) device_ = 0;
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    dp_ = hbmr_kmeans_padded_dim(p_.d);
    if (dp_ < 0) throw std::runtime_error("dimension not supported by the MFMA kernel");
    kpad_ = hbmr_kmeans_padded_k(p_.k);
    const std::vector<float> c = kmp::load_centroids(p_.centroids, p_.k, p_.d);
    HIP_OK(hipMalloc(&cen_, sizeof(float) * c.size()));
    HIP_OK(hipMalloc(&cbf_, 2 * (size_t)kpad_ * dp_));
    HIP_OK(hipMalloc(&chalf_, sizeof(float) * kpad_));
    HIP_OK(hipMemcpyAsync(cen_, c.data(), sizeof(float) * c.size(), hipMemcpyHostToDevice, st_));
    HIP_OK(hipMemsetAsync(cbf_, 0, 2 * (size_t)kpad_ * dp_, st_));
    // sums/counts == NULL: rebuild the bf16 image and -|c|²/2 from cen
    int rc = hbmr_kmeans_update(nullptr, nullptr, p_.fx, p_.k, p_.d, dp_, kpad_, cen_, cbf_,
                                chalf_, nullptr, st_);
    if (rc) throw std::runtime_error("hbmr_kmeans_update failed");
    points_ = ctx.getCounter("KMEANS", "POINTS");
    gpu_ = ctx.getCounter("KMEANS", "GPU_MAPS");
  }

  ~KMeansGpuMapper() override {
    hipFree(cen_);
    hipFree(cbf_);
    hipFree(chalf_);
    hipStreamDestroy(st_);
  }

  void map(HadoopPipes::MapContext& ctx) override {
    const std::string& v = ctx.getInputValue();
    const long n = (long)(v.size() / (sizeof(float) * p_.d));
    std::vector<long long> sums((size_t)p_.k * dp_), counts((size_t)p_.k);
    if (n > 0) {
      float* x32 = nullptr;
      void* xb = nullptr;
      int32_t* lab = nullptr;
      long long *dsums = nullptr, *dcounts = nullptr;
      void* ws = nullptr;
      const long wsb = hbmr_kmeans_accum_workspace_bytes(n, p_.k);
      HIP_OK(hipMalloc(&x32, v.size()));
      HIP_OK(hipMalloc(&xb, 2 * (size_t)n * dp_));
      HIP_OK(hipMalloc(&lab, 4 * (size_t)n));
      HIP_OK(hipMalloc(&dsums, 8 * sums.size()));
      HIP_OK(hipMalloc(&dcounts, 8 * counts.size()));
      HIP_OK(hipMalloc(&ws, (size_t)wsb));
      HIP_OK(hipMemcpyAsync(x32, v.data(), v.size(), hipMemcpyHostToDevice, st_));
      HIP_OK(hipMemsetAsync(dsums, 0, 8 * sums.size(), st_));
      HIP_OK(hipMemsetAsync(dcounts, 0, 8 * counts.size(), st_));
      int rc = hbmr_f32_to_bf16_pad(x32, n, p_.d, dp_, xb, st_);
      if (!rc) rc = hbmr_kmeans_assign_bf16(xb, n, dp_, cbf_, chalf_, kpad_, lab, nullptr, st_);
      if (!rc)
        rc = hbmr_kmeans_accum_bf16(xb, n, dp_, lab, p_.k, dsums, dcounts, p_.fx, ws, wsb, 0, st_);
      if (rc) throw std::runtime_error("K-Means kernels failed: " + std::to_string(rc));
      HIP_OK(hipMemcpyAsync(sums.data(), dsums, 8 * sums.size(), hipMemcpyDeviceToHost, st_));
      HIP_OK(hipMemcpyAsync(counts.data(), dcounts, 8 * counts.size(), hipMemcpyDeviceToHost, st_));
      HIP_OK(hipStreamSynchronize(st_));
      hipFree(x32);
      hipFree(xb);
      hipFree(lab);
      hipFree(dsums);
      hipFree(dcounts);
      hipFree(ws);
    }
    kmp::emit_partials(ctx, p_.k, p_.d, reinterpret_cast<const int64_t*>(sums.data()), dp_,
                       reinterpret_cast<const int64_t*>(counts.data()));
    ctx.incrementCounter(points_, (uint64_t)n);
    ctx.incrementCounter(gpu_, 1);
  }

 private:
  kmp::Params p_;
  int device_ = 0, dp_ = 0, kpad_ = 0;
  hipStream_t st_ = nullptr;
  float* cen_ = nullptr;
  void* cbf_ = nullptr;
  float* chalf_ = nullptr;
  HadoopPipes::TaskContext::Counter* points_;
  HadoopPipes::TaskContext::Counter* gpu_;
};

int main(int argc, char** argv) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<KMeansGpuMapper, kmp::KMeansReducer, void, void,
                                          kmp::SplitPointsReader>())
             ? 0
             : 1;
}
