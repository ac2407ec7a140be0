// CPU K-Means map + combiner, used by CPU map slots of the hybrid scheduler
// (the CPU side of SURVEY.md G1/G4: "mapred.tasktracker.map.cpu.tasks.maximum"
// slots run the job's CPU binary, hadoop-1.0.3/src/mapred/org/apache/hadoop/
// mapred/pipes/Application.java:162-170 picks cache slot 0 for CPU tasks).
//
// Same contract as the GPU path: labels[i] = argmin_j ||x_i - c_j||² and
// per-cluster (sum, count) partials.  fp32 throughout; blocked so the centroid
// panel stays in L1/L2 while a block of points streams.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/hbmr/hbmr.h"

namespace {

constexpr int kPB = 32;   // points per block
constexpr int kCB = 64;   // centroids per panel

inline float dot(const float* __restrict__ a, const float* __restrict__ b, int d) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, s5 = 0.f, s6 = 0.f, s7 = 0.f;
  int i = 0;
  for (; i + 8 <= d; i += 8) {
    s0 += a[i] * b[i]; s1 += a[i + 1] * b[i + 1]; s2 += a[i + 2] * b[i + 2];
    s3 += a[i + 3] * b[i + 3]; s4 += a[i + 4] * b[i + 4]; s5 += a[i + 5] * b[i + 5];
    s6 += a[i + 6] * b[i + 6]; s7 += a[i + 7] * b[i + 7];
  }
  for (; i < d; ++i) s0 += a[i] * b[i];
  return ((s0 + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7));
}

// Exact mode: a point whose fp32 margin (best - runner-up score) is within
// twice the fp32 error bound E = (d+2)·2^-23·(|x|·cmax + cmax²/2) of any score
// is re-scored against every centroid in fp64; all others are certified
// (every other cluster scores at most the runner-up).
int rescore_fp64(const float* x, int d, const float* C, int k) {
  double best = 0.0;
  int bi = 0;
  for (int j = 0; j < k; ++j) {
    double s = 0.0;
    for (int t = 0; t < d; ++t) {
      const double e = (double)x[t] - (double)C[(long)j * d + t];
      s += e * e;
    }
    if (j == 0 || s < best) { best = s; bi = j; }
  }
  return bi;
}

void worker(const float* X, long lo, long hi, int d, const float* C, const float* chalf, int k,
            int32_t* labels, long long* sums, long long* counts, double* cost, float scale,
            bool exact, double cmax, long* rescored) {
  std::vector<float> best(kPB), second(kPB);
  std::vector<int> bidx(kPB);
  double c = 0.0;
  long nres = 0;
  for (long p0 = lo; p0 < hi; p0 += kPB) {
    const int np = (int)std::min<long>(kPB, hi - p0);
    for (int i = 0; i < np; ++i) {
      best[i] = second[i] = -3.0e38f;
      bidx[i] = 0;
    }
    for (int j0 = 0; j0 < k; j0 += kCB) {
      const int nj = std::min(kCB, k - j0);
      for (int i = 0; i < np; ++i) {
        const float* x = X + (p0 + i) * (long)d;
        float bv = best[i], sv = second[i];
        int bi = bidx[i];
        for (int j = 0; j < nj; ++j) {
          const float s = dot(x, C + (long)(j0 + j) * d, d) + chalf[j0 + j];
          if (s > bv) { sv = bv; bv = s; bi = j0 + j; }
          else if (s > sv) sv = s;
        }
        best[i] = bv;
        second[i] = sv;
        bidx[i] = bi;
      }
    }
    for (int i = 0; i < np; ++i) {
      const long p = p0 + i;
      int lab = bidx[i];
      if (exact && k > 1) {
        const float* x = X + p * (long)d;
        double xn = 0.0;
        for (int t = 0; t < d; ++t) xn += (double)x[t] * x[t];
        xn = std::sqrt(xn) * (1.0 + 1e-6);
        const double e = (d + 2) * std::ldexp(1.0, -23) * 1.01 * (xn * cmax + 0.5 * cmax * cmax);
        if ((double)best[i] - (double)second[i] <= 2.0 * e + std::fabs((double)best[i]) * 1e-6) {
          lab = rescore_fp64(x, d, C, k);
          ++nres;
        }
      }
      if (labels) labels[p] = lab;
      const float* x = X + p * (long)d;
      long long* s = sums + (long)lab * d;
      float nx = 0.f;
      for (int t = 0; t < d; ++t) {
        s[t] += std::llrint(x[t] * scale);
        nx += x[t] * x[t];
      }
      counts[lab] += 1;
      c += (double)nx - 2.0 * (double)best[i];
    }
  }
  *cost = c;
  *rescored = nres;
}

}  // namespace

// sums / counts: 64-bit fixed point, identical encoding to the GPU combiner
// (native/kernels/kmeans.hip): sum = Σ round(x · 2^fx_shift).
// exact != 0: fp32 scoring certified per point, fp64 re-score of near ties
// (hbmr.kmeans.exact); *rescored (if given) += re-scored points.
extern "C" int hbmr_kmeans_map_cpu_f32_ex(const float* X, long n, int d, const float* C, int k,
                                          int32_t* labels, long long* sums, long long* counts,
                                          double* cost, int fx_shift, int nthreads, int exact,
                                          long* rescored) {
  const float scale = std::ldexp(1.0f, fx_shift);
  if (n < 0 || d <= 0 || k <= 0) return -22;
  std::vector<float> chalf(k);
  double cmax = 0.0;
  for (int j = 0; j < k; ++j) {
    float s = 0.f;
    double s64 = 0.0;
    for (int t = 0; t < d; ++t) {
      s += C[(long)j * d + t] * C[(long)j * d + t];
      s64 += (double)C[(long)j * d + t] * C[(long)j * d + t];
    }
    chalf[j] = -0.5f * s;
    cmax = std::max(cmax, std::sqrt(s64) * (1.0 + 1e-6));
  }
  if (nthreads < 1) nthreads = 1;
  const long per = (n + nthreads - 1) / nthreads;
  std::vector<std::vector<long long>> ps(nthreads), pc(nthreads);
  std::vector<double> costs(nthreads, 0.0);
  std::vector<long> res(nthreads, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    const long lo = t * per, hi = std::min(n, lo + per);
    if (lo >= hi) break;
    ps[t].assign((size_t)k * d, 0);
    pc[t].assign(k, 0);
    th.emplace_back(worker, X, lo, hi, d, C, chalf.data(), k, labels, ps[t].data(), pc[t].data(),
                    &costs[t], scale, exact != 0, cmax, &res[t]);
  }
  for (auto& x : th) x.join();
  double total = 0.0;
  for (size_t t = 0; t < th.size(); ++t) {
    for (size_t i = 0; i < (size_t)k * d; ++i) sums[i] += ps[t][i];
    for (int j = 0; j < k; ++j) counts[j] += pc[t][j];
    total += costs[t];
  }
  if (cost) *cost += total;
  if (rescored)
    for (size_t t = 0; t < th.size(); ++t) *rescored += res[t];
  return 0;
}

extern "C" int hbmr_kmeans_map_cpu_f32(const float* X, long n, int d, const float* C, int k,
                                       int32_t* labels, long long* sums, long long* counts,
                                       double* cost, int fx_shift, int nthreads) {
  return hbmr_kmeans_map_cpu_f32_ex(X, n, d, C, k, labels, sums, counts, cost, fx_shift, nthreads,
                                    0, nullptr);
}
