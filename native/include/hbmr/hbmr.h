// hbmr native C API (libhbmr.so).
//
// GPU entry points take raw device pointers and the hipStream_t to launch on;
// they return 0 on success or a hipError_t code.  CPU entry points return 0 on
// success or a negative errno-style code.  The Python runtime binds these with
// ctypes (hbmr/ops/_lib.py); the Pipes GPU task binaries link the same objects.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hbmr_stream_t;

// ---- K-Means (native/kernels/kmeans.hip) -----------------------------------
#ifndef HBMR_NO_HIP_DECLS
#include <hip/hip_runtime_api.h>
int hbmr_kmeans_assign_bf16(const void* X, long n, int dp, const void* C, const float* chalf,
                            int k_pad, int32_t* labels, float* scores, hipStream_t st);
// sums/counts are 64-bit fixed point: sum = Σ round(x · 2^fx_shift)
// mode 0 = auto, 1 = LDS-privatised, 2 = counting-sort + segmented sum (needs workspace)
int hbmr_kmeans_accum_bf16(const void* X, long n, int dp, const int32_t* labels, int k,
                           long long* sums, long long* counts, int fx_shift, void* ws,
                           long ws_bytes, int mode, hipStream_t st);
// Exact mode (hbmr.kmeans.exact): fp32-data combiner, top-2 assign, fp64 re-score
int hbmr_kmeans_accum_f32(const float* X, long n, int dp, const int32_t* labels, int k,
                          long long* sums, long long* counts, int fx_shift, void* ws,
                          long ws_bytes, int mode, hipStream_t st);
// cand: [2n] runner-ups (second | third), margin: [2n] best-second | best-third
int hbmr_kmeans_assign_top3_bf16(const void* X, long n, int dp, const void* C, const float* chalf,
                                 int k_pad, int32_t* labels, int32_t* cand, float* scores,
                                 float* margin, hipStream_t st);
int hbmr_kmeans_assign_top3_f16(const void* X, long n, int dp, const void* C, const float* chalf,
                                int k_pad, int32_t* labels, int32_t* cand, float* scores,
                                float* margin, hipStream_t st);
// exact-mode staging: 16-bit MFMA copy (f16 = 1: fp16, else bf16) + |x|, |x~|^2, |x - x~|
int hbmr_kmeans_exact_prep(const float* x, long n, int d, int ldx, int dp, int f16, void* x16,
                           float* xnorm, float* xn2, float* xerr, hipStream_t st);
// 16-bit centroid image + chalf, |c|, |c - c~|, maxima[2]
// exact mode's centroid neighbour table: di/dv [k, L] (the L nearest by a
// lower bound rounded down, ascending, itself first), pd [k, k] upper bounds
// rounded up (may be null); k <= 8192, d <= 256
int hbmr_kmeans_centroid_nbr(const float* cen, int k, int d, int L, int32_t* di, float* dv,
                             float* pd, hipStream_t st);
int hbmr_kmeans_image16(const float* cen, int k, int d, int dp, int k_pad, int f16, void* c16,
                        float* chalf, float* cnorm, float* cerr, float* maxima, hipStream_t st);
// tiled (piece-major per 32-row tile) copy of a 16-bit image for the v3 assign
int hbmr_kmeans_image16_tiled(const void* c16, int k_pad, int dp, void* c16t, hipStream_t st);
int hbmr_kmeans_set_stamps(void* p);
int hbmr_kmeans_refine_f32(const float* X32, long n, int d, int ldx, const float* xnorm,
                           const float* xbn2, const float* xerr, const float* C32, int k,
                           int k_pad, const float* cnorm, const float* cmax, const float* cerr,
                           const float* cerrmax, const int32_t* nbr_idx,
                           const float* nbr_dist, int L, int32_t* labels, const int32_t* cand,
                           const float* scores, const float* margin, unsigned long long* stats,
                           int nstats, hipStream_t st);
int hbmr_kmeans_assign_top3_q1_grouped(int nsplit, const void* const* X, const long* n, int dp,
                                       int f16, const void* C, const void* Ct,
                                       const float* chalf, int k_pad,
                                       int32_t* labels, const float* const* xnorm,
                                       const float* const* xbn2, const float* const* xerr,
                                       int d, int k, const float* cnorm, const float* cmax,
                                       const float* cerr, const float* cerrmax, void* ws,
                                       long ws_bytes, const float* dcc, hipStream_t st);
int hbmr_kmeans_assign_top3_grouped(int nsplit, const void* const* X, const long* n, int dp,
                                    int f16, const void* C, const float* chalf, int k_pad,
                                    int32_t* labels, int32_t* cand, float* scores, float* margin,
                                    hipStream_t st);
int hbmr_kmeans_refine_batch_q1g(int nsplit, const long* ns, int d, int k, int k_pad,
                                 const float* const* xnorm, const float* const* xbn2,
                                 const float* const* xerr, const float* cnorm, const float* cmax,
                                 const float* cerr, const float* cerrmax, const int32_t* labels,
                                 const int32_t* cand, const float* scores, const float* margin,
                                 void* ws, long ws_bytes, const float* dcc, hipStream_t st);
// refine v3 over a batch of splits (see kmeans.hip): q1 per split, finish once
long hbmr_kmeans_refine_batch_bytes(int nsplit, const long* ns);
int hbmr_kmeans_refine_batch_q1(int nsplit, const long* ns, int s, int d, int k, int k_pad,
                                const float* xnorm, const float* xbn2, const float* xerr,
                                const float* cnorm, const float* cmax, const float* cerr,
                                const float* cerrmax, const int32_t* labels, const int32_t* cand,
                                const float* scores, const float* margin,
                                unsigned long long* stats, void* ws, long ws_bytes, int reset,
                                const float* dcc, hipStream_t st);
int hbmr_kmeans_refine_batch_finish(int nsplit, const long* ns, const float* const* x32,
                                    int32_t* const* labels, int d, int ldx, const float* C32,
                                    int k, int k_pad, const float* cmax, const float* cerrmax,
                                    const int32_t* nbr_idx, const float* nbr_dist, int L,
                                    unsigned long long* stats, int nstats, void* ws,
                                    long ws_bytes, hipStream_t st);
int hbmr_kmeans_update(const long long* sums, const long long* counts, int fx_shift, int k, int d,
                       int dp, int k_pad, float* cen, void* cbf, float* chalf, float* shift2,
                       hipStream_t st);
// a batch of map tasks (one per split): assign + combine into sums[t] / counts[t]
int hbmr_kmeans_map_batch(int ntasks, const void* const* X, const long* n, int dp,
                          const void* C, const float* chalf, int k_pad, int k, int32_t* labels,
                          void* ws, long ws_bytes, long long* sums, long long* counts,
                          int fx_shift, int zero_outputs, hipStream_t st);
// fp32 [n, d] row-major → bf16 [n, dp] (round-to-nearest-even, columns d..dp zero)
int hbmr_f32_to_bf16_pad(const float* src, long n, int d, int dp, void* dst, hipStream_t st);
#endif
int hbmr_kmeans_padded_dim(int d);

// ---- sort / shuffle (native/kernels/sort.hip) ----------------------------------
#ifndef HBMR_NO_HIP_DECLS
// LSD radix sort of (uint64 key, uint32 value) by key bits [begin_bit, end_bit),
// stable; keys/vals in and out, tkeys/tvals scratch of the same size.
int hbmr_radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t* tkeys, uint32_t* tvals,
                              long n, int begin_bit, int end_bit, void* ws, long ws_bytes,
                              hipStream_t st);
// Hadoop TeraGen records [first_row, first_row + nrows) (100 B each)
int hbmr_teragen(long first_row, long nrows, void* out, hipStream_t st);
int hbmr_tera_keys(const void* records, long n, int stride, uint64_t* hi, uint64_t* lo,
                   hipStream_t st);
int hbmr_gather_u64(const uint64_t* src, const uint32_t* perm, long n, uint64_t* dst,
                    hipStream_t st);
int hbmr_gather_records(const void* src, const uint32_t* perm, long n, int record_bytes, void* dst,
                        hipStream_t st);
int hbmr_split_offsets(const uint64_t* hi, const uint64_t* lo, long n, const uint64_t* shi,
                       const uint64_t* slo, int nparts, long* offsets, hipStream_t st);
int hbmr_check_sorted(const uint64_t* hi, const uint64_t* lo, long n, unsigned long long* bad,
                      hipStream_t st);
int hbmr_tera_keys_part(const void* records, long n, int stride, const uint64_t* shi,
                        const uint64_t* slo, int nsplit, uint64_t* hi, uint64_t* lo,
                        uint64_t* pid, hipStream_t st);
int hbmr_tera_collect(const uint64_t* const* his, const uint64_t* const* los,
                      const uint32_t* const* rows, const long* starts, const long* prefix, int S,
                      long n, uint64_t* ohi, uint64_t* olo, uint32_t* osplit, uint32_t* orow,
                      hipStream_t st);
// static-shape shuffle slots: W x C (split, row) entries from device offsets
// (split 0xFFFFFFFF past a slot's count; hbmr_gather_records_multi skips those)
int hbmr_tera_collect_slots(const uint32_t* const* rows, const long* starts, const long* pre,
                            int S, int W, long C, uint32_t* osplit, uint32_t* orow,
                            hipStream_t st);
int hbmr_gather_records_multi(const void* const* bases, const uint32_t* split, const uint32_t* row,
                              const uint32_t* perm, long n, int record_bytes, void* dst,
                              hipStream_t st);
int hbmr_tera_collect_gid(const uint64_t* const* his, const uint32_t* const* rows,
                          const long* starts, const long* prefix, int S, long n, int pack,
                          uint64_t vlo, unsigned int m, unsigned int R, int sh, uint64_t* ohi,
                          uint32_t* ogid, hipStream_t st);
int hbmr_gather_records_gid(const void* const* bases, const uint32_t* gid, const uint64_t* packed,
                            long n, int record_bytes, void* dst, uint64_t* hi, uint64_t* lo,
                            uint32_t* win, hipStream_t st);
long hbmr_radix_onesweep_workspace_bytes(long n);
long hbmr_radix_onesweep_status_bytes(long n);
int hbmr_radix_sort_keys_u64(uint64_t* keys, uint64_t* tkeys, long n, int begin_bit, int end_bit,
                             void* ws, long ws_bytes, void* status, long status_bytes,
                             unsigned int* epoch, uint32_t* err, int copy_back, hipStream_t st);
long hbmr_tera_tie_fix_scratch_bytes(long cap, int record_bytes);
int hbmr_tera_group_stats(const uint64_t* hi, const uint64_t* lo, long n, const uint64_t* ph,
                          const uint64_t* pl, unsigned long long* acc, hipStream_t st);
int hbmr_tera_tie_fix_records(uint64_t* hi, uint64_t* lo, void* rec, long n, int record_bytes,
                              uint64_t vlo, unsigned int m, unsigned int R, int sh,
                              const uint32_t* win, unsigned int* flag, void* scratch, long cap,
                              hipStream_t st);
int hbmr_merge_path(const uint64_t* ahi, const uint64_t* alo, const uint32_t* av, long na,
                    const uint64_t* bhi, const uint64_t* blo, const uint32_t* bv, long nb,
                    uint64_t* ohi, uint64_t* olo, uint32_t* ov, hipStream_t st);
int hbmr_tera_tie_fix(const uint64_t* hi, uint64_t* lo, uint32_t* perm, long n,
                      unsigned int* flag, hipStream_t st);
int hbmr_tera_partition(const void* records, long n, int stride, const uint64_t* shi,
                        const uint64_t* slo, int nsplit, uint64_t* ohi, uint64_t* olo,
                        uint32_t* orow, long* offsets, unsigned long long* kmm, void* ws,
                        long ws_bytes, hipStream_t st);
#endif
long hbmr_radix_sort_workspace_bytes(long n);
long hbmr_tera_partition_workspace_bytes(long n, int nparts);

// ---- GEMM (native/kernels/gemm.hip) -------------------------------------------
#ifndef HBMR_NO_HIP_DECLS
// C[M,N] = alpha · A[M,K] · Bt[N,K]ᵀ (bf16 in, fp32 accumulate; C fp32 or bf16).
// M, N multiples of 256, K of 64.
int hbmr_gemm_bf16_tn(const void* A, const void* Bt, void* C, long M, long N, long K, float alpha,
                      int out_bf16, hipStream_t st);
// ... plus partials[(M/256)·(N/256)] = fp64 sum of each 256×256 tile of C (null: none)
int hbmr_gemm_bf16_tn_ex(const void* A, const void* Bt, void* C, long M, long N, long K,
                         float alpha, int out_bf16, double* partials, hipStream_t st);
#endif
// ---- text / WordCount (native/kernels/text.hip) ---------------------------------
#ifndef HBMR_NO_HIP_DECLS
long hbmr_wc_tiles(long n);
int hbmr_wc_tokenize_count(const uint8_t* buf, long n, uint32_t* tile_counts, hipStream_t st);
int hbmr_wc_tokenize_write(const uint8_t* buf, long n, const long* tile_base, uint32_t* starts,
                           uint32_t* lens, hipStream_t st);
int hbmr_wc_insert(const uint8_t* buf, long n, const uint32_t* starts, const uint32_t* lens,
                   const int64_t* weights, long nwords, uint64_t* tkeys, uint64_t* tcounts,
                   long cap, int* overflow, hipStream_t st);
int hbmr_wc_compact(const uint8_t* buf, long n, const uint64_t* tkeys, const uint64_t* tcounts,
                    long cap, int R, uint32_t* ustart, uint32_t* ulen, int64_t* ucount,
                    int32_t* upart, unsigned int* counter, hipStream_t st);
int hbmr_wc_pack(const uint8_t* buf, const uint32_t* ustart, const uint32_t* ulen,
                 const int64_t* order, long nu, const int64_t* out_off, uint8_t* out,
                 hipStream_t st);
#endif
int hbmr_kmeans_padded_k(int k);
long hbmr_kmeans_accum_workspace_bytes(long n, int k);
long hbmr_kmeans_batch_workspace_bytes(long total_n, int ntasks, int k);

// ---- CPU kernels (native/cpu) ------------------------------------------------
int hbmr_kmeans_map_cpu_f32(const float* X, long n, int d, const float* C, int k,
                            int32_t* labels, long long* sums, long long* counts, double* cost,
                            int fx_shift, int nthreads);
int hbmr_kmeans_map_cpu_f32_ex(const float* X, long n, int d, const float* C, int k,
                               int32_t* labels, long long* sums, long long* counts, double* cost,
                               int fx_shift, int nthreads, int exact, long* rescored);

#ifdef __cplusplus
}
#endif
