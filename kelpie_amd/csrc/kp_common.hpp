// kp_common.hpp -- shared host/device helpers of the Kelpie HIP library (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kelpie_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define KP_WAVE 64

// ----------------------------------------------------------------------------
// error plumbing
// ----------------------------------------------------------------------------
struct KpError {
  int code;
  std::string msg;
};

#define KP_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess)                                                         \
      throw KpError{KP_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
  } while (0)

#define KP_REQUIRE(cond, msg)                         \
  do {                                                \
    if (!(cond)) throw KpError{KP_EINVAL, (msg)};     \
  } while (0)

// grow-only device buffer.  A buffer bound to its context's stream (`s`, set by
// kp_ctx_create for the context's own workspaces) grows stream-ordered: the new
// allocation comes from the device's default memory pool (hipMallocAsync) and the old one
// goes back to it (hipFreeAsync) once the stream reaches the free -- no device-wide
// synchronisation (hipFree waits for the whole device, every context's queued work
// included, which stalled the batch thread that grew the buffer behind the other batches
// in flight), and no superseded allocation is kept.  An unbound buffer (call-local
// scratch) keeps its superseded allocations until release().
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipStream_t s = nullptr;
  hipMemPool_t pool = nullptr;  // the library's own pool of the device (kp_device_pool)
  std::vector<void*> old;
  void* ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
      const size_t want = bytes + bytes / 4;
      void* q = nullptr;
      if (s) {
        if (pool)
          KP_HIP(hipMallocFromPoolAsync(&q, want, pool, s));
        else
          KP_HIP(hipMallocAsync(&q, want, s));
        if (p) KP_HIP(hipFreeAsync(p, s));
      } else {
        KP_HIP(hipMalloc(&q, want));
        if (p) old.push_back(p);
      }
      p = q;
      cap = want;
    }
    return p;
  }
  template <class T>
  T* as() { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) (void)(s ? hipFreeAsync(p, s) : hipFree(p));
    for (void* q : old) (void)hipFree(q);
    old.clear();
    p = nullptr;
    cap = 0;
  }
};

struct Timing {
  double device_s = 0.0;  // whole call on the device (first upload .. last kernel)
  double loop_s = 0.0;    // post-training loop
  double hot_s = 0.0;     // sum of the dominant kernel's launch durations
  int64_t hot_launches = 0;
  double hot_work = 0.0;  // work units of the dominant kernel (see kp_last_timing)
};

struct kp_train_state;  // kp_train.hip: optimizer state of a full-model training run
struct kp_cv_train;     // kp_train_conve.hip: ConvE full-model training state

struct kp_ctx {
  int device = 0;
  int n_cu = 256;  // compute units of the device (one attention workgroup per CU)
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int model = 0;
  int n_ent = 0, n_rel2 = 0, dim = 0, dp = 0;  // dp: padded row stride (multiple of 16)
  int hidden = 0;                              // ConvE
  float* dE = nullptr;                         // [n_ent][dp] zero-padded
  float* dR = nullptr;                         // [n_rel2][dp]
  float* dEt = nullptr;                        // TransE: ||E_e||^2 etc (unused for others)
  // ConvE frozen layers
  float* d_conv_w = nullptr;
  float* d_conv_b = nullptr;
  float* d_fc_w = nullptr;   // [dim][hidden]
  float* d_fc_b = nullptr;
  float* d_bn_a = nullptr;
  float* d_bn_b = nullptr;
  std::vector<float> hE;     // host copy (ConvE/TransE helpers)
  DevBuf ws[32];             // workspace slots (see each model file)
  std::string err;
  Timing timing;
  bool time_hot = true;
  // attention contraction: 0 = fp32 MFMA (kp_attn.hpp), 1 = bf16x3 MFMA (kp_attn3.hpp)
  int attn_mode = 0;
  int attn_part = 0;  // kp_attn3 partition: 0 chosen per launch, 1 stream-K, 2 XCD-grouped ranges (KP_ATTN_PART)
  DevBuf e3;               // kp_attn3's split image of dE, built on first use
  bool e3_ready = false;
  DevBuf e3ts, e3pre;      // kp_attn3's fp64 tile sums / prefix sums of dE over tiles
  bool e3pre_ready = false;
  DevBuf eT;               // dE transposed [dp][round_up(n_ent, 256)] fp32 (fp64 rank scoring), on first use
  bool eT_ready = false;
  int cv_fused = 1;        // ConvE d = 200: fused encoder kernels (kp_cv_fused.hpp), KP_CV_FUSED
  int cv_rank64 = 1;       // ConvE post-training rank on fp64 logits (KP_CV_RANK=f32: fp32 sigmoid scores)
  int cv_dx_block = 0;     // ConvE: the 256-thread kp_cv_dx instead of kp_cv_dx1 (KP_CV_DX=block, A/B)
  int te_norm = 2;         // TransE score norm p (kp_model_desc.norm_p): 2 or 1
  int te_rank64 = 1;       // TransE post-training rank on fp64 squared distances (KP_TE_RANK=f32: fp32 norms)
  DevBuf cvf_fw3, cvf_bw3;  // their permuted split images of the FC weight (built once)
  bool cvf_ready = false;
  int cv_shared = 1;        // ConvE fused path: the shared-encoder split (kp_cv_fused.hpp), KP_CV_SHARED
  DevBuf cv_wtm, cv_trel;   // its map-row-18-19 FC columns and the relations' FC terms (built once)
  DevBuf cv_wtl, cv_wfm;    // the kelpie rows' FC columns and the mid columns, transposed (built once)
  DevBuf cv_wlc;            // the kelpie rows' FC columns [dim][4608] (built once)
  bool cv_shared_ready = false;
  DevBuf cvs[14];           // per-batch ConvE workspaces (kp_conve.hip)
  int attn3_wpc[2] = {0, 0};  // co-resident kp_attn3 workgroups per CU, [softmax, BCE] (occupancy API)
  kp_train_state* train = nullptr;  // kp_train_epoch's state (freed with the context)
  kp_cv_train* cvtrain = nullptr;   // kp_conve_train_*'s state (freed with the context)
  std::vector<hipEvent_t> evpool;
  std::vector<std::pair<double, double>> hot_pairs;  // (work units, seconds) per hot launch
  std::vector<double> hot_iv;  // [start, end] per hot launch, seconds since the device's time base
  // the workspaces that live on the context's stream (DevBuf::s)
  std::vector<DevBuf*> bound_buffers() {
    std::vector<DevBuf*> v = {&e3, &e3ts, &e3pre, &eT, &cvf_fw3, &cvf_bw3,
                              &cv_wtm, &cv_trel, &cv_wtl, &cv_wfm, &cv_wlc};
    for (auto& b : ws) v.push_back(&b);
    for (auto& b : cvs) v.push_back(&b);
    return v;
  }
  hipEvent_t event(size_t i) {
    while (evpool.size() <= i) {
      hipEvent_t e;
      KP_HIP(hipEventCreate(&e));
      evpool.push_back(e);
    }
    return evpool[i];
  }
};


static inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// upload helper
template <class T>
static inline T* upload(kp_ctx* c, DevBuf& b, const T* src, size_t n) {
  T* d = reinterpret_cast<T*>(b.ensure(n * sizeof(T)));
  if (n) KP_HIP(hipMemcpyAsync(d, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return d;
}

// ----------------------------------------------------------------------------
// device helpers
// ----------------------------------------------------------------------------
// Sum over each 16-lane row with DPP (VALU lane moves, no LDS round trip):
// xor 1, xor 2 (quad_perm), half-mirror (quads of 8), mirror (halves of 16).
// Every lane of the row ends with the same bits (each step adds a symmetric pair).
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ----------------------------------------------------------------------------
// entry points implemented per model family
// ----------------------------------------------------------------------------
void complex_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* b);
void complex_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out);
// scores of n (head, rel) pairs over the frozen entities into a device buffer [n][ld]
void complex_scores_dev(kp_ctx* c, int n, const int32_t* d_heads, const int32_t* d_rels, float* d_out, int ld);
void transe_scores_dev(kp_ctx* c, int n, const int32_t* d_heads, const int32_t* d_rels, float* d_out, int ld);
void conve_scores_dev(kp_ctx* c, int n, const int32_t* d_heads, const int32_t* d_rels, float* d_out, int ld);
void launch_convertible_reduce(kp_ctx* c, int n, const float* d_scores, int ld, int obj, const int32_t* d_fo,
                               const int32_t* d_f, int minimizer, uint8_t* d_keep);
void transe_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* b);
void transe_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out);
void conve_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* b);
void conve_all_scores(kp_ctx* c, int n, const int32_t* heads, const int32_t* rels, float* out);
// ConvE encoder output (eval mode) of n (lhs, rel) pairs -> [n][dp] (criage_first_step, conve.py:102-124)
void conve_encode_dev(kp_ctx* c, int n, const int2* d_src, float* d_out);
// baseline engines (kp_baselines.hip)
void dp_relevance(kp_ctx* c, int n, const int32_t* items, float eps, float lambd, int step_sign, int rel_sign,
                  float* out);
void criage_relevance(kp_ctx* c, int n, const int32_t* items, int n_ents, const int32_t* ent_ids,
                      const int32_t* tails_off, const int32_t* tails, double* out, int32_t* status);

// shared rank kernel launcher (kp_rank.hip): scores [n][ld] already on device,
// column `kcol` = kelpie score (or -1 when absent)
void launch_score_gemm(kp_ctx* c, const float* dQ, int nq, float* d_out, int ld, int act);
// kp_train.hip: one MultiClassNLLOptimizer epoch on the context's tables (ComplEx)
void complex_train_epoch(kp_ctx* c, const kp_hp* hp, int n, const int32_t* triples, const int32_t* perm, int epoch);
// kp_train.hip: one PairwiseRankingOptimizer epoch (TransE): positive and corrupted rows in order
void transe_train_epoch(kp_ctx* c, const kp_hp* hp, int n, const int32_t* pos, const int32_t* neg, int epoch);
void train_state_free(kp_ctx* c);
// kp_train_conve.hip: ConvE BCEOptimizer training (see include/kelpie_hip.h kp_conve_train_*)
void cv_train_free(kp_ctx* c);
void conve_train_begin(kp_ctx* c, const float* bn_w, const float* bn_b, const float* bn_m, const float* bn_v);
void conve_train_step(kp_ctx* c, int B, const int32_t* pairs, const int32_t* tail_off, const int32_t* tails,
                      const float* in_noise, const float* fm_noise, const float* hid_noise, float lr,
                      float label_smoothing, int bn_train);
void conve_train_read(kp_ctx* c, float* conv_w, float* conv_b, float* fc_w, float* fc_b, float* bn_w, float* bn_b,
                      float* bn_m, float* bn_v);
// out[z][m][n] = act(sum_{k in split z} A[m][k] B[n][k] + (z == 0 ? bias[n] : 0)), fp32 MFMA
void launch_gemm_abt(kp_ctx* c, const float* A, int lda, int M, const float* B, int ldb, int N, int K, float* out,
                     int ldo, const float* bias, int act, int ksplit);
enum { RANK_TRIPLE_RESULTS = 0, RANK_PREDICT_TAILS = 1, RANK_SORT_POSITION = 2 };
// get_triple_results of a maximizer in fp64 (kp_rank.hip): q64 [n][dp] the ranking queries,
// t64 [n] their target scores (q . E_o, or the kelpie column when o is the kelpie),
// kcol64 [n] the kelpie column scores q . x; rank = #{e not filtered : score_e >= target}
// over the frozen entities (scores q . E_e summed in fp64, sequentially over d) plus the
// kelpie column.  The target itself counts unless filtered.
// launch_rank_f64's score kinds
enum { RANK64_DOT = 0, RANK64_SIGMOID = 1, RANK64_DIST = 2, RANK64_DIST1 = 3 };
void launch_rank_f64(kp_ctx* c, int n_slots, const double* d_q64, const double* d_t64, const double* d_kcol64,
                     const int32_t* d_pred_o, const int32_t* d_filt_off, const int32_t* d_filt, float* d_target,
                     int64_t* d_rank, int act = 0);
void launch_rank_count(kp_ctx* c, int n_slots, const float* d_scores, int ld, int n_cols,
                       const int32_t* d_pred_o, const int32_t* d_filt_off, const int32_t* d_filt,
                       int minimizer, float* d_target, int64_t* d_rank,
                       int mode = 0);

// Per-device time base: one event recorded (and completed) when the device's first
// context is created.  Hot-launch intervals of every context on the device are taken
// against it, so launches of contexts that run at once can be merged on one axis
// (kp_hot_intervals).
inline hipEvent_t kp_time_base(int device, hipStream_t stream) {
  static std::mutex mu;
  static hipEvent_t base[64] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (device < 0 || device >= 64) return nullptr;
  if (!base[device]) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    if (hipEventRecord(e, stream) != hipSuccess || hipEventSynchronize(e) != hipSuccess) {
      (void)hipEventDestroy(e);
      return nullptr;
    }
    base[device] = e;
  }
  return base[device];
}

// append the [start, end] of one timed launch (events a -> b) to c->hot_iv
inline void kp_push_interval(kp_ctx* c, hipEvent_t a, hipEvent_t b) {
  const hipEvent_t t0 = kp_time_base(c->device, c->stream);
  float ms_a = 0.f, ms_b = 0.f;
  if (!t0 || hipEventElapsedTime(&ms_a, t0, a) != hipSuccess || hipEventElapsedTime(&ms_b, t0, b) != hipSuccess)
    return;
  c->hot_iv.push_back(ms_a * 1e-3);
  c->hot_iv.push_back(ms_b * 1e-3);
}
