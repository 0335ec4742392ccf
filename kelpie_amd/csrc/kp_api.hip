// kp_api.hip -- C ABI entry points of libkelpie_hip.so (include/kelpie_hip.h).
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "kp_common.hpp"

int cx_pick_db(int dim);

static thread_local std::string g_tls_err;

template <class F>
static int guarded(kp_ctx* c, F&& f) {
  try {
    f();
    if (c) c->err.clear();
    return KP_OK;
  } catch (const KpError& e) {
    if (c) c->err = e.msg;
    g_tls_err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    if (c) c->err = "host out of memory";
    g_tls_err = "host out of memory";
    return KP_ENOMEM;
  } catch (...) {
    if (c) c->err = "unknown error";
    g_tls_err = "unknown error";
    return KP_EINVAL;
  }
}

static void upload_padded(kp_ctx* c, float** dst, const float* src, int rows, int dim, int dp) {
  std::vector<float> tmp((size_t)rows * dp, 0.f);
  for (int r = 0; r < rows; ++r) std::memcpy(&tmp[(size_t)r * dp], src + (size_t)r * dim, sizeof(float) * dim);
  KP_HIP(hipMalloc(dst, sizeof(float) * tmp.size() + 64));
  KP_HIP(hipMemcpy(*dst, tmp.data(), sizeof(float) * tmp.size(), hipMemcpyHostToDevice));
}

// One private stream-ordered pool per device for the contexts' workspaces, created on
// first use and kept for the process (never destroyed: contexts on several threads share
// it).  Its release threshold is unbounded, so freed workspace stays with the pool.
static hipMemPool_t device_pool(int device) {
  static std::mutex mu;
  static std::vector<hipMemPool_t> pools;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)pools.size() <= device) pools.resize(device + 1, nullptr);
  if (!pools[device]) {
    hipMemPoolProps props;
    std::memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    hipMemPool_t pool = nullptr;
    KP_HIP(hipMemPoolCreate(&pool, &props));
    uint64_t keep = UINT64_MAX;
    KP_HIP(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
    pools[device] = pool;
  }
  return pools[device];
}

static void upload_plain(float** dst, const float* src, size_t n) {
  KP_HIP(hipMalloc(dst, sizeof(float) * n + 64));
  KP_HIP(hipMemcpy(*dst, src, sizeof(float) * n, hipMemcpyHostToDevice));
}

extern "C" {

const char* kp_version(void) { return "kelpie_hip 0.1 (gfx950)"; }

const char* kp_last_error(const kp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_tls_err.c_str(); }

int kp_host_alloc(size_t bytes, void** out) {
  if (!out) return KP_EINVAL;
  *out = nullptr;
  return guarded(nullptr, [&] {
    KP_REQUIRE(bytes > 0, "kp_host_alloc: zero bytes");
    void* p = nullptr;
    KP_HIP(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    *out = p;
  });
}

int kp_host_free(void* p) {
  return guarded(nullptr, [&] {
    if (p) KP_HIP(hipHostFree(p));
  });
}

int kp_ctx_create(int device, const kp_model_desc* m, kp_ctx** out) {
  if (!out || !m) return KP_EINVAL;
  *out = nullptr;
  kp_ctx* c = new kp_ctx();
  int rc = guarded(nullptr, [&] {
    KP_REQUIRE(m->n_ent > 0 && m->n_rel2 > 0 && m->dim > 0, "kp_ctx_create: empty model");
    KP_REQUIRE(m->entity && m->relation, "kp_ctx_create: missing tables");
    KP_REQUIRE(m->model >= KP_MODEL_TRANSE && m->model <= KP_MODEL_CONVE, "kp_ctx_create: unknown model");
    c->device = device;
    c->model = m->model;
    c->n_ent = m->n_ent;
    c->n_rel2 = m->n_rel2;
    c->dim = m->dim;
    KP_REQUIRE(m->norm_p == 0 || (m->model == KP_MODEL_TRANSE && (m->norm_p == 1 || m->norm_p == 2)),
               "kp_ctx_create: norm_p must be 1 or 2 (TransE) or 0");
    c->te_norm = m->norm_p == 1 ? 1 : 2;
    KP_HIP(hipSetDevice(device));
    KP_HIP(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    (void)kp_time_base(device, nullptr);
    if (m->model == KP_MODEL_COMPLEX || m->model == KP_MODEL_CONVE) {
      KP_REQUIRE(m->model != KP_MODEL_COMPLEX || m->dim % 2 == 0, "ComplEx: row width must be even ([Re | Im])");
      int db = cx_pick_db(m->dim);
      KP_REQUIRE(db > 0, "row width > 400 not supported yet for ComplEx / ConvE");
      c->dp = 16 * db;
    } else {
      c->dp = round_up(m->dim, 16);
    }
    // attention contraction (kp_attn3.hpp): bf16x3 MFMA by default, KP_ATTN=f32 selects
    // the fp32-MFMA kernel of kp_attn.hpp
    c->attn_mode = 1;
    if (const char* a = std::getenv("KP_ATTN")) c->attn_mode = std::strcmp(a, "f32") == 0 ? 0 : 1;
    // ConvE d = 200: fused conv + FC forward and FC^T + transposed-conv backward
    // (kp_cv_fused.hpp) by default; KP_CV_FUSED=0 selects the separate kernels (A/B)
    c->cv_fused = 1;
    if (const char* a = std::getenv("KP_CV_FUSED")) c->cv_fused = std::atoi(a) != 0;
    // on the fused path without input / feature-map dropout: the encoder split into kelpie
    // row, pair and relation terms (kp_cv_fused.hpp); KP_CV_SHARED=0 runs the whole map per pair
    c->cv_shared = 1;
    if (const char* a = std::getenv("KP_CV_SHARED")) c->cv_shared = std::atoi(a) != 0;
    // ConvE rank of the post-trained row on fp64 logits (sigmoid is monotone), as a fp64
    // reference ranks; KP_CV_RANK=f32 ranks the fp32 sigmoid scores (A/B)
    if (const char* a = std::getenv("KP_CV_RANK")) c->cv_rank64 = std::strcmp(a, "f32") != 0;
    // ConvE dL/dfc: one wave per pair (kp_cv_dx1, no LDS: co-resident with the attention) by
    // default; KP_CV_DX=block selects the 256-thread form (A/B; bitwise the same)
    if (const char* a = std::getenv("KP_CV_DX")) c->cv_dx_block = std::strcmp(a, "block") == 0;
    // TransE rank of the post-trained row on fp64 squared distances (sqrt is monotone);
    // KP_TE_RANK=f32 ranks the fp32 norms (A/B)
    if (const char* a = std::getenv("KP_TE_RANK")) c->te_rank64 = std::strcmp(a, "f32") != 0;
    if (const char* a = std::getenv("KP_ATTN_PART"))
      c->attn_part = std::strcmp(a, "streamk") == 0 ? 1 : std::strcmp(a, "ranges") == 0 ? 2 : 0;
    KP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // the context's own workspaces grow stream-ordered on its stream (DevBuf), from the
    // library's private pool of the device, which keeps what they give back instead of
    // returning it to the driver; the device's default pool (torch, RCCL) is left alone
    {
      hipMemPool_t pool = device_pool(device);
      for (DevBuf* d : c->bound_buffers()) {
        d->s = c->stream;
        d->pool = pool;
      }
    }
    KP_HIP(hipEventCreate(&c->ev0));
    KP_HIP(hipEventCreate(&c->ev1));
    upload_padded(c, &c->dE, m->entity, m->n_ent, m->dim, c->dp);
    upload_padded(c, &c->dR, m->relation, m->n_rel2, m->dim, c->dp);
    if (m->model == KP_MODEL_CONVE) {
      KP_REQUIRE(m->conv_w && m->conv_b && m->fc_w && m->fc_b && m->bn_alpha && m->bn_beta,
                 "ConvE: missing frozen layers");
      KP_REQUIRE(m->dim % 20 == 0 && m->dim / 20 >= 3, "ConvE: dim must be 20*h with h >= 3");
      c->hidden = 32 * 38 * (m->dim / 20 - 2);
      upload_plain(&c->d_conv_w, m->conv_w, 32 * 9);
      upload_plain(&c->d_conv_b, m->conv_b, 32);
      upload_plain(&c->d_fc_w, m->fc_w, (size_t)m->dim * c->hidden);
      upload_plain(&c->d_fc_b, m->fc_b, m->dim);
      upload_plain(&c->d_bn_a, m->bn_alpha, 1 + 32 + m->dim);
      upload_plain(&c->d_bn_b, m->bn_beta, 1 + 32 + m->dim);
    }
  });
  if (rc != KP_OK) {
    kp_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return KP_OK;
}

int kp_ctx_destroy(kp_ctx* c) {
  if (!c) return KP_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (float* p : {c->dE, c->dR, c->dEt, c->d_conv_w, c->d_conv_b, c->d_fc_w, c->d_fc_b, c->d_bn_a, c->d_bn_b})
    if (p) (void)hipFree(p);
  for (auto& b : c->ws) b.release();
  c->e3.release();
  c->e3ts.release();
  c->e3pre.release();
  c->eT.release();
  c->cvf_fw3.release();
  c->cvf_bw3.release();
  for (DevBuf* b : {&c->cv_wtm, &c->cv_trel, &c->cv_wtl, &c->cv_wfm, &c->cv_wlc}) b->release();
  for (auto& b : c->cvs) b.release();
  if (c->stream) (void)hipStreamSynchronize(c->stream);  // the stream-ordered frees above
  train_state_free(c);
  cv_train_free(c);
  for (auto e : c->evpool) (void)hipEventDestroy(e);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return KP_OK;
}

int kp_posttrain_rank(kp_ctx* c, const kp_hp* hp, const kp_batch* b) {
  if (!c || !hp || !b) return KP_EINVAL;
  return guarded(c, [&] {
    KP_REQUIRE(b->n_slots >= 0, "kp_posttrain_rank: negative n_slots");
    if (b->n_slots == 0) return;
    KP_REQUIRE(b->x0 && b->row_off && b->pred && b->filt_off && b->out_score && b->out_rank,
               "kp_posttrain_rank: missing buffer");
    KP_HIP(hipSetDevice(c->device));
    switch (c->model) {
      case KP_MODEL_COMPLEX: complex_posttrain_rank(c, hp, b); break;
      case KP_MODEL_TRANSE: transe_posttrain_rank(c, hp, b); break;
      case KP_MODEL_CONVE: conve_posttrain_rank(c, hp, b); break;
    }
  });
}

int kp_all_scores(kp_ctx* c, int32_t n, const int32_t* heads, const int32_t* rels, float* out) {
  if (!c || n < 0 || (n > 0 && (!heads || !rels || !out))) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    for (int i = 0; i < n; ++i) {
      KP_REQUIRE(heads[i] >= 0 && heads[i] < c->n_ent, "kp_all_scores: head out of range");
      KP_REQUIRE(rels[i] >= 0 && rels[i] < c->n_rel2, "kp_all_scores: relation out of range");
    }
    switch (c->model) {
      case KP_MODEL_COMPLEX: complex_all_scores(c, n, heads, rels, out); break;
      case KP_MODEL_TRANSE: transe_all_scores(c, n, heads, rels, out); break;
      case KP_MODEL_CONVE: conve_all_scores(c, n, heads, rels, out); break;
    }
  });
}

int kp_convertible(kp_ctx* c, int32_t n, const int32_t* heads, int32_t rel, int32_t obj, const int32_t* filt_off,
                   const int32_t* filt, uint8_t* keep) {
  if (!c || n < 0 || (n > 0 && (!heads || !filt_off || !keep))) return KP_EINVAL;
  return guarded(c, [&] {
    KP_REQUIRE(obj >= 0 && obj < c->n_ent, "kp_convertible: object out of range");
    KP_REQUIRE(rel >= 0 && rel < c->n_rel2, "kp_convertible: relation out of range");
    if (n == 0) return;
    KP_HIP(hipSetDevice(c->device));
    for (int i = 0; i < n; ++i) KP_REQUIRE(heads[i] >= 0 && heads[i] < c->n_ent, "kp_convertible: head out of range");
    // engine.py:94-120 -- score chunks of heads on the device, mask the filter, compare with the extreme
    const size_t budget = (size_t)256 << 20;
    const int chunk = (int)std::max<size_t>(64, std::min<size_t>(4096, budget / ((size_t)c->n_ent * 4)));
    const int ld = c->n_ent;
    std::vector<int32_t> rels(chunk, rel), fo(chunk + 1);
    DevBuf bS, bH, bR, bFo, bF, bK;
    float* dS = reinterpret_cast<float*>(bS.ensure(sizeof(float) * (size_t)chunk * ld));
    const bool minimizer = (c->model == KP_MODEL_TRANSE);
    for (int i0 = 0; i0 < n; i0 += chunk) {
      const int m = std::min(chunk, n - i0);
      int32_t* dH = upload(c, bH, heads + i0, (size_t)m);
      int32_t* dR = upload(c, bR, rels.data(), (size_t)m);
      for (int j = 0; j <= m; ++j) fo[j] = filt_off[i0 + j] - filt_off[i0];
      int32_t* dFo = upload(c, bFo, fo.data(), (size_t)m + 1);
      int32_t* dF = upload(c, bF, filt + filt_off[i0], (size_t)std::max(1, fo[m]));
      uint8_t* dK = reinterpret_cast<uint8_t*>(bK.ensure((size_t)m));
      switch (c->model) {
        case KP_MODEL_COMPLEX: complex_scores_dev(c, m, dH, dR, dS, ld); break;
        case KP_MODEL_TRANSE: transe_scores_dev(c, m, dH, dR, dS, ld); break;
        case KP_MODEL_CONVE: conve_scores_dev(c, m, dH, dR, dS, ld); break;
      }
      launch_convertible_reduce(c, m, dS, ld, obj, dFo, dF, minimizer ? 1 : 0, dK);
      KP_HIP(hipMemcpyAsync(keep + i0, dK, (size_t)m, hipMemcpyDeviceToHost, c->stream));
      KP_HIP(hipStreamSynchronize(c->stream));
    }
    for (DevBuf* b : {&bS, &bH, &bR, &bFo, &bF, &bK}) b->release();
  });
}

int kp_train_epoch(kp_ctx* c, const kp_hp* hp, int32_t n, const int32_t* triples, const int32_t* aux,
                   int32_t epoch) {
  if (!c || !hp || n <= 0 || !triples || !aux || epoch < 0) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    if (c->model == KP_MODEL_TRANSE)
      transe_train_epoch(c, hp, n, triples, aux, epoch);
    else
      complex_train_epoch(c, hp, n, triples, aux, epoch);
  });
}

int kp_conve_train_begin(kp_ctx* c, const float* bn_weight, const float* bn_bias, const float* bn_mean,
                         const float* bn_var) {
  if (!c || !bn_weight || !bn_bias || !bn_mean || !bn_var) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    conve_train_begin(c, bn_weight, bn_bias, bn_mean, bn_var);
  });
}

int kp_conve_train_step(kp_ctx* c, int32_t B, const int32_t* pairs, const int32_t* tail_off, const int32_t* tails,
                        const float* in_noise, const float* fm_noise, const float* hid_noise, float lr,
                        float label_smoothing, int32_t bn_train) {
  if (!c || B <= 0 || !pairs || !tail_off || (tail_off[B] > 0 && !tails)) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    conve_train_step(c, B, pairs, tail_off, tails, in_noise, fm_noise, hid_noise, lr, label_smoothing, bn_train);
  });
}

int kp_conve_train_read(kp_ctx* c, float* conv_w, float* conv_b, float* fc_w, float* fc_b, float* bn_weight,
                        float* bn_bias, float* bn_mean, float* bn_var) {
  if (!c || !conv_w || !conv_b || !fc_w || !fc_b || !bn_weight || !bn_bias || !bn_mean || !bn_var) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    conve_train_read(c, conv_w, conv_b, fc_w, fc_b, bn_weight, bn_bias, bn_mean, bn_var);
  });
}

int kp_read_tables(kp_ctx* c, float* entity, float* relation) {
  if (!c || !entity || !relation) return KP_EINVAL;
  return guarded(c, [&] {
    KP_HIP(hipSetDevice(c->device));
    KP_HIP(hipStreamSynchronize(c->stream));
    KP_HIP(hipMemcpy2D(entity, sizeof(float) * c->dim, c->dE, sizeof(float) * c->dp, sizeof(float) * c->dim,
                       c->n_ent, hipMemcpyDeviceToHost));
    KP_HIP(hipMemcpy2D(relation, sizeof(float) * c->dim, c->dR, sizeof(float) * c->dp, sizeof(float) * c->dim,
                       c->n_rel2, hipMemcpyDeviceToHost));
  });
}

int kp_predict_tails(kp_ctx* c, int32_t n, const int32_t* triples, const int32_t* filt_off, const int32_t* filt,
                     float* out_score, int64_t* out_rank) {
  if (!c || n < 0 || (n > 0 && (!triples || !filt_off || !out_score || !out_rank))) return KP_EINVAL;
  return guarded(c, [&] {
    if (n == 0) return;
    KP_HIP(hipSetDevice(c->device));
    for (int i = 0; i < n; ++i) {
      KP_REQUIRE(triples[3 * i] >= 0 && triples[3 * i] < c->n_ent, "kp_predict_tails: head out of range");
      KP_REQUIRE(triples[3 * i + 1] >= 0 && triples[3 * i + 1] < c->n_rel2, "kp_predict_tails: relation out of range");
      KP_REQUIRE(triples[3 * i + 2] >= 0 && triples[3 * i + 2] < c->n_ent, "kp_predict_tails: tail out of range");
      KP_REQUIRE(filt_off[i + 1] >= filt_off[i], "kp_predict_tails: bad filter offsets");
    }
    // Model.predict_tails (model.py:42-68) / ConvE.predict_tails (conve.py:160-184):
    // score chunks of triples against every entity, then the filtered rank
    const size_t budget = (size_t)256 << 20;
    const int chunk = (int)std::max<size_t>(64, std::min<size_t>(4096, budget / ((size_t)c->n_ent * 4)));
    const int ld = c->n_ent;
    const int mode = (c->model == KP_MODEL_CONVE) ? RANK_SORT_POSITION : RANK_PREDICT_TAILS;
    const bool minimizer = (c->model == KP_MODEL_TRANSE);
    std::vector<int32_t> h(chunk), r(chunk), o(chunk), fo(chunk + 1);
    DevBuf bS, bH, bR, bO, bFo, bF, bT, bK;
    float* dS = reinterpret_cast<float*>(bS.ensure(sizeof(float) * (size_t)chunk * ld));
    for (int i0 = 0; i0 < n; i0 += chunk) {
      const int m = std::min(chunk, n - i0);
      for (int j = 0; j < m; ++j) {
        h[j] = triples[3 * (i0 + j)];
        r[j] = triples[3 * (i0 + j) + 1];
        o[j] = triples[3 * (i0 + j) + 2];
      }
      for (int j = 0; j <= m; ++j) fo[j] = filt_off[i0 + j] - filt_off[i0];
      int32_t* dH = upload(c, bH, h.data(), (size_t)m);
      int32_t* dR = upload(c, bR, r.data(), (size_t)m);
      int32_t* dO = upload(c, bO, o.data(), (size_t)m);
      int32_t* dFo = upload(c, bFo, fo.data(), (size_t)m + 1);
      int32_t* dF = upload(c, bF, filt + filt_off[i0], (size_t)std::max(1, fo[m]));
      float* dT = reinterpret_cast<float*>(bT.ensure(sizeof(float) * (size_t)m));
      int64_t* dK = reinterpret_cast<int64_t*>(bK.ensure(sizeof(int64_t) * (size_t)m));
      switch (c->model) {
        case KP_MODEL_COMPLEX: complex_scores_dev(c, m, dH, dR, dS, ld); break;
        case KP_MODEL_TRANSE: transe_scores_dev(c, m, dH, dR, dS, ld); break;
        case KP_MODEL_CONVE: conve_scores_dev(c, m, dH, dR, dS, ld); break;
      }
      launch_rank_count(c, m, dS, ld, c->n_ent, dO, dFo, dF, minimizer ? 1 : 0, dT, dK, mode);
      KP_HIP(hipMemcpyAsync(out_score + i0, dT, sizeof(float) * m, hipMemcpyDeviceToHost, c->stream));
      KP_HIP(hipMemcpyAsync(out_rank + i0, dK, sizeof(int64_t) * m, hipMemcpyDeviceToHost, c->stream));
      KP_HIP(hipStreamSynchronize(c->stream));
    }
    for (DevBuf* b : {&bS, &bH, &bR, &bO, &bFo, &bF, &bT, &bK}) b->release();
  });
}

int kp_dp_relevance(kp_ctx* c, int32_t n, const int32_t* items, float epsilon, float lambd, int32_t step_sign,
                    int32_t rel_sign, float* out) {
  if (!c || n < 0 || (n > 0 && (!items || !out)) || (step_sign != 1 && step_sign != -1) ||
      (rel_sign != 1 && rel_sign != -1))
    return KP_EINVAL;
  return guarded(c, [&] {
    if (n == 0) return;
    KP_HIP(hipSetDevice(c->device));
    dp_relevance(c, n, items, epsilon, lambd, step_sign, rel_sign, out);
  });
}

int kp_criage_relevance(kp_ctx* c, int32_t n, const int32_t* items, int32_t n_ents, const int32_t* ent_ids,
                        const int32_t* tails_off, const int32_t* tails, double* out, int32_t* status) {
  if (!c || n < 0 || n_ents < 0 || (n > 0 && (!items || !out || !status || n_ents == 0)) ||
      (n_ents > 0 && (!ent_ids || !tails_off)))
    return KP_EINVAL;
  return guarded(c, [&] {
    if (n == 0) return;
    KP_HIP(hipSetDevice(c->device));
    criage_relevance(c, n, items, n_ents, ent_ids, tails_off, tails, out, status);
  });
}

// The host RNG protocol entry points (kp_rng_*, kp_mt19937_discard) are in kp_rng.cpp.

int kp_hot_intervals(const kp_ctx* c, int64_t cap, double* out, int64_t* n) {
  if (!c || cap < 0 || (cap > 0 && !out)) return KP_EINVAL;
  const int64_t have = (int64_t)(c->hot_iv.size() / 2);
  if (n) *n = have;
  for (int64_t i = 0; i < std::min(cap, have); ++i) {
    out[2 * i] = c->hot_iv[2 * i];
    out[2 * i + 1] = c->hot_iv[2 * i + 1];
  }
  return KP_OK;
}

int kp_last_timing(const kp_ctx* c, double* dev_s, double* hot_s, int64_t* hot_n, double* hot_w) {
  if (!c) return KP_EINVAL;
  if (hot_w) *hot_w = c->timing.hot_work;
  if (dev_s) *dev_s = c->timing.device_s;
  if (hot_s) *hot_s = c->timing.hot_s;
  if (hot_n) *hot_n = c->timing.hot_launches;
  return KP_OK;
}

}  // extern "C"
