/*
 * kelpie_hip.h -- C ABI of the MI355X-native Kelpie relevance engine.
 *
 * The reference has no FFI: its relevance engine is the Python class API of
 * src/relevance_engines/post_training_engine.py.  This library replaces the
 * arithmetic below that API (KelpieModel construction, the Kelpie optimizers'
 * post-training loop and get_triple_results' all-entity filtered rank); the
 * Python package kelpie_amd binds it with ctypes and re-exposes the
 * reference's class interface (NecessaryPostTrainingEngine, ...).  Each entry
 * point names the reference code it replaces.
 *
 * Conventions
 *   - every function returns 0 on success, a negative KP_E* code otherwise;
 *     kp_last_error(ctx) describes the last failure (thread-local when ctx is
 *     NULL, e.g. for a failed kp_ctx_create);
 *   - all pointers are HOST pointers owned by the caller; the context copies
 *     what it needs to device memory and owns that copy;
 *   - calls are synchronous at return; a context is not re-entrant (one host
 *     thread per context);
 *   - entity ids: frozen entities are [0, n_ent); the kelpie ("mimic") entity
 *     of a slot has id n_ent, like KelpieDataset.kelpie_entity
 *     (src/data/kelpie_dataset.py:20-25);
 *   - relation ids: [0, n_rel2) with n_rel2 = 2|R|; inverse of p is p+|R|
 *     (src/data/dataset.py:319-331).
 */
#ifndef KELPIE_HIP_H
#define KELPIE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KP_OK 0
#define KP_EINVAL (-22)
#define KP_ENOMEM (-12)
#define KP_EDEVICE (-5)
#define KP_ENOTSUP (-95)
/* kp_rng_transe_calls_async only: no walker thread could start, so the walk ran inline
 * on the caller's thread; torch_state then holds the advanced stream (not an error) */
#define KP_INLINE 1

/* model families (src/link_prediction/__init__.py:5-9, MODEL_REGISTRY) */
#define KP_MODEL_TRANSE 0
#define KP_MODEL_COMPLEX 1
#define KP_MODEL_CONVE 2

/* optimizers (multiclass_nll_optimizer.py:41-48; Kelpie TransE / ConvE use Adam) */
#define KP_OPT_ADAGRAD 0
#define KP_OPT_ADAM 1
#define KP_OPT_SGD 2

typedef struct kp_ctx kp_ctx;

/* Frozen model tables.  Replaces the E/R clones every KelpieModel makes per
 * candidate (transe.py:86-87, complex.py:146-147, conve.py:206-207): the
 * tables are uploaded ONCE per context and shared by every slot. */
typedef struct {
  int32_t model;      /* KP_MODEL_* */
  int32_t n_ent;      /* |E| */
  int32_t n_rel2;     /* 2|R| */
  int32_t dim;        /* row width: TransE/ConvE d, ComplEx 2d ([Re | Im], complex.py:24-25) */
  const float* entity;   /* [n_ent][dim] */
  const float* relation; /* [n_rel2][dim] */
  /* ConvE frozen layers (conve.py:40-52, frozen copies at :214-237); NULL otherwise */
  const float* conv_w;   /* [32][3][3] (Conv2d(1,32,3) weight) */
  const float* conv_b;   /* [32] */
  const float* fc_w;     /* [dim][hidden], hidden = 32*38*(dim/20-2) */
  const float* fc_b;     /* [dim] */
  const float* bn_alpha; /* [1 + 32 + dim]: eval-mode BN1|BN2|BN3 scale  w/sqrt(var+eps) */
  const float* bn_beta;  /* [1 + 32 + dim]: eval-mode BN1|BN2|BN3 shift  b - mean*scale  */
  /* TransE score norm p (TransEHyperParams.norm, transe.py:12-15,46; tune.py:19 searches
   * {1, 2}): 2 = L2, 1 = L1, 0 = the default 2; must be 0 for the other models */
  int32_t norm_p;
} kp_model_desc;

/* Post-training hyper-parameters (the *_explanation.json "training" block,
 * validated by the optimizers' HyperParams classes). */
typedef struct {
  int32_t optimizer;     /* KP_OPT_*; TransE and ConvE: KP_OPT_ADAM */
  int32_t epochs;
  int32_t batch_size;
  float lr;              /* ConvE: 1e-3 (KelpieBCEOptimizer ignores hp lr, bce_optimizer.py:165) */
  float beta1, beta2;    /* Adam betas */
  float eps;             /* Adagrad 1e-10, Adam 1e-8 */
  float reg_weight;      /* ComplEx N3 weight / TransE L2 weight */
  float margin;          /* TransE */
  int32_t neg_ratio;     /* TransE negative_triples_ratio */
  float label_smoothing; /* ConvE */
  float hidden_dropout;  /* ConvE hidden dropout rate (masks are inputs) */
  float input_dropout;   /* ConvE input dropout rate (conve.py:142) */
  float fmap_dropout;    /* ConvE feature-map Dropout2d rate (conve.py:147) */
  int32_t reg_kind;      /* ComplEx regulariser (multiclass_nll_optimizer.py:45-48): KP_REG_N3 | KP_REG_N2 */
} kp_hp;

enum { KP_REG_N3 = 0, KP_REG_N2 = 1 }; /* regularizers.py:37-46 (N3), :25-35 (N2) */

/* One batch of post-training slots.  A slot is one KelpieModel post-training
 * (PostTrainingEngine.post_train, post_training_engine.py:64-76) followed by
 * get_triple_results (:101-125).  Base and post-trained models are both just
 * slots.
 *
 *   x0          [n_slots][dim]   initial kelpie row (after the model's init:
 *                                ComplEx init*init_scale, TransE xavier, ConvE raw)
 *   row_off     [n_slots+1]      CSR offsets into rows
 *   rows        [total][3]       training rows of each slot: the kelpie triples
 *                                followed by their inverses, in reference order
 *                                (optimizer.train's vstack(triples, inverse))
 *   rng_off     [n_slots+1]      CSR offsets (in int32 words) into rng
 *   rng         [...]            per-slot random draws, generated on the host in
 *                                reference order (RNG-as-input):
 *       ComplEx: epochs x R permutation (torch.randperm, multiclass_nll_optimizer.py:148)
 *       TransE:  epochs x [R row order | R negative entities | R head_or_tail]
 *                (pairwise_ranking_optimizer.py:166-181; only rows [0,R) are stepped)
 *       ConvE:   per step: ceil(b*dim/32) words of hidden-dropout keep bits
 *   pred        [n_slots][3]     kelpie-form triple to rank (s = n_ent)
 *   filt_off    [n_slots+1]      CSR offsets into filt
 *   filt        [...]            entities filtered out of the rank (to_filter[(s,p)]
 *                                of the slot's KelpieDataset after the edit)
 * outputs:
 *   out_x       [n_slots][dim]   final kelpie rows (may be NULL)
 *   out_score   [n_slots]        target score  (all_scores[o])
 *   out_rank    [n_slots]        filtered rank (minimizer: <=, o restored before
 *                                counting; maximizer: >=, o excluded if filtered)
 */
typedef struct {
  int32_t n_slots;
  const float* x0;
  const int32_t* row_off;
  const int32_t* rows;
  const int64_t* rng_off;
  const int32_t* rng;
  const int32_t* pred;
  const int32_t* filt_off;
  const int32_t* filt;
  float* out_x;
  float* out_score;
  int64_t* out_rank;
} kp_batch;

/* Create a context on HIP device `device` and upload the frozen tables. */
int kp_ctx_create(int device, const kp_model_desc* model, kp_ctx** out);
int kp_ctx_destroy(kp_ctx* ctx);
const char* kp_last_error(const kp_ctx* ctx);

/* Page-locked host memory (hipHostMalloc) for the buffers the caller fills and a
 * context uploads every batch: the deferred-draw arenas of kelpie_amd.rng, which
 * kp_posttrain_rank then reads by DMA with no staging copy (the reference has no
 * counterpart: its draws never leave the host).  KP_EDEVICE without a usable GPU. */
int kp_host_alloc(size_t bytes, void** out);
int kp_host_free(void* p);

/* Post-train every slot of the batch and rank its target triple.
 * Replaces, per slot: KelpieX(...) construction, Kelpie*Optimizer.train
 * (pairwise_ranking_optimizer.py:160-203, multiclass_nll_optimizer.py:138-164,
 * bce_optimizer.py:161-208) and PostTrainingEngine.get_triple_results
 * (post_training_engine.py:101-125). */
int kp_posttrain_rank(kp_ctx* ctx, const kp_hp* hp, const kp_batch* batch);

/* Model.all_scores (model.py:19; transe.py:48-65, complex.py:88-112,
 * conve.py:133-158) for n (head, relation) pairs over the frozen entities:
 * out[n][n_ent].  The RelevanceEngine.select_entities_to_convert sweep
 * (engine.py:94-101) is built on it. */
int kp_all_scores(kp_ctx* ctx, int32_t n, const int32_t* heads, const int32_t* rels, float* out);

/* Filtered-rank sweep of engine.py:89-120 for n candidate heads e with
 * relation p and object o: keep[i] = 1 iff o is not the model's top-1 for
 * (e,p,.) once to_filter[(e,p)] is masked to +-1e6.  filt CSR as in kp_batch. */
int kp_convertible(kp_ctx* ctx, int32_t n, const int32_t* heads, int32_t rel, int32_t obj,
                   const int32_t* filt_off, const int32_t* filt, uint8_t* keep);

/* Model.predict_tails (src/link_prediction/models/model.py:42-68; ConvE:
 * conve.py:160-184) for n frozen triples (h, r, t), r in [0, n_rel2) (inverse
 * relations give head prediction, model.py:30-31): out_score[i] = score of t,
 * out_rank[i] = filtered rank of t among all entities with to_filter[(h, r)]
 * (CSR as in kp_batch) masked to +-1e6 and t restored, counting <= (TransE) or
 * >= (ComplEx) the target; ConvE ranks by a descending sort with filtered
 * entries at 0.0, i.e. 1 + #(scores > target).  The Evaluator's MRR / Hits@k
 * (link_prediction/evaluation.py:16-48) are computed from these ranks. */
int kp_predict_tails(kp_ctx* ctx, int32_t n, const int32_t* triples, const int32_t* filt_off, const int32_t* filt,
                     float* out_score, int64_t* out_rank);

/* One training epoch of the context's OWN tables, for the retraining of
 * verify_explanations.py:141-143 / :230-232 (RNG-as-input: the host draws what the
 * optimizer draws).  The optimizer state persists across calls and restarts at
 * epoch == 0.
 *  ComplEx: MultiClassNLLOptimizer.epoch (src/link_prediction/optimization/
 *    multiclass_nll_optimizer.py:101-135; ComplEx.forward complex.py:58-86, N3
 *    regularizers.py): triples [n][3] are train()'s stack of the training triples and
 *    their inverses (:66-67), aux [n] this epoch's torch.randperm(n) (:102); batches of
 *    min(hp->batch_size, n) start every hp->batch_size rows (:112-118); Adagrad / Adam /
 *    SGD (hp->optimizer).
 *  TransE: PairwiseRankingOptimizer.epoch (pairwise_ranking_optimizer.py:102-157;
 *    TransE.forward transe.py:67-75, L2 regularizers.py): triples [n][3] are this
 *    epoch's positive rows in order (the stack after its in-place np.random.shuffle),
 *    aux [n][3] the matching corrupted rows (the first n of the epoch's ratio * n
 *    torch.randint draws); MarginRankingLoss(hp->margin), L2 (hp->reg_weight), Adam.
 * ConvE contexts: KP_EINVAL. */
int kp_train_epoch(kp_ctx* ctx, const kp_hp* hp, int32_t n, const int32_t* triples, const int32_t* aux,
                   int32_t epoch);

/* Copy the context's tables to the host: entity [n_ent][dim], relation [n_rel2][dim]
 * (the trained model's state_dict tensors). */
int kp_read_tables(kp_ctx* ctx, float* entity, float* relation);

/* ConvE full-model training (BCEOptimizer.train, bce_optimizer.py:45-150, on ConvE.forward
 * in train mode, conve.py:133-158), for verification's retraining
 * (verify_explanations.py:141-143): the context's tables, conv and FC layers are the
 * starting point and are trained in place; kp_conve_train_begin adds the three batch
 * norms' affine parameters and running statistics (1 + 32 + dim values each: BN1, BN2,
 * BN3) and resets Adam's state.  One kp_conve_train_step = one optimizer step on a batch
 * of B (head, relation) pairs: tails of pair b = tails[tail_off[b] .. tail_off[b+1])
 * (the er_vocab targets); in_noise [B][40 h], fm_noise [B][32], hid_noise [B][dim]: the
 * dropouts' multipliers (0 or 1 / (1 - p), drawn by the caller from the torch generator
 * in the forward's order; null = no dropout); lr = the epoch's learning rate
 * (ExponentialLR); bn_train = 0 runs the batch norms in eval mode (a one-pair batch).
 * Adam with torch's defaults on every parameter.  kp_conve_train_read copies the trained
 * layers back (the tables: kp_read_tables).  The context's eval-mode batch norm is not
 * updated: build a new context from the trained parameters to score with them. */
int kp_conve_train_begin(kp_ctx* ctx, const float* bn_weight, const float* bn_bias, const float* bn_mean,
                         const float* bn_var);
int kp_conve_train_step(kp_ctx* ctx, int32_t B, const int32_t* pairs, const int32_t* tail_off, const int32_t* tails,
                        const float* in_noise, const float* fm_noise, const float* hid_noise, float lr,
                        float label_smoothing, int32_t bn_train);
int kp_conve_train_read(kp_ctx* ctx, float* conv_w, float* conv_b, float* fc_w, float* fc_b, float* bn_weight,
                        float* bn_bias, float* bn_mean, float* bn_var);

/* Data-poisoning relevance, ComplEx (src/relevance_engines/data_poisoning_engine.py:
 * DPEngine.get_gradient :21-49, NecessaryDPEngine.compute_relevance :52-94,
 * SufficientDPEngine.compute_individual_relevance :97-137; the other models have no
 * score_embeddings and raise in the reference).  items[n][7] = (pred s, p, o,
 * perspective entity e, triple h, r, t).  Per item: g = d score(s, p, o) / d emb(e)
 * (the lhs when e == s, else the rhs), e' = emb(e) + step_sign * (epsilon * g), the
 * triple's score with e' in its head when h == e (else in its tail), and
 * out[i] = rel_sign * (score - lambd * perturbed score). */
int kp_dp_relevance(kp_ctx* ctx, int32_t n, const int32_t* items, float epsilon, float lambd, int32_t step_sign,
                    int32_t rel_sign, float* out);

/* CRIAGE score variation (src/relevance_engines/criage_engine.py: compute_hessian
 * :74-104, estimate_score_variation :107-134 / :158-177), ComplEx and ConvE.
 * items[n][5] = (z_pred s, p, z_triple s, p, entity slot); z = criage_first_step
 * (complex.py:131, conve.py:102-124).  Entity slot k is ent_ids[k] with tail
 * triples (h, r) = tails[tails_off[k] .. tails_off[k+1]) in training order.
 * out[i] = z_pred . ((1 - sig) z_triple A^{-1}), A = H_e + sig (1 - sig) z^T z,
 * sig = sigmoid(e . z_triple), in float64 (the necessary engine negates it);
 * status[i] = 1 when A is exactly singular (numpy.linalg.inv raises). */
int kp_criage_relevance(kp_ctx* ctx, int32_t n, const int32_t* items, int32_t n_ents, const int32_t* ent_ids,
                        const int32_t* tails_off, const int32_t* tails, double* out, int32_t* status);

/* Advance a torch CPU generator state (the 5056-byte torch.get_rng_state()
 * blob) by n 32-bit mt19937 outputs, in place.  Used by the host RNG protocol
 * to replay the draws of reset_parameters() that each KelpieConvE
 * construction makes (conve.py:46-52 via :202) without materialising them. */
int kp_mt19937_discard(uint8_t* state, size_t state_len, uint64_t n);

/* Batches of deferred draws (the host RNG protocol, kelpie_amd/rng.py): every task queued
 * by kp_rng_transe_enqueue / kp_rng_transe_calls_async / kp_rng_conve_masks_enqueue is
 * tagged with the batch open at the time (tasks queued by a task inherit its tag).
 * kp_rng_batch_close closes the open batch and returns its id; kp_rng_batch_wait(id)
 * returns once every task of the batches <= id is done, while later batches' tasks may
 * still be queued or running -- so the thread that packs batch k waits for batch k's
 * draws while the scheduling thread already queues batch k + 1's (kp_rng_wait waits
 * for everything). */
int kp_rng_batch_close(int64_t* id);
int kp_rng_batch_wait(int64_t id);

/* torch.empty(n).normal_(mean, std) on the CPU generator for float32, n >= 16
 * (ATen normal_fill / normal_fill_AVX2, aten/src/ATen/native/cpu/DistributionTemplates.h),
 * bit for bit, advancing the state blob like torch.  cap = 1 for torch's AVX2 / AVX512 CPU
 * kernels (torch.backends.cpu.get_cpu_capability()), 0 for its scalar default kernel.
 * Replaces the xavier_normal_ of KelpieTransE (src/link_prediction/models/transe.py:93-95). */
int kp_rng_normal(uint8_t* state, size_t state_len, int64_t n, float mean, float std, int32_t cap, float* out);

/* Keep-mask of torch.empty(n).bernoulli_(p) on the CPU generator (ATen draws
 * one random64 = (hi << 32) | lo per element; keep iff u53 * 2^-53 < p), written
 * as packed bits (bit i of word i/32) and advancing the state blob in place.
 * Replaces the per-step hidden-dropout mask draw of KelpieConvE training
 * (conve.py:151 via model.py:114-125, Dropout stays in train mode). */
int kp_rng_bernoulli_bits(uint8_t* state, size_t state_len, uint64_t n, double p, uint32_t* out_bits);

/* One TransE post-training's draws (pairwise_ranking_optimizer.py:166-172) for
 * `epochs` epochs over R rows, from the two process-global generators the
 * reference uses: per epoch np.random.shuffle of the rows (numpy's legacy
 * MT19937 state: key[624] and *pos, from np.random.get_state()), then
 * torch.randint(n_entities, ratio*R) and torch.randint(2, ratio*R) on the torch
 * CPU generator.  Writes per epoch [row order (R) | entity (R) | head_or_tail (R)]
 * (only the first R of the ratio*R draws are stepped) and advances both states. */
int kp_rng_transe_epochs(uint8_t* torch_state, size_t torch_len, uint32_t* np_key, int32_t* np_pos, int32_t R,
                         int32_t epochs, int32_t ratio, int64_t n_entities, int32_t* out);

/* Deferred form of kp_rng_transe_epochs for a batch of slots scheduled in order:
 * snapshots the torch state, advances it past the slot's randints at once, and
 * queues the draws.  One worker thread runs the queued numpy shuffles in queue
 * order on the live numpy state at np_key / np_pos (which nobody else may touch
 * until kp_rng_wait returns); a small pool (KP_RNG_THREADS, default 4) fills the
 * randints from each snapshot.  `out` must stay valid until kp_rng_wait.
 * Same draws, same final states as calling kp_rng_transe_epochs per slot. */
int kp_rng_transe_enqueue(uint8_t* torch_state, size_t torch_len, uint32_t* np_key, int32_t* np_pos, int32_t R,
                          int32_t epochs, int32_t ratio, int64_t n_entities, int32_t* out);

/* The torch / numpy draws of n TransE compute_relevance calls, in the reference's order
 * (post_training_engine.py:46-62 with transe.py:93-95 and
 * pairwise_ranking_optimizer.py:166-181), in one library call.  Per call i:
 * torch.rand(1, D) (its values are overwritten, only the state advances), xavier_normal_
 * of the base kelpie row -> x_base[i] (kp_rng_normal, std = xavier_std), the base
 * post-training's epoch draws if R_base[i] >= 0, xavier_normal_ of the post-trained row
 * -> x_pt[i], and its epoch draws if R_pt[i] >= 0 (R = -1: the call schedules no such
 * post-training).  The epoch draws (as kp_rng_transe_epochs, deferred as
 * kp_rng_transe_enqueue: complete after kp_rng_wait) go to `out` back to back in that
 * order.  want (NULL = all): per call, bit 0 = the base post-training's draws are
 * wanted, bit 1 = the post-trained one's; an unwanted post-training (one that another
 * rank runs, kelpie_amd/distributed.py) only advances both generators and takes no
 * space in `out`.  d >= 16; x_base / x_pt are [n][d]. */
int kp_rng_transe_calls(uint8_t* torch_state, size_t torch_len, uint32_t* np_key, int32_t* np_pos, int32_t cap,
                        int32_t D, int32_t d, float xavier_std, int32_t n, const int32_t* R_base,
                        const int32_t* R_pt, const uint8_t* want, int32_t epochs, int32_t ratio,
                        int64_t n_entities, float* x_base, float* x_pt, int32_t* out);

/* kp_rng_transe_calls with the torch-stream walk on the library's walker thread: returns
 * at once; x_base, x_pt and out are complete after kp_rng_wait().  The walk starts from
 * torch_state unless an earlier asynchronous walk still carries the stream (it then
 * continues that one and torch_state is not read); kp_rng_torch_take hands the stream
 * back.  Lets the scheduling thread queue calls while the generator is advanced past
 * their draws (the randint outputs alone are ~22 M words per TransE batch).  Returns
 * KP_OK when queued, KP_INLINE when it walked inline (then nothing is carried). */
int kp_rng_transe_calls_async(const uint8_t* torch_state, size_t torch_len, uint32_t* np_key, int32_t* np_pos,
                              int32_t normal_cap, int32_t D, int32_t d, float xavier_std, int32_t n,
                              const int32_t* R_base, const int32_t* R_pt, const uint8_t* want, int32_t epochs,
                              int32_t ratio, int64_t n_entities, float* x_base, float* x_pt, int32_t* out);

/* Wait for every asynchronous walk; if one carries the torch stream, store it into
 * torch_state (*taken = 1) and release it, else *taken = 0 and torch_state is untouched. */
int kp_rng_torch_take(uint8_t* torch_state, size_t torch_len, int32_t* taken);

/* Block until every slot queued by kp_rng_transe_enqueue is written. */
int kp_rng_wait(void);

/* ConvE dropout keep bits for n_steps steps of rows_per_step[i] pairs.  Per step, the
 * forward's draws in order (conve.py:142,147,151): for each segment j < n_seg,
 * torch.empty(rows, seg_elems[j]).bernoulli_(seg_keep[j]) -- the input dropout over the
 * 40 x (d/20) image, the feature-map Dropout2d over 32 channels, the hidden dropout over
 * d -- each segment starting on a fresh 32-bit word.  A segment with keep == 0 (rate 1:
 * ATen draws nothing and returns zeros) gets zero words and consumes nothing.  Advances
 * the torch state. */
int kp_rng_conve_masks(uint8_t* torch_state, size_t torch_len, int32_t n_steps, const int32_t* rows_per_step,
                       int32_t n_seg, const int32_t* seg_elems, const double* seg_keep, uint32_t* out_words);

/* Deferred form of kp_rng_conve_masks (see kp_rng_transe_enqueue): advances the
 * torch state now, fills `out_words` on the worker pool; complete after kp_rng_wait. */
int kp_rng_conve_masks_enqueue(uint8_t* torch_state, size_t torch_len, int32_t n_steps, const int32_t* rows_per_step,
                               int32_t n_seg, const int32_t* seg_elems, const double* seg_keep,
                               uint32_t* out_words);

/* Device time of the last kp_posttrain_rank (HIP events on the context's
 * stream): the whole call, the summed durations of its dominant kernel's
 * launches, their count, and the work units those launches processed
 * (ComplEx: query rows x frozen entities; TransE: slot-epochs; ConvE:
 * encoder rows x frozen entities).  bench.py derives the roofline from it. */
int kp_last_timing(const kp_ctx* ctx, double* device_seconds, double* hot_kernel_seconds,
                   int64_t* hot_kernel_launches, double* hot_work_units);

/* [start, end] (seconds, on a time base shared by every context of the device) of
 * each dominant-kernel launch of the last kp_posttrain_rank: *n = the launch count,
 * the first min(cap, *n) pairs are written to out[2 i], out[2 i + 1].  With batches
 * in flight on several contexts the launches can overlap; bench.py merges the
 * intervals to the time the device spent in the kernel. */
int kp_hot_intervals(const kp_ctx* ctx, int64_t cap, double* out, int64_t* n);

/* ---- candidate prefilters, host C++ ----------------
 * The undirected multigraph of TopologyPreFilter / WeightedTopologyPreFilter
 * (topology_prefilter.py:12-14, weighted_topology_prefilter.py:16-18): one
 * edge per training triple (h, t) over entities [0, n_ent); neighbour order is
 * networkx's insertion order.  Errors: kp_graph_last_error() (thread-local). */
typedef struct kp_graph kp_graph;
int kp_graph_create(int32_t n_ent, int64_t n_triples, const int32_t* triples, kp_graph** out);
void kp_graph_destroy(kp_graph* g);
const char* kp_graph_last_error(void);

/* Hop distance from each source to every entity, dist[i * n_ent + v]; -1 when
 * unreachable (nx.NetworkXNoPath -> 1e6 at topology_prefilter.py:36-37).  One
 * search from a prediction's object serves all of its candidates
 * (topology_prefilter.py:29-34 searches once per candidate; distances are symmetric). */
int kp_graph_bfs(const kp_graph* g, int32_t n_src, const int32_t* src, int32_t* dist);

/* Entity classes (CSR: class ids of entity v at cls[cls_off[v] .. cls_off[v+1]))
 * for the edge cost 1 - jaccard_similarity(classes(u), classes(v))
 * (weighted_topology_prefilter.py:40-44, utils/utils.py:11-14), float64. */
int kp_graph_set_classes(kp_graph* g, const int64_t* cls_off, const int32_t* cls);

/* nx.shortest_path_length(G, src[i], dst[i], weight=semantic_score) for each i
 * (weighted_topology_prefilter.py:46-56), replaying networkx's Dijkstra
 * (neighbour order, (distance, push counter) heap) so sums match bit for bit;
 * +inf when there is no path. */
int kp_graph_dijkstra_pairs(const kp_graph* g, int32_t n, const int32_t* src, const int32_t* dst, double* out);

/* ---- slot assembly of a post-training batch, host C++ ----
 * Replaces the per-call KelpieDataset work of the reference
 * (src/data/kelpie_dataset.py:13-158: the deep-copied kelpie dataset, its
 * remove_training_triples / add_training_triples edits and the to_filter lists
 * get_triple_results reads, post_training_engine.py:101-125) for a whole batch of
 * calls: one view per subject, one library call per run of calls, rows and filters
 * packed straight into kp_batch's arrays (csrc/kp_sched.cpp).
 *
 * kp_view_create: base[n][3] = the subject's training triples with the original entity
 * replaced by `kelpie` (the caller's order: Dataset.entity_to_training_triples),
 * extra[m][3] = its validation and test triples (they only enter the filters);
 * n_rel = |R| (inverse relation = p + n_rel). */
typedef struct kp_view kp_view;
typedef struct kp_sched_batch kp_sched_batch;
int kp_view_create(int32_t kelpie, int32_t n_rel, int32_t original, const int32_t* base, int32_t n,
                   const int32_t* extra, int32_t m, kp_view** out);
void kp_view_destroy(kp_view* v);
int kp_sched_batch_create(kp_sched_batch** out);
void kp_sched_batch_destroy(kp_sched_batch* b);

/* n calls: call c ranks (kelpie, rel[c], ·) after editing views[c] with the candidate
 * triples cands[cand_off[c] .. cand_off[c+1]) (original ids); flags[c]: bit 0 the call
 * needs its base post-training, bit 1 this process runs that base slot, bit 2 it runs the
 * edited (pt) slot, bit 3 sufficient mode (an addition; else a removal).  Per call and
 * slot (base, pt): slot_idx[2c + j] (-1: not run here), n_rows[2c + j] (rows incl.
 * inverses), n_filt[2c + j] (filter length).  The edits are checked in the reference's
 * order; at the first failing call fail = {call, code, triple}: code 1 a triple without
 * the entity (AssertionError), 2 not a kelpie training triple (KeyError), 3 a removal the
 * filter multiset cannot take (list.remove ValueError); that call's base slot is added,
 * nothing after it.  Otherwise fail[0] = -1.  The views must outlive the batch. */
int kp_sched_add_calls(kp_sched_batch* b, int32_t n, kp_view* const* views, const int32_t* rel, const uint8_t* flags,
                       const int32_t* cand_off, const int32_t* cands, int32_t* slot_idx, int32_t* n_rows,
                       int32_t* n_filt, int32_t* fail);

/* Rows (kelpie rows then their inverses, the optimizers' order) and rank filters of the
 * batch slots idx[0 .. n), back to back, into rows[rows_cap] / filt[filt_cap] (int32). */
int kp_sched_pack(const kp_sched_batch* b, int32_t n, const int32_t* idx, int32_t* rows, int64_t rows_cap,
                  int32_t* filt, int64_t filt_cap);

/* out[...] = the n int32 arrays (address ptrs[i], counts[i] values) back to back (the
 * slots' draws gathered into one upload buffer without holding the caller's lock). */
int kp_gather_i32(int32_t n, const uint64_t* ptrs, const int64_t* counts, int32_t* out, int64_t cap);

/* Library version string. */
const char* kp_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KELPIE_HIP_H */
