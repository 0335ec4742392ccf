// kp_transe.hip -- TransE post-training (placeholder until the kernel lands).
#include "kp_common.hpp"
void transe_posttrain_rank(kp_ctx*, const kp_hp*, const kp_batch*) {
  throw KpError{KP_ENOTSUP, "TransE kernels not built yet"};
}
void transe_all_scores(kp_ctx*, int, const int32_t*, const int32_t*, float*) {
  throw KpError{KP_ENOTSUP, "TransE kernels not built yet"};
}
void transe_scores_dev(kp_ctx*, int, const int32_t*, const int32_t*, float*, int) {
  throw KpError{KP_ENOTSUP, "transe kernels not built yet"};
}
