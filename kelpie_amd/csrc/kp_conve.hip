// kp_conve.hip -- ConvE post-training (placeholder until the kernel lands).
#include "kp_common.hpp"
void conve_posttrain_rank(kp_ctx*, const kp_hp*, const kp_batch*) {
  throw KpError{KP_ENOTSUP, "ConvE kernels not built yet"};
}
void conve_all_scores(kp_ctx*, int, const int32_t*, const int32_t*, float*) {
  throw KpError{KP_ENOTSUP, "ConvE kernels not built yet"};
}
void conve_scores_dev(kp_ctx*, int, const int32_t*, const int32_t*, float*, int) {
  throw KpError{KP_ENOTSUP, "conve kernels not built yet"};
}
