/*
 * ldpc_nms_debug.h — test infrastructure exported by libldpc_nms.so (not part of the decoder
 * ABI in ldpc_nms.h; host only, touches no device).
 */
#ifndef LDPC_NMS_DEBUG_H
#define LDPC_NMS_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Host-side bounds check of the bit-sliced kernel's reads (csrc/ldpc_bs.hip bs_bounds_check):
 * for every kernel instance (kBsInst) and UCN setting whose plan serves the proto graph with
 * the given weight properties (alpha_uniform: one check weight per iteration; beta_uniform: one
 * channel weight per iteration), the launch's own planning and host tables are built and every
 * index the kernel reads -- global tables, LDS regions, the dynamic LDS size -- is checked
 * against the allocation.  mode: the internal QMS mode (1 = q 5, 2 = q -5, 3 = q 4, 4 = q 3).
 * flags bit 0 (LDPC_BOUNDS_PRE_GUARD): check the cn_hd read without the `ql < cn_lanes` guard
 * (the round-4 fault), so a test can see the check catch it.  Returns the number of plans
 * checked (>= 0) or a negative status; *violations = out-of-bounds reads found, msg = the
 * first one ("" if none). */
int ldpc_debug_bs_bounds(const int32_t* proto, int32_t M, int32_t N, int32_t z, int32_t T,
                         int32_t mode, int32_t alpha_uniform, int32_t beta_uniform, float clip,
                         int32_t flags, int32_t* violations, char* msg, int32_t msg_len);

#ifdef __cplusplus
}
#endif

#endif /* LDPC_NMS_DEBUG_H */
