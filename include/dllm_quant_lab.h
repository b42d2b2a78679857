/* dllm_quant_lab.h -- entry points of the LAB build only (libdllm_hip_lab.so, `make lab`,
 * -DDLLM_LAB=1), for the measurement scripts' A/B runs.  Not part of the product ABI: the product
 * library (libdllm_hip.so) exports none of these, and include/dllm_quant.h does not declare them. */
#ifndef DLLM_QUANT_LAB_H
#define DLLM_QUANT_LAB_H
#include "dllm_quant.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Lab build only (libdllm_hip_lab.so): A/B schedule variants and ablation masks; mutates the
 * handle, so it is not part of the product ABI.  -1: product policy; 4: rounded-weight policy;
 * 14 / 15: exact-weight 128x256 / tile-major 256x256; 0..3, 5..13: round-1 schedules;
 * 16..23, 32..95, 100..195: ablation masks (results are garbage); 200..263: decode tile override. */
int dllm_linear_set_kernel_variant(dllm_linear_t h, int variant);
#ifdef __cplusplus
}
#endif
#endif /* DLLM_QUANT_LAB_H */
