// Entry points whose kernels land in later commits: they report
// PCOPS_ERR_UNSUPPORTED so the ABI (include/pcops.h) is complete and loadable.
#include "common.h"

extern "C" unsigned long long pcops_emd_workspace_bytes(int, int) { return 0; }
extern "C" int pcops_emd_forward(const float *, const float *, int, int, float, int, float *, int *, void *,
                                 unsigned long long, pcops_stream_t) { return PCOPS_ERR_UNSUPPORTED; }
extern "C" int pcops_emd_backward(const float *, const float *, const float *, const int *, int, int, float *,
                                  pcops_stream_t) { return PCOPS_ERR_UNSUPPORTED; }
