// denoiser.hip — placeholder (filled in with the reverse-sweep kernels)
#include "common.h"
extern "C" size_t damc_sweep_workspace_bytes(const damc_denoiser_t*, int) { return 0; }
extern "C" int damc_reverse_sweep(const damc_denoiser_t*, float*, int, int, const float*, int, const float*, uint64_t,
                                  uint64_t, float*, int, void*, size_t, void*) {
  return DAMC_ERR_UNSUPPORTED;
}
