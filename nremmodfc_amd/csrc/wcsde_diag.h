/* wcsde_diag.h -- ablation entry point of libwcsde_diag.so (tools/diag_*.py only).
 * Built with -DWCSDE_DIAG by `python -m nremmodfc_amd._build --diag`; the product
 * library libwcsde.so does not export it. */
#ifndef WCSDE_DIAG_H
#define WCSDE_DIAG_H
#include "wcsde.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Diagnostic: wc_integrate (WC_F32, no recI/recA) through compile-time kernel
 * variant `variant` (ablations / alternative tilings, see wc_sde.hip
 * launch_diag); 81 <= N <= 96 only.  Not part of the product path. */
int wc_diag_integrate(int variant, const wc_params* p, int B, int N,
                      const double* sc, const double* G, const double* sigmaE,
                      const uint64_t* keys, double* E, double* I, double* A,
                      int64_t step0, int64_t nsteps, double tau_ip,
                      int64_t rec_every, void* recE,
                      void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WCSDE_DIAG_H */
