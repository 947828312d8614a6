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

/* Diagnostic: the fp64 path's elementary functions (wc_device.h f64m) on n
 * device inputs: fn 0 exp2 (double in), 1 rcp (double), 2 log_u24 (uint32 odd
 * v: ln(v 2^-24)), 3 sincospi_v23 (uint32 odd v: out[2i], out[2i+1] = sin, cos
 * of pi v 2^-23), 4 the fp64 sigmoid 1/(1 + e^(-(x - 1) s)) of (x, s) pairs,
 * 5 sqrt_pos (double in, normal positive); 16, 18, 19: fn 0, 2, 3 with the
 * coefficients read from the constant table (TabCoef, the WC_F64_TAB = 1 form). */
int wc_diag_f64m(int fn, int64_t n, const void* in, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WCSDE_DIAG_H */
