/*
 * wcsde.h -- C ABI of libwcsde.so, the MI355X (gfx950) Wilson-Cowan SDE sweep
 * engine.  Plain pointers and sizes only; no torch types cross this boundary.
 *
 * The reference (vandal-uv/NREMmodFC) has no FFI: its boundary is the Python
 * module surface of netwWilsonCowanPlastic.  Each entry point
 * below replaces one piece of that surface; the Python mirror in
 * nremmodfc_amd/ (netwWilsonCowanPlastic.py, utils.py, sweep.py) binds them
 * with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - every array argument is DEVICE memory owned by the caller (e.g. a
 *    torch.cuda tensor's data_ptr()), contiguous, batch-major unless stated;
 *  - no allocation, no host synchronisation inside a call: work is enqueued on
 *    `stream` (a hipStream_t, NULL = default stream) and the call returns;
 *  - return 0 on success or a negative WC_E* code; wc_last_error() gives a
 *    thread-local message for the last failure on the calling thread;
 *  - reentrant: no global mutable state.
 */
#ifndef WCSDE_H
#define WCSDE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WCSDE_ABI_VERSION 1

/* Noise stream (the reference's numba RNG is seeded from os.urandom and never
 * reproducible; the build defines its own): Philox4x32-10 with
 * key (WC_PHILOX_KEY0, WC_PHILOX_KEY1) and counter
 *   (step & 0xffffffff, ((step >> 32) << 16) | quad, simkey lo32, simkey hi32)
 * for global Euler step `step` (< 2^48), node quad `quad` = node / 4 (< 2^16)
 * and the 64-bit per-simulation key; outputs x0..x3 ->
 *   u = (2*(x >> 9) + 1) * 2^-24,
 *   z[4q+0,1] = sqrt(-2 ln u0) (cos, sin)(2 pi u1),  z[4q+2,3] likewise from u2, u3,
 * and the noise of wc:80 is sqdtD * z. */
#define WC_PHILOX_KEY0 0x243F6A88u
#define WC_PHILOX_KEY1 0x85A308D3u

enum wc_precision { WC_F32 = 0, WC_F64 = 1 };

enum wc_error {
    WC_OK = 0,
    WC_EINVAL = -1,     /* bad shape / argument */
    WC_EUNSUPPORTED = -2, /* N outside the compiled tile range */
    WC_EWORKSPACE = -3, /* workspace NULL or too small */
    WC_EHIP = -4        /* a HIP runtime call failed */
};

/* Node/model constants of netwWilsonCowanPlastic.py:20-57 (drivers override P
 * and rhoE, whole_sweep_both.py:39-40).  sqdtD = D/sqrt(dtSim) is the std of
 * the per-step noise drawn inside the E sigmoid (wc:55-57, wc:80-81). */
typedef struct wc_params {
    double a_ee, a_ei, a_ii;
    double tauE, tauI;
    double P, rhoE;
    double rE, rI, mu, sigmaI;
    double sqdtD;
    double dtSim;
} wc_params;

int wcsde_abi_version(void);
const char* wc_last_error(void);

/* Bytes of device workspace wc_integrate needs for an N-node connectome (the
 * connectome's MFMA A-operand image, rebuilt by every call). */
size_t wc_workspace_size(int N, int precision);

/*
 * Advance B independent simulations by `nsteps` Euler-Maruyama steps of the
 * plastic Wilson-Cowan network.  Replaces the per-step work of
 * netwWilsonCowanPlastic.wilsonCowan (wc:77-83) and the three Euler loops of
 * run() (wc:101-135); the host calls it once per phase/chunk with that
 * phase's tau_ip (0.05, 1, 2: wc:95,110,118).
 *
 *  sc        [N][N] fp64     structural connectome CM (row i = target node)
 *  G,sigmaE  [B][N] fp64     per-simulation, per-node coupling and E slope
 *                            (homogeneous sweeps repeat one value per row;
 *                            maps mode G_i = G + dG*m_i, whole_sweep_both_maps.py:104-108)
 *  keys      [B]    uint64   Philox4x32-10 key of each simulation's noise stream
 *  E,I,A     [B][N] fp64     state (E, I, a_ie), read at entry, written at exit
 *  step0                     global step index of the first step (Philox counter)
 *  rec_every >0: store the state BEFORE the update of every local step s with
 *            s % rec_every == 0 (wc:124-125) at row s/rec_every of recE/recI/recA,
 *            layout [n_rec][B][N], element type float (WC_F32) or double (WC_F64);
 *            recI/recA may be NULL.  rec_every == 0: no recording.
 *  precision WC_F32: E, I, sigmoids in fp32; coupling as six bf16 MFMA cross
 *            terms of 3-way split operands with fp32 accumulation (fp32-
 *            equivalent); a_ie as a compensated fp32 pair;
 *            WC_F64: everything fp64 (the parity mode).
 */
int wc_integrate(const wc_params* p, int precision, int B, int N,
                 const double* sc, const double* G, const double* sigmaE,
                 const uint64_t* keys, double* E, double* I, double* A,
                 int64_t step0, int64_t nsteps, double tau_ip,
                 int64_t rec_every, void* recE, void* recI, void* recA,
                 void* workspace, size_t ws_bytes, void* stream);

/* Standard normals the integrator draws at global step `step`: out [B][N]
 * (float or double per precision).  Test hook for the noise stream. */
int wc_noise(int precision, int B, int N, const uint64_t* keys, int64_t step,
             void* out, void* stream);

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

#endif /* WCSDE_H */
