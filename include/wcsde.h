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
 *  - no allocation inside a call; work is enqueued on `stream` (a hipStream_t,
 *    NULL = default stream) and the call returns without host synchronisation
 *    (the one call that waits for the stream is wc_integrate_status, whose
 *    result is a host value);
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

#define WCSDE_ABI_VERSION 7

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
    WC_EUNSUPPORTED = -2, /* size outside what the kernels support */
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

/* Bytes of device workspace wc_integrate needs for B simulations of an N-node
 * connectome.  N <= 96: the connectome's MFMA A-operand image only (state stays
 * in registers for the whole call).  N > 96: the A-operand image plus the
 * tile-major state image and the double-buffered E operand (32 B per
 * node-simulation in fp32, padded to multiples of 64 nodes and simulations). */
size_t wc_workspace_size(int B, int N, int precision);

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
 *            s % rec_every == 0 (wc:124-125) as record k = s/rec_every in
 *            recE/recI/recA, element type float (WC_F32) or double (WC_F64);
 *            recI/recA may be NULL.  rec_every == 0: no recording.
 *  rec_ld    0: records time-major [n_rec][B][N] (Y_t[:, k, :] of run());
 *            > 0: node-major, record k of column c = b*N + n at c*rec_ld + k
 *            (a slot of the sweep pipeline's E ring, read by BOLD and Welch).
 *  precision WC_F32: E, I, sigmoids in fp32; coupling CM.E on the fp16 MFMA:
 *            CM*sA and E*2^10 each split into two fp16 parts (hi + lo, 22
 *            significant bits), three cross terms (lo.hi, hi.lo, hi.hi) with
 *            fp32 accumulation, 1/(2^10 sA) folded into G; a_ie as a
 *            compensated fp32 pair;
 *            WC_F64: everything fp64 (the parity mode).
 *  N <= 96   one launch integrates all nsteps with the state in registers;
 *  N > 96    fp32, nsteps > 1 (the default): ONE persistent cooperative launch
 *            (wc_sde_large.hip persist_kernel) -- one workgroup per CU owns 128
 *            nodes x 80 simulations with their state in registers for all nsteps;
 *            the 8 node blocks of a simulation block exchange the E operand image
 *            through the workspace every step (bounded waits).  If the grid cannot
 *            be made co-resident (cooperative launch refused: too many blocks, or
 *            the CUs are shared) or WCSDE_PERSISTENT=0, and for fp64: one
 *            GEMM-shaped launch per Euler step (step_kernel), the state in the
 *            workspace between steps.  Both give the same bits.  Every wait of
 *            the persistent path is bounded: one that times out sets the
 *            workspace's status word and poisons E, I, A with NaN (carried by
 *            every later call on that state); wc_integrate_status reports it.
 *            Same noise stream on every path.
 */
int wc_integrate(const wc_params* p, int precision, int B, int N,
                 const double* sc, const double* G, const double* sigmaE,
                 const uint64_t* keys, double* E, double* I, double* A,
                 int64_t step0, int64_t nsteps, double tau_ip,
                 int64_t rec_every, int64_t rec_ld, void* recE, void* recI, void* recA,
                 void* workspace, size_t ws_bytes, void* stream);

/* Status of the last wc_integrate call on `workspace` (same B, N, precision):
 * waits for `stream`, then returns WC_EHIP if that call's persistent N > 96
 * integrator had an inter-workgroup wait time out (its E, I, A are NaN), else 0.
 * The one wc_integrate-side call that synchronises; call it when the results are
 * needed anyway (the sweep pipeline: once per batch).  A timed-out call's NaN
 * state propagates through every later call, so a check at the end of a batch
 * also covers its earlier calls (the NaN state or this word).  N <= 96: waits
 * for the stream and returns 0. */
int wc_integrate_status(const void* workspace, int B, int N, int precision, void* stream);

/* Standard normals the integrator draws at global step `step`: out [B][N]
 * (float or double per precision).  Test hook for the noise stream. */
int wc_noise(int precision, int B, int N, const uint64_t* keys, int64_t step,
             void* out, void* stream);

/* One evaluation of netwWilsonCowanPlastic.wilsonCowan(t, X, sigmaE, mu, tau_ip, G)
 * (wc:77-83), fp64, for B simulations: X [B][3][N] rows (E, I, a_ie) -> out
 * [B][3][N] = (dE/dt, dI/dt, da_ie/dt).  The noise of wc:80 is sqdtD times the
 * normals of Philox step `step` of each key (the integrator's normals at that
 * global step); p->mu is the call's mu.  G, sigmaE [B][N]; sc [N][N]. */
int wc_rhs(const wc_params* p, int B, int N, const double* sc, const double* G,
           const double* sigmaE, const uint64_t* keys, int64_t step, double tau_ip,
           const double* X, double* out, void* stream);

/* ------------------------------------------------------------------------
 * simBOLD (netwWilsonCowanPlastic.py:140-158), streamed.
 * Columns c = b*N + n.  The caller allocates wc_bold_state_doubles() doubles
 * of device state, calls wc_bold_init once, wc_bold_chunk for consecutive
 * sample ranges [t0, t0+Tc) of the E trajectory (any chunking), and
 * wc_bold_finish once every sample 0..n_total-1 has been fed: out [M][C] is
 * filtfilt(b, a, BOLD[neq:], axis=0)[::dec], M = ceil((n_total-neq)/dec).
 * BOLD = Balloon-Windkessel of E at step dt (assumed form of the missing
 * BOLDModel.BD.Sim). */
typedef struct wc_bold_cfg {
    double dt;        /* BOLD Euler step: dt*downsamp = 0.04 (wc:144, wc:148) */
    int64_t neq;      /* leading samples dropped (Neq = 2000, wc:145) */
    int64_t n_total;  /* samples of E_t (len(wc.time) = 300000) */
    int64_t dec;      /* BOLD_downsamp (1000; cortex_run.py uses 10) */
    double b[5], a[5]; /* band-pass, a[0] = 1: bessel(2, [2*.01*dt, 2*.1*dt], 'bandpass') (wc:152) */
    double zi[4];     /* scipy.signal.lfilter_zi(b, a) */
} wc_bold_cfg;

int64_t wc_bold_blocks(const wc_bold_cfg* cfg);
size_t wc_bold_state_doubles(const wc_bold_cfg* cfg, int64_t C);
int wc_bold_init(const wc_bold_cfg* cfg, int64_t C, double* state, void* stream);
/* E: float (e_f64 = 0) or double; e_ld == 0: time-major [Tc][C]; e_ld > 0:
 * node-major, sample tt of column c at E[c*e_ld + tt].
 * copy (optional, fp32 time-major E only): the chunk is also written
 * node-major, sample tt of column c at copy[c*copy_ld + tt] (copy_ld >= Tc;
 * 16-B row stores when copy is 16-B aligned and copy_ld % 4 == 0) -- the
 * transposition the Welch stage needs, done in the same pass as the BOLD
 * stream through an LDS tile with full-line stores.
 * NULL: no copy. */
int wc_bold_chunk(const wc_bold_cfg* cfg, int64_t C, const void* E, int e_f64, int64_t e_ld,
                  int64_t t0, int64_t Tc, double* state, void* copy, int64_t copy_ld, void* stream);
int wc_bold_finish(const wc_bold_cfg* cfg, int64_t C, const double* state, double* out, void* stream);

/* Hierarchical module analysis of B FC matrices, batched (run_many_seeds.py:
 * 130-133 over HMA.Functional_HP / Balance / nodal_measures, HMA.py:30-203).
 * fc [B][N][N] fp64 (N <= 96): read, then clipped in place (FC[FC < 0] = 0,
 * as HMA.py:55 does to the caller's matrix).  Outputs: hin[B], hse[B]
 * (Balance), hin_node[B][N], hse_node[B][N] (nodal_measures); optional
 * clus_num [B][N-1] int32 (Functional_HP's Clus_num) and sv [B][N] (singular
 * values of the symmetrised positive part, descending).  Eigen-decomposition
 * by cyclic Jacobi in LDS, one workgroup per matrix. */
int wc_hma(int B, int N, double* fc, double* hin, double* hse, double* hin_node, double* hse_node,
           int* clus_num, double* sv, void* stream);

/* The same outputs for any N >= 3 (N > 96: the matrix does not fit the Jacobi's
 * LDS) from the eigensystem of F = (max(FC,0) + max(FC,0)^T)/2 computed by the
 * caller on the device: lam [B][N] eigenvalues (any order), vt [B][N][N] with row
 * j the eigenvector of lam[j].  Ranks |lam| (stable, descending), walks the
 * levels (HMA.py:62-101), Balance and nodal_measures as wc_hma.  N <= 4096
 * (the label arrays take 40 B per node of the 160 KB LDS; larger N returns
 * WC_EUNSUPPORTED). */
int wc_hma_modes(int B, int N, const double* lam, const double* vt, double* hin, double* hse,
                 double* hin_node, double* hse_node, int* clus_num, double* sv, void* stream);

/* ------------------------------------------------------------------------
 * SC optimiser (optimize_SC_Hopf.py:47-104), SURVEY.md 8f rank 4.
 * The Hopf (Stuart-Landau) network of Hopf_model_multi.py:46-156, batched over
 * simulations (random seeds):
 *   x' = (a - x^2 - y^2) x - w y + sum_j (G M_ij / norm) (x_j - x_i)
 *   y' = (a - x^2 - y^2) y + w x + sum_j (G M_ij / norm) (y_j - y_i)
 *   state += f dt + beta z sqrt(dt)    (Euler-Maruyama, :143-144)
 * fp64.  Noise: the Philox stream above with the simulation key; node i's
 * (x, y) normals are the Box-Muller pair (2i, 2i+1), i.e. quad i/2.
 * x, y [B][N] in/out; when rec_every > 0, x BEFORE every local step s with
 * s % rec_every == 0 is stored at rec[s / rec_every][B][N] (and y at rec_y,
 * which may be NULL): a run recorded from its first step gives the
 * reference's results[k] = state after k*downsamp steps (:140-149).  M is N x N
 * (row i = inputs of node i); workspace >= wc_hopf_workspace_size(B, N): the
 * weight image and one segment (512 steps) of pre-generated normals. */
typedef struct wc_hopf_params {
    double a;     /* bifurcation parameter (Hopf_model_multi.py:22) */
    double w;     /* angular frequency, 0.05 * 2 pi (:23) */
    double beta;  /* noise scale (:25) */
    double dt;    /* Euler step (:28) */
    double G;     /* global coupling (:38; optimize_SC_Hopf.py:39) */
    double norm;  /* mean column sum of M (:37, optimize_SC_Hopf.py:30,101) */
} wc_hopf_params;

size_t wc_hopf_workspace_size(int B, int N);
int wc_hopf_integrate(const wc_hopf_params* p, int B, int N, const double* M, const uint64_t* keys,
                      double* x, double* y, int64_t step0, int64_t nsteps, int64_t rec_every,
                      double* rec, double* rec_y, void* workspace, size_t ws_bytes, void* stream);

/* scipy.signal.filtfilt(b, a, x, axis=0) of every column of x [T][C] fp64 ->
 * y [T][C] (y must not alias x): odd extension of padlen = 3 (order + 1),
 * lfilter_zi initial conditions zi[order] (host, from the caller), DF2T in
 * scipy's association order.  order in {2, 4, 6, 8}; b, a, zi are HOST
 * arrays of order + 1, order + 1 and order doubles, a[0] == 1.
 * (optimize_SC_Hopf.py:63-66; also any simBOLD-style band-pass.) */
int wc_filtfilt(int order, const double* b, const double* a, const double* zi, int64_t T, int64_t C,
                const double* x, double* y, void* stream);

/* Unit phasors exp(i angle(hilbert(x, axis=0))) of every column of x [M][C]
 * (utils.kuramoto, utils.py:35-37): phasor [M][C][2] (cos, sin).  workspace:
 * >= M doubles. */
int wc_hilbert_phase(int64_t C, int M, const double* x, double* phasor, void* workspace,
                     size_t ws_bytes, void* stream);

/* Per simulation b of bold [M][B][N] (the filtered, decimated BOLD; or, with
 * bold == NULL, of the given fc_in [B][N][N]):
 *   fc_out [B][N][N]  np.corrcoef(BOLD.T)                (may be NULL)
 *   metrics [B][K][4] utils.get_all_metrics(sFC, empfc[k], data_range) = corr, euc, ssim, new_metric
 *   extra [B][3]      np.mean(sFC), kuramoto sync, meta (sync/meta 0 if phasor NULL)
 * N >= 7 (the SSIM window).  N <= 96: one workgroup per simulation with the FC in
 * LDS, no workspace (may be NULL).  N > 96 (config 5, N = 1000): the FC is tiled
 * through global memory (wc_fc_large.hip) and workspace must hold
 * wc_fc_metrics_workspace_size(B, N, M, K, fc_out != NULL) bytes (it includes
 * the B N^2 doubles of FC when fc_out is NULL).  Deterministic for every N. */
size_t wc_fc_metrics_workspace_size(int B, int N, int M, int K, int want_fc);
int wc_fc_metrics(int B, int N, int M, const double* bold, const double* fc_in, const double* empfc,
                  int K, double data_range, const double* phasor, double* fc_out, double* metrics,
                  double* extra, void* workspace, size_t ws_bytes, void* stream);

/* np.corrcoef(x[:, b, :].T) for every simulation b of a long time-major series
 * x [M][B][N] (the SC optimiser's FC, optimize_SC_Hopf.py:67-69: 6000 samples),
 * split over time blocks so a small batch still fills the GPU; fc [B][N][N],
 * clipped to [-1, 1].  N >= 2, M >= 2 (N > 96: 64 x 64 covariance tiles in
 * global memory, wc_fc_large.hip).  Deterministic (fixed blocks, fixed combine
 * order).  workspace: wc_corrcoef_workspace_size(B, N, M) bytes. */
size_t wc_corrcoef_workspace_size(int B, int N, int M);
int wc_corrcoef(int B, int N, int M, const double* x, double* fc, void* workspace, size_t ws_bytes,
                void* stream);

/* utils.kuramoto (utils.py:34-40) from unit phasors [M][B][N][2] (wc_hilbert_phase):
 * out [B][2] = (mean_t R(t), std_t R(t)), R(t) = |mean_n exp(i theta_n(t))|. */
int wc_kuramoto(int B, int N, int M, const double* phasor, double* out, void* stream);

/* ------------------------------------------------------------------------
 * Welch peak frequency (whole_sweep_both.py:90-95): signal.welch(E_t.T, fs,
 * nperseg=4000), node-mean PSD, first argmax.  wc_welch_prepare fills the
 * twiddle workspace once; wc_welch_accumulate adds nseg (1, 2 or 4) consecutive segments
 * [seg0 + 2000 k, seg0 + 2000 k + 4000), k < nseg, of every column to acc [B][2001] (fp64, zero it
 * first; the ring must hold the nseg segments' span, 4000 + 2000 (nseg - 1) samples);
 * E is node-major: sample t of column c at
 *   c*ld + ((t / slot) % nslots) * slot + t % slot   (a ring of nslots slots);
 * wc_welch_peak turns acc (nseg segments) into peak [B] (Hz) and optionally
 * the node-mean density PSD psd [B][2001]. */
size_t wc_welch_workspace_size(void);
int wc_welch_bins(void);
int wc_welch_prepare(void* workspace, size_t ws_bytes, void* stream);
int wc_welch_accumulate(int B, int N, const void* E, int e_f64, int64_t ld, int64_t slot,
                        int64_t nslots, int64_t seg0, int nseg, const void* workspace, double* acc,
                        void* stream);
int wc_welch_peak(int B, int N, int nseg, double fs, const double* acc, double* peak, double* psd,
                  void* stream);

#ifdef __cplusplus
}
#endif

#endif /* WCSDE_H */
