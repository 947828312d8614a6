/*
 * wc_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * This file is the checker for the HIP product path, never the product path
 * itself.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it (see oracle/__init__.py).  It is a plain-C, fp64 restatement of
 * the reference hot loop:
 *
 *   S(x, sigma, mu)            netwWilsonCowanPlastic.py:72-74
 *   wilsonCowan(t, X, ...)     netwWilsonCowanPlastic.py:77-83
 *   run()  (3 Euler phases)    netwWilsonCowanPlastic.py:86-137
 *
 * with the reference's numba RNG (seeded from os.urandom, never reproducible:
 * SURVEY.md 8c) replaced by the build's deterministic noise stream:
 *
 *   Philox4x32-10 (Salmon et al., SC'11 "Parallel random numbers: as easy as
 *   1, 2, 3"; Random123 constants) with the fixed key (WC_PHILOX_KEY0/1 of
 *   include/wcsde.h) and counter = (step lo32, (step hi16 << 16) | quad,
 *   simkey lo32, simkey hi32) for global Euler step `step`, node quad
 *   q = node/4 and the 64-bit per-simulation key.
 *   The four 32-bit outputs feed two Box-Muller pairs:
 *     u = (2*(x >> 9) + 1) * 2^-24           (exact in fp32 and fp64, in (0,1))
 *     z0 = sqrt(-2 ln u1) cos(2 pi u2),  z1 = sqrt(-2 ln u1) sin(2 pi u2)
 *   giving the standard normals of nodes 4q+0..4q+3 (pairs (x0,x1), (x2,x3)).
 *   noise = sqdtD * z  ==  np.random.normal(0, sqdtD, N)   (wc:80)
 *
 * Parity status: the arithmetic of S/wilsonCowan/run is restated line by line
 * (cited above) and pinned to the reference's OWN run(): tests/golden/
 * make_ref_replay.py executes /root/reference/netwWilsonCowanPlastic.py with its
 * numba decorators as identities and np.random.normal replaying this Philox
 * stream; tests/test_oracle_ref_replay.py checks this loop
 * against that Y_t at <= 1e-13 (observed 3e-15: np.dot/np.exp rounding).  Over
 * the full 1001 s schedule it is also pinned statistically to the reference's
 * shipped sweep tables (tests/test_oracle_pin.py, tests/golden/oracle_pin_cell.json).
 * BOLD (orc_bold) remains unpinned: BOLDModel is absent from the reference.
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct orc_params {
    double a_ee, a_ei, a_ii;   /* wc:23-25 */
    double tauE, tauI;         /* wc:27 */
    double P, rhoE;            /* wc:29, wc:32 (drivers: P=0.4, rhoE=0.18) */
    double rE, rI, mu, sigmaI; /* wc:35-38 */
    double sqdtD;              /* wc:57  D/sqrt(dtSim) */
    double dtSim;              /* wc:45 */
} orc_params;

/* ---------------- Philox4x32-10 ---------------- */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += PH_W0; k1 += PH_W1; }
        uint64_t p0 = (uint64_t)PH_M0 * c0;
        uint64_t p1 = (uint64_t)PH_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline double u01(uint32_t x) { return (double)(2u * (x >> 9) + 1u) * (1.0 / 16777216.0); }

static const double TWO_PI = 6.283185307179586476925286766559;

/* standard normals of the 4 nodes of quad q at global step `step` */
static inline void quad_normals(uint64_t key, int64_t step, uint32_t q, double z[4])
{
    const uint64_t st = (uint64_t)step;
    uint32_t ctr[4] = {(uint32_t)st, ((uint32_t)(st >> 32) << 16) | q, (uint32_t)key, (uint32_t)(key >> 32)};
    uint32_t k[2] = {0x243F6A88u, 0x85A308D3u};  /* WC_PHILOX_KEY0/1 */
    uint32_t x[4];
    orc_philox4x32_10(ctr, k, x);
    double r0 = sqrt(-2.0 * log(u01(x[0])));
    double r1 = sqrt(-2.0 * log(u01(x[2])));
    double a0 = TWO_PI * u01(x[1]);
    double a1 = TWO_PI * u01(x[3]);
    z[0] = r0 * cos(a0);
    z[1] = r0 * sin(a0);
    z[2] = r1 * cos(a1);
    z[3] = r1 * sin(a1);
}

/* the N standard normals of one simulation at one step (exported for tests) */
void orc_step_normals(uint64_t key, int64_t step, int N, double* z)
{
    double zz[4];
    for (int q = 0; 4 * q < N; ++q) {
        quad_normals(key, step, (uint32_t)q, zz);
        for (int r = 0; r < 4 && 4 * q + r < N; ++r) z[4 * q + r] = zz[r];
    }
}

/*
 * Advance one simulation by nsteps Euler-Maruyama steps (wc:101-135).
 * State E, I, A (= a_ie) are in/out, length N.  The Philox counter of local
 * step s is step0 + s.  When rec_every > 0, the state BEFORE the update of
 * every local step s with s % rec_every == 0 is stored at row s / rec_every of
 * recE/recI/recA (row-major [n_rec][N]; any of them may be NULL) -- wc:124-125.
 */
int orc_wc_integrate(const orc_params* p, int N, const double* sc, const double* G,
                     const double* sigmaE, uint64_t key, double* E, double* I, double* A,
                     int64_t step0, int64_t nsteps, double tau_ip, int64_t rec_every,
                     double* recE, double* recI, double* recA)
{
    if (N <= 0 || N > 4096) return -1;
    double coup[4096], z[4096 + 4], nE[4096], nI[4096];
    for (int64_t s = 0; s < nsteps; ++s) {
        if (rec_every > 0 && s % rec_every == 0) {
            int64_t k = s / rec_every;
            if (recE) memcpy(recE + k * N, E, sizeof(double) * N);
            if (recI) memcpy(recI + k * N, I, sizeof(double) * N);
            if (recA) memcpy(recA + k * N, A, sizeof(double) * N);
        }
        const int64_t gstep = step0 + s;
        for (int q = 0; 4 * q < N; ++q) quad_normals(key, gstep, (uint32_t)q, z + 4 * q);
        /* np.dot(CM, E)  (wc:81) */
        for (int i = 0; i < N; ++i) {
            const double* row = sc + (size_t)i * N;
            double acc = 0.0;
            for (int j = 0; j < N; ++j) acc += row[j] * E[j];
            coup[i] = acc;
        }
        for (int i = 0; i < N; ++i) {
            const double e = E[i], in = I[i], a = A[i];
            const double noise = p->sqdtD * z[i];
            /* wc:81  a_ee*E - a_ie*I + G*CM@E + P + noise, then S(., sigmaE, mu) */
            const double xE = p->a_ee * e - a * in + G[i] * coup[i] + p->P + noise;
            const double SE = 1.0 / (1.0 + exp(-(xE - p->mu) * sigmaE[i]));
            const double dE = (-e + (1.0 - p->rE * e) * SE) / p->tauE;
            /* wc:82 */
            const double xI = p->a_ei * e - p->a_ii * in;
            const double SI = 1.0 / (1.0 + exp(-(xI - p->mu) * p->sigmaI));
            const double dI = (-in + (1.0 - p->rI * in) * SI) / p->tauI;
            /* wc:83 */
            const double dA = (in * (e - p->rhoE)) / tau_ip;
            nE[i] = e + p->dtSim * dE;
            nI[i] = in + p->dtSim * dI;
            A[i] = a + p->dtSim * dA;
        }
        memcpy(E, nE, sizeof(double) * N);
        memcpy(I, nI, sizeof(double) * N);
    }
    return 0;
}

/* Batched form: B independent simulations, parallel over sims (one thread per
 * sim, mirroring the reference's one-process-per-simulation SLURM array).
 * G, sigmaE, E, I, A are [B][N]; recE is [B][n_rec][N] (may be NULL). */
int orc_wc_integrate_batch(const orc_params* p, int B, int N, const double* sc, const double* G,
                           const double* sigmaE, const uint64_t* keys, double* E, double* I,
                           double* A, int64_t step0, int64_t nsteps, double tau_ip,
                           int64_t rec_every, double* recE, int nthreads)
{
    int64_t n_rec = rec_every > 0 ? (nsteps + rec_every - 1) / rec_every : 0;
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int b = 0; b < B; ++b) {
        size_t o = (size_t)b * N;
        err |= orc_wc_integrate(p, N, sc, G + o, sigmaE + o, keys[b], E + o, I + o, A + o, step0,
                                nsteps, tau_ip, rec_every,
                                recE ? recE + (size_t)b * n_rec * N : NULL, NULL, NULL);
    }
    (void)nthreads;
    return err ? -1 : 0;
}

/* ---------------- Hopf network (SC optimiser) ----------------
 * Restates Hopf_model_multi.py:46-59 (Hopf_model), :63-69 (Noise) and the
 * Euler-Maruyama update of Sim (:143-144, results_temp += f dt + noise sqrt(dt)):
 *   Isyn_i = sum_j (G * M_ij / norm) * (x_j - x_i)            (:49-53)
 *   x' = (a - x^2 - y^2) x - w y + IsynX,  y' = (a - x^2 - y^2) y + w x + IsynY
 * with the numba RNG replaced by the Philox stream (node i's (x, y) normals =
 * Box-Muller pair (2i, 2i+1) = quad i/2).  x BEFORE local step s is stored at
 * rec[s / rec_every] when s % rec_every == 0.  Parity status: the reference
 * module needs numba and networkx (absent), so it is pinned by the analytic
 * noise-free solution (tests/test_oracle_hopf.py), not by running it. */
typedef struct orc_hopf_params { double a, w, beta, dt, G, norm; } orc_hopf_params;

int orc_hopf_integrate(const orc_hopf_params* p, int N, const double* M, uint64_t key, double* x, double* y,
                       int64_t step0, int64_t nsteps, int64_t rec_every, double* rec)
{
    if (N <= 0 || N > 4096) return -1;
    static const int kMax = 4096;
    double nx[kMax], ny[kMax], z[kMax + 4];
    const double sqdt = sqrt(p->dt);
    for (int64_t s = 0; s < nsteps; ++s) {
        if (rec_every > 0 && s % rec_every == 0) memcpy(rec + (s / rec_every) * N, x, sizeof(double) * N);
        for (int q = 0; 2 * q < N; ++q) quad_normals(key, step0 + s, (uint32_t)q, z + 4 * q);
        for (int i = 0; i < N; ++i) {
            double cx = 0.0, cy = 0.0;
            for (int j = 0; j < N; ++j) {
                const double m = p->G * M[(size_t)i * N + j] / p->norm;
                cx += m * (x[j] - x[i]);
                cy += m * (y[j] - y[i]);
            }
            const double r = p->a - x[i] * x[i] - y[i] * y[i];
            const double fx = r * x[i] - p->w * y[i] + cx;
            const double fy = r * y[i] + p->w * x[i] + cy;
            nx[i] = x[i] + (fx * p->dt + (z[2 * i] * p->beta) * sqdt);
            ny[i] = y[i] + (fy * p->dt + (z[2 * i + 1] * p->beta) * sqdt);
        }
        memcpy(x, nx, sizeof(double) * N);
        memcpy(y, ny, sizeof(double) * N);
    }
    return 0;
}

/* B simulations (x, y [B][N], rec [B][n_rec][N] or NULL), parallel over sims */
int orc_hopf_integrate_batch(const orc_hopf_params* p, int B, int N, const double* M, const uint64_t* keys,
                             double* x, double* y, int64_t step0, int64_t nsteps, int64_t rec_every, double* rec)
{
    const int64_t n_rec = rec_every > 0 ? (nsteps + rec_every - 1) / rec_every : 0;
    int err = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int b = 0; b < B; ++b)
        err |= orc_hopf_integrate(p, N, M, keys[b], x + (size_t)b * N, y + (size_t)b * N, step0, nsteps,
                                  rec_every, rec ? rec + (size_t)b * n_rec * N : NULL);
    return err ? -1 : 0;
}

/* Balloon-Windkessel BOLD (assumed form of the missing BOLDModel.BD.Sim, see
 * DESIGN.md "BOLD model"): Euler at dt per E sample, y0 = (s,f,v,q) = (0,1,1,1),
 * BOLD[t] computed from the state after t steps.  rE is [T][N]; out is [T][N]. */
void orc_bold(const double* rE, int64_t T, int N, double dt, double* out)
{
    const double itaus = 1.0 / 0.65, itauf = 1.0 / 0.41, itauo = 1.0 / 0.98;
    const double ialpha = 1.0 / 0.32, Eo = 0.4, vo = 0.04;
    const double k1 = 7.0 * Eo, k2 = 2.0, k3 = 2.0 * Eo - 0.2;
    for (int n = 0; n < N; ++n) {
        double s = 0.0, f = 1.0, v = 1.0, q = 1.0;
        for (int64_t t = 0; t < T; ++t) {
            out[t * N + n] = vo * (k1 * (1.0 - q) + k2 * (1.0 - q / v) + k3 * (1.0 - v));
            const double x = rE[t * N + n];
            const double vpow = pow(v, ialpha);
            const double ds = x - itaus * s - itauf * (f - 1.0);
            const double df = s;
            const double dv = (f - vpow) * itauo;
            const double dq = (f * (1.0 - pow(1.0 - Eo, 1.0 / f)) / Eo - q * vpow / v) * itauo;
            s += dt * ds; f += dt * df; v += dt * dv; q += dt * dq;
        }
    }
}

/* Direct-form-II-transposed IIR (scipy.signal.lfilter semantics, a[0] == 1),
 * fp64, over n samples of each of m independent columns of x ([n][m] row-major).
 * zi [order][m] in/out (final state), y [n][m]. */
void orc_lfilter(const double* b, const double* a, int order, const double* x, int64_t n, int m,
                 double* zi, double* y)
{
    for (int c = 0; c < m; ++c) {
        double z[16];
        for (int k = 0; k < order; ++k) z[k] = zi[(size_t)k * m + c];
        for (int64_t i = 0; i < n; ++i) {
            const double xi = x[(size_t)i * m + c];
            /* association order of scipy's lfilter.c (z + x*b - y*a): the narrow
             * band-pass is ill-conditioned, so rounding order shows at ~1e-9 */
            const double yi = z[0] + xi * b[0];
            for (int k = 0; k < order - 1; ++k) z[k] = z[k + 1] + xi * b[k + 1] - yi * a[k + 1];
            z[order - 1] = xi * b[order] - yi * a[order];
            y[(size_t)i * m + c] = yi;
        }
        for (int k = 0; k < order; ++k) zi[(size_t)k * m + c] = z[k];
    }
}
