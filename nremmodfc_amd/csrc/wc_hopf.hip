// wc_hopf.hip -- the SC optimiser's Hopf (Stuart-Landau) network SDE and a
// batched filtfilt, on gfx950.
//
// Replaces, for a batch of random seeds at once, the inner loop of
// optimize_SC_Hopf.py:52-71:
//   HM.Sim()                 Hopf_model_multi.py:79-156 (Hopf_model :46-59,
//                            Noise :63-69): Euler-Maruyama of
//     x' = (a - x^2 - y^2) x - w y + G/norm sum_j M_ij (x_j - x_i)
//     y' = (a - x^2 - y^2) y + w x + G/norm sum_j M_ij (y_j - y_i)
//     state += f dt + beta N(0,1) sqrt(dt)      (independent normals for x, y)
//   signal.filtfilt(b, a, x, axis=0)            optimize_SC_Hopf.py:63-66
//     (order-2K IIR, odd extension of padlen = 3 max(len(a), len(b)),
//      lfilter_zi initial conditions: the published SciPy algorithm).
//
// Hopf layout: one workgroup per simulation, four lanes per node (N <= 256); x, y in
// registers for the whole launch, G M / norm transposed in LDS (conflict-free
// column reads), the node states exchanged through a double-buffered LDS image
// (one barrier per step).  Noise: the build's Philox4x32-10 stream
// (include/wcsde.h), node i's (x, y) normals = the Box-Muller pair 2i, 2i+1 of
// the simulation's stream, i.e. quad i/2.
//
// filtfilt layout: one thread per column of a time-major [T][C] array (every
// access coalesced across the wave); the forward pass writes its output in
// place of y, keeps the padlen outputs of the back extension in registers and
// runs the backward pass over them and then over y in reverse.  DF2T in SciPy's
// association order with FMA contraction off: the same arithmetic as
// scipy.signal.lfilter.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "wc_common.h"
#include "wc_device.h"

namespace {

constexpr int kHopfMaxN = 1024;
constexpr int kHopfLdsN = 128;  // G M / norm in LDS up to N = 128 (128 KB), else read from global (L2)

struct HopfArgs {
    double a, w, beta, dt, sqdt;
    const double* mg;  // workspace: G M_ij / norm, transposed: mg[j*N + i]
    const uint64_t* keys;
    double* x;
    double* y;
    double* rec;
    double* rec_y;
    int64_t step0, nsteps, rec_every;
    int B, N;
};

// G * M / norm (Hopf_model_multi.py:52-53 evaluates G * M / norm elementwise), transposed
__global__ void hopf_weights_kernel(const double* __restrict__ M, int N, double G, double norm, double* __restrict__ mg) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * N) return;
    const int j = idx / N, i = idx % N;
    mg[idx] = G * M[(size_t)i * N + j] / norm;
}

// LPN lanes per node (adjacent lanes): lane q of node i sums j = q, q + LPN, ...; two
// xor-shuffles combine the partial sums (commutative: every lane gets the same bits),
// and every lane then carries the same x, y; lane 0 publishes and records.
template <bool LDS, int LPN>
__global__ void __launch_bounds__(kHopfMaxN) hopf_kernel(const HopfArgs p) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int N = p.N;
    const int i = threadIdx.x / LPN, q = threadIdx.x % LPN;
    const int b = blockIdx.x;
    const bool live = i < N;
    const bool lead = live && q == 0;
    double* xs = sm + (LDS ? (size_t)N * N : 0);  // [2][N]
    double* ys = xs + 2 * N;                     // [2][N]
    const double* mg = p.mg;
    if constexpr (LDS) {
        double* l = sm;
        for (int k = threadIdx.x; k < N * N; k += blockDim.x) l[k] = p.mg[k];
        mg = l;
    }
    const int ii = live ? i : N - 1;  // tail lanes shadow the last node, never store
    double x = p.x[(size_t)b * N + ii];
    double y = p.y[(size_t)b * N + ii];
    const uint64_t key = p.keys[b];
    const double a = p.a, w = p.w, dt = p.dt, bs = p.beta;
    for (int64_t s = 0; s < p.nsteps; ++s) {
        const int buf = (int)(s & 1);
        if (p.rec_every > 0 && s % p.rec_every == 0 && lead) {
            const int64_t o = ((s / p.rec_every) * p.B + b) * (int64_t)N + i;
            p.rec[o] = x;
            if (p.rec_y) p.rec_y[o] = y;
        }
        if (lead) {
            xs[buf * N + i] = x;
            ys[buf * N + i] = y;
        }
        // the step's normals do not depend on the state: drawn before the barrier wait
        double z[4];
        wcdev::quad_normals((uint64_t)(p.step0 + s), (uint32_t)(ii >> 1), key, z);
        __syncthreads();  // also orders the LDS weight image before the first step
        // Isyn_i = sum_j (G M_ij / norm) (x_j - x_i)    (Hopf_model_multi.py:49-53)
        double cx = 0.0, cy = 0.0;
        const double* xb = xs + buf * N;
        const double* yb = ys + buf * N;
        for (int j = q; j < N; j += LPN) {
            const double m = mg[(size_t)j * N + ii];
            cx += m * (xb[j] - x);
            cy += m * (yb[j] - y);
        }
#pragma unroll
        for (int o = 1; o < LPN; o <<= 1) {
            cx += __shfl_xor(cx, o);
            cy += __shfl_xor(cy, o);
        }
        const double zx = z[2 * (ii & 1)], zy = z[2 * (ii & 1) + 1];
        const double r = a - x * x - y * y;
        const double fx = r * x - w * y + cx;   // Hopf_model_multi.py:55
        const double fy = r * y + w * x + cy;   // :56
        // results_temp += Hopf_model(...) * dt + Noise(...) * sqrt(dt)   (:143-144)
        x += fx * dt + (zx * bs) * p.sqdt;
        y += fy * dt + (zy * bs) * p.sqdt;
    }
    if (lead) {
        p.x[(size_t)b * N + i] = x;
        p.y[(size_t)b * N + i] = y;
    }
}

// ---------------- batched filtfilt ----------------
struct FiltArgs {
    double b[9], a[9], zi[8];
    const double* x;
    double* y;
    int64_t T, C;
};

#pragma clang fp contract(off)
template <int K>
__device__ __forceinline__ double df2t(double z[K], double x, const FiltArgs& f) {
    const double y = z[0] + x * f.b[0];
#pragma unroll
    for (int k = 0; k < K - 1; ++k) z[k] = z[k + 1] + x * f.b[k + 1] - y * f.a[k + 1];
    z[K - 1] = x * f.b[K] - y * f.a[K];
    return y;
}

// K = filter order (len(a) - 1), padlen = 3 (K + 1) (scipy.signal.filtfilt's default)
template <int K>
__global__ void __launch_bounds__(256) filtfilt_kernel(const FiltArgs f) {
    constexpr int PL = 3 * (K + 1);
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= f.C) return;
    const int64_t C = f.C, T = f.T;
    const double* __restrict__ x = f.x + c;
    double* __restrict__ y = f.y + c;
    double z[K];
    // odd extension in front: ext[k] = 2 x0 - x[PL - k], k = 0..PL-1; zi * ext[0]
    const double x0 = x[0];
    const double e0 = 2.0 * x0 - x[PL * C];
#pragma unroll
    for (int k = 0; k < K; ++k) z[k] = f.zi[k] * e0;
    for (int k = 0; k < PL; ++k) df2t<K>(z, 2.0 * x0 - x[(PL - k) * C], f);
    // main samples in batches of 16: the batch's loads are issued together (one
    // latency per batch instead of one per sample: the recursion itself is short)
    int64_t t = 0;
    for (; t + 16 <= T; t += 16) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = x[(t + k) * C];
#pragma unroll
        for (int k = 0; k < 16; ++k) y[(t + k) * C] = df2t<K>(z, v[k], f);
    }
    for (; t < T; ++t) y[t * C] = df2t<K>(z, x[t * C], f);
    // odd extension at the end: 2 x[T-1] - x[T-2-k], k = 0..PL-1 (outputs kept for the backward pass)
    const double xl = x[(T - 1) * C];
    double yt[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) yt[k] = df2t<K>(z, 2.0 * xl - x[(T - 2 - k) * C], f);
    // backward pass from the end of the extended forward output, zi * its last value
#pragma unroll
    for (int k = 0; k < K; ++k) z[k] = f.zi[k] * yt[PL - 1];
#pragma unroll
    for (int k = PL - 1; k >= 0; --k) df2t<K>(z, yt[k], f);
    t = T - 1;
    for (; t >= 15; t -= 16) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = y[(t - k) * C];
#pragma unroll
        for (int k = 0; k < 16; ++k) y[(t - k) * C] = df2t<K>(z, v[k], f);
    }
    for (; t >= 0; --t) y[t * C] = df2t<K>(z, y[t * C], f);
}
#pragma clang fp contract(on)

}  // namespace

extern "C" {

size_t wc_hopf_workspace_size(int N) { return N > 0 ? (size_t)N * N * sizeof(double) : 0; }

int wc_hopf_integrate(const wc_hopf_params* hp, int B, int N, const double* M, const uint64_t* keys, double* x,
                      double* y, int64_t step0, int64_t nsteps, int64_t rec_every, double* rec, double* rec_y,
                      void* workspace, size_t ws_bytes, void* stream) {
    wc_clear_err();
    if (!hp || B <= 0 || N <= 0 || nsteps < 0 || step0 < 0 || step0 + nsteps > (int64_t(1) << 48) || rec_every < 0 ||
        !M || !keys || !x || !y || (rec_every > 0 && !rec))
        return wc_set_err(WC_EINVAL, "wc_hopf_integrate: bad arguments");
    if (N > kHopfMaxN) return wc_set_err(WC_EUNSUPPORTED, "wc_hopf_integrate: N > 1024");
    if (!workspace || ws_bytes < wc_hopf_workspace_size(N))
        return wc_set_err(WC_EWORKSPACE, "wc_hopf_integrate: workspace too small");
    if (!(hp->norm != 0.0) || !(hp->dt > 0.0)) return wc_set_err(WC_EINVAL, "wc_hopf_integrate: norm == 0 or dt <= 0");
    if (nsteps == 0) return WC_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    double* mg = static_cast<double*>(workspace);
    hipLaunchKernelGGL(hopf_weights_kernel, dim3((N * N + 255) / 256), dim3(256), 0, st, M, N, hp->G, hp->norm, mg);
    HopfArgs p;
    p.a = hp->a; p.w = hp->w; p.beta = hp->beta; p.dt = hp->dt; p.sqdt = sqrt(hp->dt);
    p.mg = mg; p.keys = keys; p.x = x; p.y = y; p.rec = rec; p.rec_y = rec_y;
    p.step0 = step0; p.nsteps = nsteps; p.rec_every = rec_every; p.B = B; p.N = N;
    // 4 lanes per node while 4N threads fit one workgroup (N <= 256), else 1
    const int lpn = N <= kHopfMaxN / 4 ? 4 : 1;
    const int threads = ((lpn * N + 63) / 64) * 64;
    const bool lds = N <= kHopfLdsN;
    const size_t bytes = ((lds ? (size_t)N * N : 0) + 4 * (size_t)N) * sizeof(double);
    auto kern = lds ? (lpn == 4 ? hopf_kernel<true, 4> : hopf_kernel<true, 1>)
                    : (lpn == 4 ? hopf_kernel<false, 4> : hopf_kernel<false, 1>);
    if (bytes > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(kern, dim3(B), dim3(threads), bytes, st, p);
    return wc_hip_check("wc_hopf_integrate");
}

int wc_filtfilt(int order, const double* b, const double* a, const double* zi, int64_t T, int64_t C, const double* x,
                double* y, void* stream) {
    wc_clear_err();
    if (!b || !a || !zi || !x || !y || C <= 0 || x == y)
        return wc_set_err(WC_EINVAL, "wc_filtfilt: NULL pointer, C <= 0 or y aliasing x");
    if (order != 2 && order != 4 && order != 6 && order != 8)
        return wc_set_err(WC_EUNSUPPORTED, "wc_filtfilt: order must be 2, 4, 6 or 8");
    if (T <= 3 * (order + 1)) return wc_set_err(WC_EINVAL, "wc_filtfilt: T must exceed padlen = 3 (order + 1)");
    if (a[0] != 1.0) return wc_set_err(WC_EINVAL, "wc_filtfilt: a[0] must be 1");
    FiltArgs f = {};
    for (int k = 0; k <= order; ++k) {
        f.b[k] = b[k];
        f.a[k] = a[k];
    }
    for (int k = 0; k < order; ++k) f.zi[k] = zi[k];
    f.x = x; f.y = y; f.T = T; f.C = C;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((C + 255) / 256));
    switch (order) {
        case 2: hipLaunchKernelGGL(filtfilt_kernel<2>, grid, dim3(256), 0, st, f); break;
        case 4: hipLaunchKernelGGL(filtfilt_kernel<4>, grid, dim3(256), 0, st, f); break;
        case 6: hipLaunchKernelGGL(filtfilt_kernel<6>, grid, dim3(256), 0, st, f); break;
        default: hipLaunchKernelGGL(filtfilt_kernel<8>, grid, dim3(256), 0, st, f); break;
    }
    return wc_hip_check("wc_filtfilt");
}

}  // extern "C"
