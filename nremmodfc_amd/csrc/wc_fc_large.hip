// wc_fc_large.hip -- FC (np.corrcoef), goodness of fit and mean(FC) for N > 96.
//
// The N <= 96 kernels (wc_fc_metrics_kernel, wc_corr.hip) hold a simulation's
// whole N x N FC in one workgroup's LDS.  At N = 1000 (BASELINE config 5) the FC is
// 8 MB per simulation, so it lives in global memory and the work is tiled:
//
//   1. node means over time                  one thread per column, time order
//   2. centred cross products, 64 x 64 tiles of the upper triangle, one workgroup
//      per (tile, simulation); every (i, j) sums its samples in time order
//      (np.cov: x - mean, then the dot product, then 1/(M-1))      -> cov, sd
//   3. np.corrcoef: c / sd_i / sd_j and c / sd_j / sd_i (numpy's division order
//      for the two triangles), clipped to [-1, 1]; one workgroup per row
//   4. get_all_metrics vs each empirical FC (utils.py:42-50) and mean(FC)
//      (whole_sweep_both.py:94): per-(band of rows) partial sums in a fixed thread
//      mapping, combined in band order -- deterministic, no atomics:
//        a. sum FC, upper-triangle sums of FC and of each empFC
//        b. centred upper-triangle sums (Pearson), squared differences (L2) and
//           the SSIM map (7 x 7 uniform window, cov_norm 49/48, crop 3) of each k
//        c. one thread per simulation: combine the bands, write metrics/extra.
// FC and the partials are HBM-bound (the FC is written once and read once per
// empirical FC); the cov tiles are fp64-FMA-bound (M N^2 / 2 FMAs per simulation).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "wc_common.h"

namespace {

constexpr int kT = 64;      // cov tile edge
constexpr int kTC = 16;     // samples per LDS stage
constexpr int kRows = 8;    // FC rows per gof band
constexpr int kThreads = 256;

__device__ double wg_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    double s = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    __syncthreads();
    return s;
}

// 1. mean[c] = sum_t x[t][c] / M  (c = b*N + n)
__global__ void __launch_bounds__(kThreads) mean_kernel(int64_t C, int M, const double* __restrict__ x,
                                                        double* __restrict__ mean) {
    const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c >= C) return;
    double s = 0.0;
    for (int t = 0; t < M; ++t) s += x[(int64_t)t * C + c];
    mean[c] = s / M;
}

// 2. cov[b][i][j] (i <= j, upper triangle only) = sum_t xc[t][i] xc[t][j] / (M-1); sd[b][i] = sqrt(cov_ii)
// grid (NB (NB+1)/2, B); thread (ty, tx) of 16 x 16 owns rows i0+4ty.., columns j0+4tx..
__global__ void __launch_bounds__(kThreads) cov_tile_kernel(int B, int N, int M, const double* __restrict__ x,
                                                            const double* __restrict__ mean,
                                                            double* __restrict__ cov, double* __restrict__ sd) {
    __shared__ __attribute__((aligned(16))) double As[2][kTC][kT];
    __shared__ __attribute__((aligned(16))) double Bs[2][kTC][kT];
    const int NB = (N + kT - 1) / kT;
    const int b = blockIdx.y;
    int bi = 0, rem = blockIdx.x;
    while (rem >= NB - bi) {  // row-major over the upper triangle of NB x NB tiles
        rem -= NB - bi;
        ++bi;
    }
    const int bj = bi + rem;
    const int i0 = bi * kT, j0 = bj * kT;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int64_t C = (int64_t)B * N;
    const double* xb = x + (int64_t)b * N;
    const double* mb = mean + (int64_t)b * N;
    // staging: element e = tid + 256 k of a (kTC x 64) stage is (tt = e / 64, n = e % 64): 64 consecutive nodes
    constexpr int kPer = kTC * kT / kThreads;  // 4
    double ma[kPer], mbv[kPer];
    bool oka[kPer], okb[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int n = (tid + kThreads * k) & (kT - 1);
        oka[k] = i0 + n < N;
        okb[k] = j0 + n < N;
        ma[k] = oka[k] ? mb[i0 + n] : 0.0;
        mbv[k] = okb[k] ? mb[j0 + n] : 0.0;
    }
    double ra[kPer], rb[kPer];
    auto load = [&](int t0) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int e = tid + kThreads * k, tt = e / kT, n = e & (kT - 1);
            const int t = t0 + tt;
            ra[k] = (oka[k] && t < M) ? xb[(int64_t)t * C + i0 + n] - ma[k] : 0.0;
            rb[k] = (okb[k] && t < M) ? xb[(int64_t)t * C + j0 + n] - mbv[k] : 0.0;
        }
    };
    auto store = [&](int st) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int e = tid + kThreads * k, tt = e / kT, n = e & (kT - 1);
            As[st][tt][n] = ra[k];
            Bs[st][tt][n] = rb[k];
        }
    };
    double acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = 0.0;
    load(0);
    store(0);
    __syncthreads();
    const int nst = (M + kTC - 1) / kTC;
    for (int s = 0; s < nst; ++s) {
        const int cur = s & 1;
        if (s + 1 < nst) load((s + 1) * kTC);  // next stage's loads in flight during this stage's FMAs
        const int tn = min(kTC, M - s * kTC);
        for (int tt = 0; tt < tn; ++tt) {  // time order for every (i, j)
            const double2 a0 = *reinterpret_cast<const double2*>(&As[cur][tt][4 * ty]);
            const double2 a1 = *reinterpret_cast<const double2*>(&As[cur][tt][4 * ty + 2]);
            const double2 b0 = *reinterpret_cast<const double2*>(&Bs[cur][tt][4 * tx]);
            const double2 b1 = *reinterpret_cast<const double2*>(&Bs[cur][tt][4 * tx + 2]);
            const double xi[4] = {a0.x, a0.y, a1.x, a1.y}, xj[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[r][q] += xi[r] * xj[q];
        }
        if (s + 1 < nst) store(cur ^ 1);
        __syncthreads();
    }
    const double fact = 1.0 / (M - 1);
    double* cb = cov + (int64_t)b * N * N;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + 4 * ty + r, j = j0 + 4 * tx + q;
            if (i < N && j < N && i <= j) {
                const double c = acc[r][q] * fact;
                cb[(int64_t)i * N + j] = c;
                if (i == j) sd[(int64_t)b * N + i] = sqrt(c);
            }
        }
}

// 3. row i of simulation b: upper entries read, both triangles written (in place)
__global__ void __launch_bounds__(128) corr_norm_kernel(int N, const double* __restrict__ sd, double* __restrict__ fc) {
    const int64_t bi = blockIdx.x;
    const int64_t b = bi / N;
    const int i = (int)(bi % N);
    const int64_t NN = (int64_t)N * N;
    double* f = fc + b * NN;
    const double* s = sd + b * N;
    const double si = s[i];
    for (int j = i + threadIdx.x; j < N; j += 128) {
        const double c = f[(int64_t)i * N + j];
        double v = c / si;
        v = v / s[j];
        f[(int64_t)i * N + j] = fmin(1.0, fmax(-1.0, v));
        if (j != i) {
            double w = c / s[j];
            w = w / si;
            f[(int64_t)j * N + i] = fmin(1.0, fmax(-1.0, w));
        }
    }
}

// 4a. per band: [0] sum of all FC entries, [1] upper-triangle sum of FC, [2 + k] of empFC k
__global__ void __launch_bounds__(kThreads) gof_sums_kernel(int N, int K, int nbands, const double* __restrict__ fc,
                                                            const double* __restrict__ emp, double* __restrict__ part) {
    __shared__ double red[kThreads / 64];
    const int band = blockIdx.x, b = blockIdx.y;
    const int r0 = band * kRows, r1 = min(N, r0 + kRows);
    const int64_t NN = (int64_t)N * N;
    const double* f = fc + (int64_t)b * NN;
    double sall = 0, sx = 0;
    for (int r = r0; r < r1; ++r)
        for (int q = threadIdx.x; q < N; q += kThreads) {
            const double v = f[(int64_t)r * N + q];
            sall += v;
            if (q > r) sx += v;
        }
    double* o = part + ((int64_t)b * nbands + band) * (2 + K);
    sall = wg_sum(sall, red);
    sx = wg_sum(sx, red);
    if (threadIdx.x == 0) {
        o[0] = sall;
        o[1] = sx;
    }
    for (int k = 0; k < K; ++k) {
        const double* e = emp + (int64_t)k * NN;
        double sy = 0;
        for (int r = r0; r < r1; ++r)
            for (int q = r + 1 + threadIdx.x; q < N; q += kThreads) sy += e[(int64_t)r * N + q];
        sy = wg_sum(sy, red);
        if (threadIdx.x == 0) o[2 + k] = sy;
    }
}

// 4b. per band and k: sxx, syy, sxy, see (upper triangle, centred on the flat means) and the SSIM sum
// of the interior pixels whose row is in the band (same arithmetic as the N <= 96 kernel)
__global__ void __launch_bounds__(kThreads) gof_centred_kernel(int N, int K, int nbands, double data_range,
                                                               const double* __restrict__ fc,
                                                               const double* __restrict__ emp,
                                                               const double* __restrict__ part1,
                                                               double* __restrict__ part2) {
    __shared__ double red[kThreads / 64];
    const int band = blockIdx.x, b = blockIdx.y;
    const int r0 = band * kRows, r1 = min(N, r0 + kRows);
    const int64_t NN = (int64_t)N * N;
    const double* f = fc + (int64_t)b * NN;
    const double nflat = (double)N * (N - 1) / 2;
    const double C1 = (0.01 * data_range) * (0.01 * data_range), C2 = (0.03 * data_range) * (0.03 * data_range);
    const double cov_norm = 49.0 / 48.0;
    // flat means: the band partial sums in band order
    double sx = 0;
    for (int q = 0; q < nbands; ++q) sx += part1[((int64_t)b * nbands + q) * (2 + K) + 1];
    const double mx = sx / nflat;
    for (int k = 0; k < K; ++k) {
        const double* e = emp + (int64_t)k * NN;
        double sy = 0;
        for (int q = 0; q < nbands; ++q) sy += part1[((int64_t)b * nbands + q) * (2 + K) + 2 + k];
        const double my = sy / nflat;
        double sxx = 0, syy = 0, sxy = 0, see = 0;
        for (int r = r0; r < r1; ++r)
            for (int q = r + 1 + threadIdx.x; q < N; q += kThreads) {
                const double xv = f[(int64_t)r * N + q], yv = e[(int64_t)r * N + q];
                const double dx = xv - mx, dy = yv - my, de = yv - xv;
                sxx += dx * dx;
                syy += dy * dy;
                sxy += dx * dy;
                see += de * de;
            }
        double ssum = 0;
        const int ia = max(r0, 3), ib = min(r1, N - 3);
        for (int i = ia; i < ib; ++i)
            for (int j = 3 + threadIdx.x; j < N - 3; j += kThreads) {
                double vx = 0, vy = 0, vxx = 0, vyy = 0, vxy = 0;
                for (int di = -3; di <= 3; ++di) {
                    const int64_t ro = (int64_t)(i + di) * N;
                    double hx = 0, hy = 0, hxx = 0, hyy = 0, hxy = 0;
                    for (int dj = -3; dj <= 3; ++dj) {
                        const double xv = f[ro + j + dj], yv = e[ro + j + dj];
                        hx += xv;
                        hy += yv;
                        hxx += xv * xv;
                        hyy += yv * yv;
                        hxy += xv * yv;
                    }
                    vx += hx / 7.0;
                    vy += hy / 7.0;
                    vxx += hxx / 7.0;
                    vyy += hyy / 7.0;
                    vxy += hxy / 7.0;
                }
                const double ux = vx / 7.0, uy = vy / 7.0, uxx = vxx / 7.0, uyy = vyy / 7.0, uxy = vxy / 7.0;
                const double sx2 = cov_norm * (uxx - ux * ux), sy2 = cov_norm * (uyy - uy * uy),
                             sxy2 = cov_norm * (uxy - ux * uy);
                const double A1 = 2 * ux * uy + C1, A2 = 2 * sxy2 + C2;
                const double B1 = ux * ux + uy * uy + C1, B2 = sx2 + sy2 + C2;
                ssum += (A1 * A2) / (B1 * B2);
            }
        sxx = wg_sum(sxx, red);
        syy = wg_sum(syy, red);
        sxy = wg_sum(sxy, red);
        see = wg_sum(see, red);
        ssum = wg_sum(ssum, red);
        if (threadIdx.x == 0) {
            double* o = part2 + (((int64_t)b * nbands + band) * K + k) * 5;
            o[0] = sxx;
            o[1] = syy;
            o[2] = sxy;
            o[3] = see;
            o[4] = ssum;
        }
    }
}

// 4c. one thread per simulation: combine the bands in order
__global__ void gof_final_kernel(int B, int N, int K, int nbands, const double* __restrict__ part1,
                                 const double* __restrict__ part2, const double* __restrict__ kur,
                                 double* __restrict__ metrics, double* __restrict__ extra) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const double nflat = (double)N * (N - 1) / 2;
    double sall = 0, sx = 0;
    for (int q = 0; q < nbands; ++q) {
        sall += part1[((int64_t)b * nbands + q) * (2 + K)];
        sx += part1[((int64_t)b * nbands + q) * (2 + K) + 1];
    }
    const double mx = sx / nflat;
    const double P = N - 6;
    for (int k = 0; k < K; ++k) {
        double sy = 0, s[5] = {0, 0, 0, 0, 0};
        for (int q = 0; q < nbands; ++q) {
            sy += part1[((int64_t)b * nbands + q) * (2 + K) + 2 + k];
            const double* o = part2 + (((int64_t)b * nbands + q) * K + k) * 5;
            for (int m = 0; m < 5; ++m) s[m] += o[m];
        }
        const double my = sy / nflat;
        const double f1 = 1.0 / (nflat - 1);
        double corr = (s[2] * f1) / sqrt(s[0] * f1) / sqrt(s[1] * f1);
        corr = fmin(1.0, fmax(-1.0, corr));
        double* o = metrics + ((int64_t)b * K + k) * 4;
        o[0] = corr;
        o[1] = sqrt(s[3]);
        o[2] = s[4] / (P * P);
        o[3] = 1.0 - corr + (mx - my) * (mx - my);
    }
    extra[(int64_t)b * 3 + 0] = sall / ((double)N * N);
    extra[(int64_t)b * 3 + 1] = kur ? kur[2 * b] : 0.0;
    extra[(int64_t)b * 3 + 2] = kur ? kur[2 * b + 1] : 0.0;
}

__global__ void copy_kernel(int64_t n, const double* __restrict__ src, double* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

int nbands_for(int N) { return (N + kRows - 1) / kRows; }

// np.corrcoef of every simulation of time-major x [M][B][N] -> fc [B][N][N]; ws: mean + sd (2 B N doubles)
int large_fc(int B, int N, int M, const double* x, double* fc, double* ws, hipStream_t st) {
    const int64_t C = (int64_t)B * N;
    double* mean = ws;
    double* sd = ws + C;
    const int NB = (N + kT - 1) / kT;
    if (B > 65535) return wc_set_err(WC_EUNSUPPORTED, "large FC: B > 65535");
    hipLaunchKernelGGL(mean_kernel, dim3((unsigned)((C + kThreads - 1) / kThreads)), dim3(kThreads), 0, st, C, M, x,
                       mean);
    hipLaunchKernelGGL(cov_tile_kernel, dim3((unsigned)(NB * (NB + 1) / 2), (unsigned)B), dim3(kThreads), 0, st, B, N,
                       M, x, mean, fc, sd);
    hipLaunchKernelGGL(corr_norm_kernel, dim3((unsigned)C), dim3(128), 0, st, N, sd, fc);
    return WC_OK;
}

size_t fc_ws_doubles(int B, int N, int K, bool own_fc) {
    const size_t C = (size_t)B * N;
    return 2 * C + (own_fc ? C * N : 0) + (size_t)B * nbands_for(N) * (2 + K + 5 * K);
}

}  // namespace

// ---- internal entry points (wc_corr.hip, wc_signal.hip dispatch here for N > 96) ----
size_t wc_large_corrcoef_workspace_size(int B, int N) { return 2 * (size_t)B * N * sizeof(double); }

int wc_large_corrcoef(int B, int N, int M, const double* x, double* fc, void* workspace, size_t ws_bytes,
                      hipStream_t st) {
    if (!workspace || ws_bytes < wc_large_corrcoef_workspace_size(B, N))
        return wc_set_err(WC_EWORKSPACE, "wc_corrcoef: workspace too small");
    const int rc = large_fc(B, N, M, x, fc, static_cast<double*>(workspace), st);
    return rc ? rc : wc_hip_check("wc_corrcoef (N > 96)");
}

size_t wc_large_fc_metrics_workspace_size(int B, int N, int K, int own_fc) {
    return fc_ws_doubles(B, N, K, own_fc != 0) * sizeof(double);
}

// kuramoto(B, N, M, phasor, out) is launched by the caller into kur (may be NULL)
int wc_large_fc_metrics(int B, int N, int M, const double* bold, const double* fc_in, const double* empfc, int K,
                        double data_range, const double* kur, double* fc_out, double* metrics, double* extra,
                        void* workspace, size_t ws_bytes, hipStream_t st) {
    const bool own = fc_out == nullptr;
    if (!workspace || ws_bytes < wc_large_fc_metrics_workspace_size(B, N, K, own))
        return wc_set_err(WC_EWORKSPACE, "wc_fc_metrics: workspace too small for N > 96 "
                                         "(wc_fc_metrics_workspace_size)");
    double* ws = static_cast<double*>(workspace);
    const size_t C = (size_t)B * N;
    double* fc = own ? ws + 2 * C : fc_out;
    double* part1 = ws + 2 * C + (own ? C * N : 0);
    const int nb = nbands_for(N);
    double* part2 = part1 + (size_t)B * nb * (2 + K);
    if (B > 65535) return wc_set_err(WC_EUNSUPPORTED, "wc_fc_metrics: B > 65535 for N > 96");
    if (bold) {
        const int rc = large_fc(B, N, M, bold, fc, ws, st);
        if (rc) return rc;
    } else {
        const int64_t n = (int64_t)C * N;
        hipLaunchKernelGGL(copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, fc_in, fc);
    }
    const dim3 grid((unsigned)nb, (unsigned)B);
    hipLaunchKernelGGL(gof_sums_kernel, grid, dim3(kThreads), 0, st, N, K, nb, fc, empfc, part1);
    if (K > 0)
        hipLaunchKernelGGL(gof_centred_kernel, grid, dim3(kThreads), 0, st, N, K, nb, data_range, fc, empfc, part1,
                           part2);
    hipLaunchKernelGGL(gof_final_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, B, N, K, nb, part1, part2,
                       kur, metrics, extra);
    return wc_hip_check("wc_fc_metrics (N > 96)");
}
