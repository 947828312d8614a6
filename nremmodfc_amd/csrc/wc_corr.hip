// wc_corr.hip -- np.corrcoef of long series for a small batch, split over time.
//
// Replaces the FC of the SC optimiser's inner loop (optimize_SC_Hopf.py:67-69:
// np.corrcoef(x[cut0:cut1].T) per seed, 6000 samples x 90 nodes, 10 seeds). One
// workgroup per simulation (wc_fc_metrics) keeps 10 CUs busy; here every
// simulation's series is cut into time blocks so that B x nblk workgroups share the
// work, in four stream-ordered launches:
//   1. block sums of every node            -> part[b][k][n]
//   2. means (block sums in block order), centred cross products of the block as
//      4 x 4 register tiles of the upper triangle -> covp[b][k][i][j] (i <= j)
//   3. sum over blocks in block order, 1/(M-1), corrcoef scaling and [-1, 1] clip
//      (standard deviations first, then one workgroup per row).
// Two-pass (np.cov centres before multiplying), deterministic: fixed block sizes
// and a fixed combine order, independent of the launch's scheduling.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "wc_common.h"

// N > 96: wc_fc_large.hip (FC tiles in global memory)
size_t wc_large_corrcoef_workspace_size(int B, int N);
int wc_large_corrcoef(int B, int N, int M, const double* x, double* fc, void* workspace, size_t ws_bytes,
                      hipStream_t st);

namespace {

constexpr int kThreads = 256;
constexpr int kMaxN = 96;
constexpr int kMinBlock = 64;  // samples per time block at least

struct CorrGeo {
    int nblk, tb;  // blocks per simulation, samples per block (the last may be shorter)
};

CorrGeo corr_geo(int B, int M) {
    CorrGeo g;
    int nb = (2 * 256 + B - 1) / B;  // ~2 workgroups per CU over the batch
    nb = nb < 1 ? 1 : nb;
    const int most = (M + kMinBlock - 1) / kMinBlock;
    nb = nb > most ? most : nb;
    g.tb = (M + nb - 1) / nb;
    g.nblk = (M + g.tb - 1) / g.tb;
    return g;
}

size_t part_doubles(int B, int N, const CorrGeo& g) { return (size_t)B * g.nblk * N; }

// 1. part[b][k][n] = sum over the block's samples (time order) of x[t][b][n]
__global__ void __launch_bounds__(kThreads) block_sum_kernel(int B, int N, int M, int tb, int nblk,
                                                             const double* __restrict__ x, double* __restrict__ part) {
    const int b = blockIdx.x / nblk, k = blockIdx.x % nblk;
    const int t0 = k * tb, t1 = min(M, t0 + tb);
    const int64_t C = (int64_t)B * N;
    for (int n = threadIdx.x; n < N; n += kThreads) {
        double s = 0.0;
        for (int t = t0; t < t1; ++t) s += x[(int64_t)t * C + (int64_t)b * N + n];
        part[((int64_t)b * nblk + k) * N + n] = s;
    }
}

// 2. the block's centred cross products, upper-triangle 4 x 4 tiles
__global__ void __launch_bounds__(kThreads) block_cov_kernel(int B, int N, int M, int tb, int nblk,
                                                             const double* __restrict__ x,
                                                             const double* __restrict__ part,
                                                             double* __restrict__ covp) {
    __shared__ __attribute__((aligned(16))) double mean[kMaxN];
    __shared__ __attribute__((aligned(16))) double stage[64 * kMaxN];  // 64 samples x Np
    const int b = blockIdx.x / nblk, k = blockIdx.x % nblk;
    const int t0 = k * tb, t1 = min(M, t0 + tb);
    const int tid = threadIdx.x;
    const int64_t C = (int64_t)B * N;
    for (int n = tid; n < N; n += kThreads) {
        double s = 0.0;
        for (int q = 0; q < nblk; ++q) s += part[((int64_t)b * nblk + q) * N + n];
        mean[n] = s / M;
    }
    __syncthreads();
    const int Np = (N + 3) & ~3, NB = Np / 4;
    const int ntiles = NB * (NB + 1) / 2;  // <= 300 for N <= 96: at most 2 per thread
    constexpr int kT = ((kMaxN / 4) * (kMaxN / 4 + 1) / 2 + kThreads - 1) / kThreads;
    double acc[kT][4][4];
    int ti[kT], tj[kT];
#pragma unroll
    for (int u = 0; u < kT; ++u) {
        const int p = min(tid + u * kThreads, ntiles - 1);
        int bi = 0, rem = p;
        while (rem >= NB - bi) {  // row-major over the upper triangle of NB x NB tiles
            rem -= NB - bi;
            ++bi;
        }
        ti[u] = 4 * bi;
        tj[u] = 4 * (bi + rem);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[u][r][q] = 0.0;
    }
    for (int s0 = t0; s0 < t1; s0 += 64) {
        const int tn = min(64, t1 - s0);
        for (int i = tid; i < tn * Np; i += kThreads) {
            const int tt = i / Np, n = i % Np;
            stage[i] = n < N ? x[(int64_t)(s0 + tt) * C + (int64_t)b * N + n] - mean[n] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kT; ++u) {
            if (tid + u * kThreads < ntiles) {
                for (int tt = 0; tt < tn; ++tt) {
                    const double2* row = reinterpret_cast<const double2*>(stage + tt * Np);
                    const double2 a0 = row[ti[u] / 2], a1 = row[ti[u] / 2 + 1];
                    const double2 b0 = row[tj[u] / 2], b1 = row[tj[u] / 2 + 1];
                    const double xi[4] = {a0.x, a0.y, a1.x, a1.y}, xj[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[u][r][q] += xi[r] * xj[q];
                }
            }
        }
        __syncthreads();
    }
    double* out = covp + ((int64_t)b * nblk + k) * N * N;
#pragma unroll
    for (int u = 0; u < kT; ++u) {
        if (tid + u * kThreads < ntiles) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = ti[u] + r, j = tj[u] + q;
                    if (i < N && j < N && i <= j) out[i * N + j] = acc[u][r][q];
                }
        }
    }
}

// 3a. sd[b][n] = sqrt(cov_nn) from the summed blocks
__global__ void __launch_bounds__(kThreads) corr_sd_kernel(int B, int N, int M, int nblk,
                                                           const double* __restrict__ covp, double* __restrict__ sd) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= B * N) return;
    const int b = i / N, n = i % N;
    const int64_t NN = (int64_t)N * N;
    const double* cb = covp + (int64_t)b * nblk * NN + n * N + n;
    double s = 0.0;
    for (int q = 0; q < nblk; ++q) s += cb[q * NN];
    sd[i] = sqrt(s * (1.0 / (M - 1)));
}

// 3b. row i of fc[b] (np.corrcoef: c / sd_i / sd_j, clipped), one workgroup per (b, i):
// the blocks hold the upper triangle, summed in block order for j >= i and mirrored
__global__ void __launch_bounds__(128) corr_row_kernel(int N, int M, int nblk, const double* __restrict__ covp,
                                                       const double* __restrict__ sd, double* __restrict__ fc) {
    const int b = blockIdx.x / N, i = blockIdx.x % N;
    const int64_t NN = (int64_t)N * N;
    const double* cb = covp + (int64_t)b * nblk * NN + (int64_t)i * N;
    const double* sdb = sd + (int64_t)b * N;
    const double fact = 1.0 / (M - 1);
    for (int j = i + threadIdx.x; j < N; j += 128) {
        double s = 0.0;
        for (int q = 0; q < nblk; ++q) s += cb[q * NN + j];
        double v = (s * fact) / sdb[i];
        v = v / sdb[j];
        v = fmin(1.0, fmax(-1.0, v));
        fc[(int64_t)b * NN + (int64_t)i * N + j] = v;
        if (j != i) {  // np.corrcoef: c[j][i] / sd_j / sd_i (division order as numpy, not mirrored bits)
            double w = (s * fact) / sdb[j];
            w = w / sdb[i];
            fc[(int64_t)b * NN + (int64_t)j * N + i] = fmin(1.0, fmax(-1.0, w));
        }
    }
}

}  // namespace

extern "C" {

size_t wc_corrcoef_workspace_size(int B, int N, int M) {
    if (B <= 0 || N <= 0 || M <= 0) return 0;
    if (N > kMaxN) return wc_large_corrcoef_workspace_size(B, N);
    const CorrGeo g = corr_geo(B, M);
    return (part_doubles(B, N, g) + (size_t)B * g.nblk * N * N + (size_t)B * N) * sizeof(double);
}

int wc_corrcoef(int B, int N, int M, const double* x, double* fc, void* workspace, size_t ws_bytes, void* stream) {
    wc_clear_err();
    if (B <= 0 || N < 2 || M < 2 || !x || !fc)
        return wc_set_err(WC_EINVAL, "wc_corrcoef: needs B >= 1, N >= 2, M >= 2 and non-NULL x, fc");
    if (N > kMaxN) return wc_large_corrcoef(B, N, M, x, fc, workspace, ws_bytes, static_cast<hipStream_t>(stream));
    if (!workspace || ws_bytes < wc_corrcoef_workspace_size(B, N, M))
        return wc_set_err(WC_EWORKSPACE, "wc_corrcoef: workspace too small");
    const CorrGeo g = corr_geo(B, M);
    if ((int64_t)B * g.nblk > INT32_MAX) return wc_set_err(WC_EUNSUPPORTED, "wc_corrcoef: grid too large");
    double* part = static_cast<double*>(workspace);
    double* covp = part + part_doubles(B, N, g);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)(B * g.nblk));
    hipLaunchKernelGGL(block_sum_kernel, grid, dim3(kThreads), 0, st, B, N, M, g.tb, g.nblk, x, part);
    hipLaunchKernelGGL(block_cov_kernel, grid, dim3(kThreads), 0, st, B, N, M, g.tb, g.nblk, x, part, covp);
    double* sd = covp + (size_t)B * g.nblk * N * N;
    hipLaunchKernelGGL(corr_sd_kernel, dim3((unsigned)((B * N + kThreads - 1) / kThreads)), dim3(kThreads), 0, st, B,
                       N, M, g.nblk, covp, sd);
    hipLaunchKernelGGL(corr_row_kernel, dim3((unsigned)(B * N)), dim3(128), 0, st, N, M, g.nblk, covp, sd, fc);
    return wc_hip_check("wc_corrcoef");
}

}  // extern "C"
