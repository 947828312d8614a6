// wc_hma.hip -- hierarchical module analysis (integration / segregation) of a
// batch of FC matrices on gfx950.
//
// Replaces, for B simulations at once, the per-simulation host epilogue of
// run_many_seeds.py:130-133:
//   Clus_num, Clus_size, H_all = HMA.Functional_HP(sFC)      (HMA.py:30-103)
//   Hin, Hse = HMA.Balance(sFC, Clus_num, Clus_size)          (HMA.py:107-151)
//   Hin_node, Hse_node = HMA.nodal_measures(sFC, ...)         (HMA.py:155-203)
// Each of those clips FC < 0 to 0 in place, symmetrises and takes the SVD of the
// N x N result.  F = (F + F^T)/2 is symmetric, so its SVD is its eigensystem:
// singular values |lambda_i| in descending order, left singular vectors = the
// eigenvectors up to sign.  Every output is sign-invariant: Hin / Hse / nodal
// values use s^2 and u^2, and the module counts / sizes of a level are the
// classes of nodes with equal sign patterns over u_1..u_m, whatever the sign of
// each u_k (flipping u_k swaps the two halves of every split).
//
// One workgroup per matrix (N <= 96): F and the eigenvector matrix V live in
// LDS (2 x 96 x 96 fp64 = 144 KB), cyclic Jacobi with the round-robin
// (tournament) ordering: every round rotates N/2 disjoint (p, q) pairs in
// parallel (A <- J^T A J, V <- V J), N - 1 rounds per sweep, sweeps until the
// off-diagonal mass is below 1e-30 of the total.  Then the ranks of |lambda|
// (stable descending, as LAPACK's ordering), the level-by-level module labels
// (label <- 2 label + [u_m >= 0], compacted; HMA.py:62-101) and the sums.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "wc_common.h"

namespace {

constexpr int kMaxN = 96;
constexpr int kThreads = 256;
constexpr int kMaxSweeps = 30;

__global__ void __launch_bounds__(kThreads) hma_kernel(int N, double* __restrict__ fc, double* __restrict__ hin,
                                                       double* __restrict__ hse, double* __restrict__ hin_node,
                                                       double* __restrict__ hse_node, int* __restrict__ clus_num,
                                                       double* __restrict__ sv_out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int Np = N + (N & 1);  // even: a zero pad row/column (its rotations are identities)
    const int P = Np / 2;
    double* A = lds;              // [Np][Np]
    double* V = A + Np * Np;      // [Np][Np], V[k][j] = component k of eigenvector j
    double* cs = V + Np * Np;     // [P][2] (c, s) of this round
    double* lam = cs + 2 * P;     // [Np] eigenvalues
    double* red = lam + Np;       // [kThreads] reduction scratch
    double* hf = red + kThreads;  // [Np] HF (HMA.py:141)
    int* rank = reinterpret_cast<int*>(hf + Np);  // [Np] index of the mode with rank r
    int* lab = rank + Np;                         // [Np] module label of node k
    int* cnt = lab + Np;                          // [2 Np] module sizes of a level
    int* newid = cnt + 2 * Np;                    // [2 Np] compacted ids

    const int tid = threadIdx.x;
    double* F = fc + (size_t)blockIdx.x * N * N;

    // ---- F = (max(FC, 0) + max(FC, 0)^T) / 2, and the in-place clip of the caller's FC (HMA.py:55) ----
    for (int i = tid; i < Np * Np; i += kThreads) {
        const int r = i / Np, c = i % Np;
        double x = 0.0;
        if (r < N && c < N) {
            const double a = fmax(F[r * N + c], 0.0), b = fmax(F[c * N + r], 0.0);
            x = (a + b) / 2;
        }
        A[i] = x;
        V[i] = r == c ? 1.0 : 0.0;
    }
    __syncthreads();
    for (int i = tid; i < N * N; i += kThreads)
        if (F[i] < 0) F[i] = 0.0;  // every thread reads F before any writes it (barrier above)

    // ---- cyclic Jacobi, round-robin ordering ----
    for (int sweep = 0; sweep < kMaxSweeps; ++sweep) {
        // convergence: off-diagonal mass vs total (one reduction per sweep)
        double off = 0.0, tot = 0.0;
        for (int i = tid; i < Np * Np; i += kThreads) {
            const double x = A[i] * A[i];
            tot += x;
            if (i / Np != i % Np) off += x;
        }
        red[tid] = off;
        __syncthreads();
        for (int o = kThreads / 2; o > 0; o >>= 1) {
            if (tid < o) red[tid] += red[tid + o];
            __syncthreads();
        }
        const double offs = red[0];
        __syncthreads();
        red[tid] = tot;
        __syncthreads();
        for (int o = kThreads / 2; o > 0; o >>= 1) {
            if (tid < o) red[tid] += red[tid + o];
            __syncthreads();
        }
        const double tots = red[0];
        __syncthreads();
        if (!(offs > 1e-30 * tots)) break;  // uniform: every thread read the same sums

        for (int rnd = 0; rnd < Np - 1; ++rnd) {
            // pair k of round rnd: (rnd, Np-1) for k = 0, ((rnd+k) mod (Np-1), (rnd-k) mod (Np-1)) otherwise
            if (tid < P) {
                const int k = tid, m = Np - 1;
                int p = k == 0 ? rnd : (rnd + k) % m;
                int q = k == 0 ? m : (rnd - k + m) % m;
                if (p > q) { const int t = p; p = q; q = t; }
                const double apq = A[p * Np + q];
                double c = 1.0, s = 0.0;
                if (apq != 0.0) {
                    const double app = A[p * Np + p], aqq = A[q * Np + q];
                    const double th = (aqq - app) / (2.0 * apq);
                    const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
                    c = 1.0 / sqrt(fma(t, t, 1.0));
                    s = t * c;
                }
                cs[2 * k] = c;
                cs[2 * k + 1] = s;
            }
            __syncthreads();
            // columns p, q of A and V: A <- A J, V <- V J
            for (int i = tid; i < P * Np; i += kThreads) {
                const int k = i / Np, row = i % Np, m = Np - 1;
                int p = k == 0 ? rnd : (rnd + k) % m;
                int q = k == 0 ? m : (rnd - k + m) % m;
                if (p > q) { const int t = p; p = q; q = t; }
                const double c = cs[2 * k], s = cs[2 * k + 1];
                const double ap = A[row * Np + p], aq = A[row * Np + q];
                A[row * Np + p] = c * ap - s * aq;
                A[row * Np + q] = s * ap + c * aq;
                const double vp = V[row * Np + p], vq = V[row * Np + q];
                V[row * Np + p] = c * vp - s * vq;
                V[row * Np + q] = s * vp + c * vq;
            }
            __syncthreads();
            // rows p, q of A: A <- J^T A
            for (int i = tid; i < P * Np; i += kThreads) {
                const int k = i / Np, col = i % Np, m = Np - 1;
                int p = k == 0 ? rnd : (rnd + k) % m;
                int q = k == 0 ? m : (rnd - k + m) % m;
                if (p > q) { const int t = p; p = q; q = t; }
                const double c = cs[2 * k], s = cs[2 * k + 1];
                const double ap = A[p * Np + col], aq = A[q * Np + col];
                A[p * Np + col] = c * ap - s * aq;
                A[q * Np + col] = s * ap + c * aq;
            }
            __syncthreads();
        }
    }

    // ---- singular values = |lambda|, ranked descending (stable in the index); the pad is last ----
    for (int i = tid; i < Np; i += kThreads) lam[i] = i < N ? fabs(A[i * Np + i]) : -1.0;
    __syncthreads();
    for (int i = tid; i < Np; i += kThreads) {
        const double li = lam[i];
        int r = 0;
        for (int j = 0; j < Np; ++j) r += (lam[j] > li) || (lam[j] == li && j < i);
        rank[r] = i;
    }
    __syncthreads();

    // ---- hierarchical modules, level by level (one wave; HMA.py:62-101) ----
    // level 0: one module of N nodes; level m >= 1: nodes split by the signs of u_1..u_m
    // (HMA.py:63-64 / :81-82 use u >= 0 vs u < 0).  Clus_num[m] = modules of level m,
    // p[m] = sum |size - N / Clus_num[m]| / N (HMA.py:136-138), for m = 0 .. N-3.
    if (tid < 64) {
        for (int k = tid; k < Np; k += 64) lab[k] = 0;
        int C = 1;  // modules at the current level (labels 0..C-1)
        for (int m = 0; m <= N - 2; ++m) {
            // module sizes of level m (labels are compact)
            for (int j = tid; j < C; j += 64) cnt[j] = 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            for (int k = tid; k < N; k += 64) atomicAdd(&cnt[lab[k]], 1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            double pm = 0.0;
            for (int j = tid; j < C; j += 64) pm += fabs((double)cnt[j] - (double)N / C);
            for (int o = 32; o > 0; o >>= 1) pm += __shfl_xor(pm, o);
            if (tid == 0) {
                const double sm = lam[rank[m]];
                // HF = s^2 Clus_num (1 - p); p[N-2] is never set by the reference (stays 0)
                hf[m] = sm * sm * C * (1.0 - (m < N - 2 ? pm / N : 0.0));
                if (clus_num) clus_num[(size_t)blockIdx.x * (N - 1) + m] = C;
            }
            if (m == N - 2) break;
            // split every module by the sign of u_{m+1}; compact the 2C candidate labels
            const int um = rank[m + 1];
            for (int j = tid; j < 2 * C; j += 64) cnt[j] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int k = tid; k < N; k += 64) {
                lab[k] = 2 * lab[k] + (V[k * Np + um] >= 0.0 ? 1 : 0);
                atomicOr(&cnt[lab[k]], 1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (tid == 0) {
                int nc = 0;
                for (int j = 0; j < 2 * C; ++j) {
                    newid[j] = nc;
                    nc += cnt[j];
                }
                C = nc;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            C = __shfl(C, 0);
            for (int k = tid; k < N; k += 64) lab[k] = newid[lab[k]];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();

    // ---- Balance (HMA.py:140-144) and nodal_measures (HMA.py:193-201) ----
    const double N2 = (double)N * N;
    if (tid < 64) {
        double s = 0.0;
        for (int m = 1 + tid; m <= N - 2; m += 64) s += hf[m];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (tid == 0) {
            hin[blockIdx.x] = hf[0] / N2;
            hse[blockIdx.x] = s / N2;
        }
    }
    for (int k = tid; k < N; k += kThreads) {
        const double u0 = V[k * Np + rank[0]];
        hin_node[(size_t)blockIdx.x * N + k] = hf[0] / N * u0 * u0;
        double s = 0.0;
        for (int m = 1; m <= N - 2; ++m) {
            const double um = V[k * Np + rank[m]];
            s += hf[m] / N * um * um;
        }
        hse_node[(size_t)blockIdx.x * N + k] = s;
    }
    if (sv_out)
        for (int m = tid; m < N; m += kThreads) sv_out[(size_t)blockIdx.x * N + m] = lam[rank[m]];
}

// ---- N > 96: the module / Balance / nodal stages from a given eigensystem ----
// lam [N] eigenvalues and vt [N][N] (row j = eigenvector j) of F = (max(FC,0) + max(FC,0)^T)/2,
// from a batched library eigensolver on the device (the matrix no longer fits LDS for the Jacobi
// above).  Same ranking, levels and sums as hma_kernel; the eigenvector rows are read from
// global memory (coalesced: one row per level).  Compaction of a level's 2C candidate labels is
// a wave-wide ballot scan instead of a serial loop (C grows to N).
__global__ void __launch_bounds__(kThreads) hma_modes_kernel(int N, const double* __restrict__ lam_in,
                                                             const double* __restrict__ vt_all,
                                                             double* __restrict__ hin, double* __restrict__ hse,
                                                             double* __restrict__ hin_node,
                                                             double* __restrict__ hse_node, int* __restrict__ clus_num,
                                                             double* __restrict__ sv_out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* lam = lds;                                // [N] |lambda|
    double* hf = lam + N;                             // [N]
    int* rank = reinterpret_cast<int*>(hf + N);       // [N]
    int* lab = rank + N;                              // [N]
    int* flag = lab + N;                              // [2N]
    int* newid = flag + 2 * N;                        // [2N]
    const int tid = threadIdx.x;
    const size_t b = blockIdx.x;
    const double* vt = vt_all + b * (size_t)N * N;
    for (int i = tid; i < N; i += kThreads) lam[i] = fabs(lam_in[b * N + i]);
    __syncthreads();
    for (int i = tid; i < N; i += kThreads) {
        const double li = lam[i];
        int r = 0;
        for (int j = 0; j < N; ++j) r += (lam[j] > li) || (lam[j] == li && j < i);
        rank[r] = i;
    }
    __syncthreads();
    if (tid < 64) {
        for (int k = tid; k < N; k += 64) lab[k] = 0;
        int C = 1;
        for (int m = 0; m <= N - 2; ++m) {
            for (int j = tid; j < C; j += 64) flag[j] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int k = tid; k < N; k += 64) atomicAdd(&flag[lab[k]], 1);  // module sizes of level m
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double pm = 0.0;
            for (int j = tid; j < C; j += 64) pm += fabs((double)flag[j] - (double)N / C);
            for (int o = 32; o > 0; o >>= 1) pm += __shfl_xor(pm, o);
            if (tid == 0) {
                const double sm = lam[rank[m]];
                hf[m] = sm * sm * C * (1.0 - (m < N - 2 ? pm / N : 0.0));  // HMA.py:141-147 (p[N-2] stays 0)
                if (clus_num) clus_num[b * (N - 1) + m] = C;
            }
            if (m == N - 2) break;
            const double* u = vt + (size_t)rank[m + 1] * N;
            for (int j = tid; j < 2 * C; j += 64) flag[j] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int k = tid; k < N; k += 64) {
                const int l = 2 * lab[k] + (u[k] >= 0.0 ? 1 : 0);  // HMA.py:78-82: u >= 0 vs u < 0
                lab[k] = l;
                flag[l] = 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int run = 0;  // exclusive scan of the non-empty flags: compact ids in candidate order
            for (int base = 0; base < 2 * C; base += 64) {
                const int j = base + tid;
                const bool f = j < 2 * C && flag[j] != 0;
                const uint64_t mask = __ballot(f);
                if (j < 2 * C) newid[j] = run + __popcll(mask & ((1ull << tid) - 1ull));
                run += __popcll(mask);
            }
            C = run;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int k = tid; k < N; k += 64) lab[k] = newid[lab[k]];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
    const double N2 = (double)N * N;
    if (tid < 64) {
        double s = 0.0;
        for (int m = 1 + tid; m <= N - 2; m += 64) s += hf[m];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (tid == 0) {
            hin[b] = hf[0] / N2;
            hse[b] = s / N2;
        }
    }
    // nodal measures (HMA.py:193-201): row rank[m] of vt is u_m, read coalesced per level
    for (int k0 = 0; k0 < N; k0 += kThreads) {
        const int k = k0 + tid;
        if (k >= N) break;
        const double u0 = vt[(size_t)rank[0] * N + k];
        hin_node[b * N + k] = hf[0] / N * u0 * u0;
        double s = 0.0;
        for (int m = 1; m <= N - 2; ++m) {
            const double um = vt[(size_t)rank[m] * N + k];
            s += hf[m] / N * um * um;
        }
        hse_node[b * N + k] = s;
    }
    if (sv_out)
        for (int m = tid; m < N; m += kThreads) sv_out[b * N + m] = lam[rank[m]];
}

size_t hma_modes_lds_bytes(int N) { return sizeof(double) * 2 * (size_t)N + sizeof(int) * 6 * (size_t)N; }

size_t hma_lds_bytes(int N) {
    const int Np = N + (N & 1), P = Np / 2;
    return sizeof(double) * (2 * (size_t)Np * Np + 2 * P + Np + kThreads + Np) + sizeof(int) * (2 * Np + 4 * Np);
}

}  // namespace

extern "C" {

int wc_hma(int B, int N, double* fc, double* hin, double* hse, double* hin_node, double* hse_node, int* clus_num,
           double* sv, void* stream) {
    wc_clear_err();
    if (B <= 0 || N < 3 || !fc || !hin || !hse || !hin_node || !hse_node)
        return wc_set_err(WC_EINVAL, "wc_hma: bad B/N or NULL output");
    if (N > kMaxN) return wc_set_err(WC_EUNSUPPORTED, "wc_hma: N > 96 (F and V must fit in LDS)");
    const size_t lds = hma_lds_bytes(N);
    hipError_t e = hipFuncSetAttribute((const void*)hma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    hipLaunchKernelGGL(hma_kernel, dim3(B), dim3(kThreads), lds, static_cast<hipStream_t>(stream), N, fc, hin, hse,
                       hin_node, hse_node, clus_num, sv);
    return wc_hip_check("wc_hma");
}

int wc_hma_modes(int B, int N, const double* lam, const double* vt, double* hin, double* hse, double* hin_node,
                 double* hse_node, int* clus_num, double* sv, void* stream) {
    wc_clear_err();
    if (B <= 0 || N < 3 || !lam || !vt || !hin || !hse || !hin_node || !hse_node)
        return wc_set_err(WC_EINVAL, "wc_hma_modes: bad B/N or NULL argument");
    const size_t lds = hma_modes_lds_bytes(N);
    if (lds > 160 * 1024) return wc_set_err(WC_EUNSUPPORTED, "wc_hma_modes: N too large for the LDS label arrays");
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)hma_modes_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(hma_modes_kernel, dim3(B), dim3(kThreads), lds, static_cast<hipStream_t>(stream), N, lam, vt,
                       hin, hse, hin_node, hse_node, clus_num, sv);
    return wc_hip_check("wc_hma_modes");
}

}  // extern "C"
