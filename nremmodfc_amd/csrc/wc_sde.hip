// wc_sde.hip -- batched Wilson-Cowan Euler-Maruyama integrator for gfx950.
//
// Replaces the numba hot loop of netwWilsonCowanPlastic.py (wilsonCowan
// wc:77-83, run wc:86-137) for a whole batch of (G, sigmaE, seed) simulations.
//
// Layout (DESIGN.md "Kernel 1"): one wave64 integrates 16 simulations.  Lane
// l = 16*g + j owns simulation j of the wave and, for every 16-node tile t,
// the four nodes 16t + 4g + r (r = 0..3) -- E, I, a_ie live in registers for
// the whole launch.  That register layout is simultaneously
//   * the C/D layout of the coupling MFMA  D[node][sim] = CM . E^T  and
//   * the B-operand layout of the next step's MFMA (k-step (t, r) feeds
//     register (t, r) of every lane),
// so the dense SC@E contraction moves no data between lanes, LDS or HBM:
// the matrix pipe is the data movement.  The connectome is the A operand,
// pre-arranged once per launch in an LDS fragment image (conflict-free
// ds_read_b128, one 16-B chunk per lane per (out tile, k tile)).
//   fp32: v_mfma_f32_16x16x4_f32 (exact f32 fma chain)
//   fp64: v_mfma_f64_16x16x4_f64 (C/D rows permuted by sigma(rho), below)
// The elementwise update (two logistic sigmoids, plasticity, Philox4x32-10
// noise + Box-Muller) runs on the VALU between the MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../include/wcsde.h"

namespace {

thread_local char g_err[512];
int set_err(int code, const char* msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
    return code;
}

constexpr int kWaves = 4;              // waves per workgroup
constexpr int kSimsPerWave = 16;
constexpr int kSimsPerBlock = kWaves * kSimsPerWave;
constexpr int kMaxTiles = 6;           // N <= 96 on the register-resident path

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// ---------------- Philox4x32-10 (must match oracle/wc_oracle.c) ----------------
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// u = (2*(x>>9)+1) * 2^-24, exact in fp32/fp64, in (0,1)
__device__ __forceinline__ float u01f(uint32_t x) { return (float)(2u * (x >> 9) + 1u) * 5.9604644775390625e-8f; }
__device__ __forceinline__ double u01d(uint32_t x) { return (double)(2u * (x >> 9) + 1u) * 5.9604644775390625e-8; }

// Box-Muller normals of nodes 4q..4q+3 -- fp32 hardware transcendentals
__device__ __forceinline__ void quad_normals(uint32_t s_lo, uint32_t s_hi, uint32_t q, uint32_t k0,
                                             uint32_t k1, float z[4]) {
    uint32_t x[4];
    philox4x32_10(s_lo, s_hi, q, 0u, k0, k1, x);
    // ln(u) = log2(u) * ln2 ; v_sin/v_cos take revolutions: sin(2*pi*u)
    const float r0 = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01f(x[0])));
    const float r1 = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01f(x[2])));
    const float a0 = u01f(x[1]), a1 = u01f(x[3]);
    z[0] = r0 * __builtin_amdgcn_cosf(a0);
    z[1] = r0 * __builtin_amdgcn_sinf(a0);
    z[2] = r1 * __builtin_amdgcn_cosf(a1);
    z[3] = r1 * __builtin_amdgcn_sinf(a1);
}

__device__ __forceinline__ void quad_normals(uint32_t s_lo, uint32_t s_hi, uint32_t q, uint32_t k0,
                                             uint32_t k1, double z[4]) {
    uint32_t x[4];
    philox4x32_10(s_lo, s_hi, q, 0u, k0, k1, x);
    const double r0 = sqrt(-2.0 * log(u01d(x[0])));
    const double r1 = sqrt(-2.0 * log(u01d(x[2])));
    double s0, c0, s1, c1;  // sin/cos(2*pi*u) with exact pi-reduction
    sincospi(2.0 * u01d(x[1]), &s0, &c0);
    sincospi(2.0 * u01d(x[3]), &s1, &c1);
    z[0] = r0 * c0;
    z[1] = r0 * s0;
    z[2] = r1 * c1;
    z[3] = r1 * s1;
}

// ---------------- precision traits ----------------
template <typename Real> struct Tr;
template <> struct Tr<float> {
    typedef f32x4 acc_t;
    __device__ static __forceinline__ acc_t mfma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // logistic 1/(1+exp(-(x-mu)*sigma)) with sl = sigma*log2(e) precomputed
    __device__ static __forceinline__ float sig(float x, float mu, float sl) {
        return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f((mu - x) * sl));
    }
    __device__ static __forceinline__ float slope(double s) { return (float)(s * 1.4426950408889634); }
    // output row rho of an f32 16x16x4 tile is (lane>>4)*4 + reg: identity map
    __host__ __device__ static __forceinline__ int row_node(int rho) { return rho; }
};
template <> struct Tr<double> {
    typedef f64x4 acc_t;
    __device__ static __forceinline__ acc_t mfma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static __forceinline__ double sig(double x, double mu, double s) {
        return 1.0 / (1.0 + exp(-(x - mu) * s));
    }
    __device__ static __forceinline__ double slope(double s) { return s; }
    // f64 16x16x4 C/D row is (lane>>4) + 4*reg; permute so that lane group g,
    // register r still means node 4g + r of the tile
    __host__ __device__ static __forceinline__ int row_node(int rho) { return 4 * (rho & 3) + (rho >> 2); }
};

struct KArgs {
    // model constants
    double a_ee, a_ei, a_ii, tauE, tauI, P, rhoE, rE, rI, mu, sigmaI, sqdtD, dtSim;
    double tau_ip;
    const double* G;
    const double* sigmaE;
    const uint64_t* keys;
    double* E;
    double* I;
    double* A;
    const void* frag;  // [NT*NT][64][4] Real
    void* recE;
    void* recI;
    void* recA;
    int64_t step0;
    int64_t rec_every;
    int nsteps;
    int B, N;
};

// Build the A-operand fragment image: frag[(T*NT + t)*64 + lane][r] =
//   CM[16T + row_node(lane&15)][16t + 4(lane>>4) + r]   (0 outside N)
template <typename Real, int NT>
__global__ void build_frag(const double* __restrict__ sc, int N, Real* __restrict__ frag) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = NT * NT * 64 * 4;
    if (idx >= total) return;
    const int r = idx & 3;
    const int lane = (idx >> 2) & 63;
    const int tt = idx >> 8;  // T*NT + t
    const int T = tt / NT, t = tt % NT;
    const int row = 16 * T + Tr<Real>::row_node(lane & 15);
    const int col = 16 * t + 4 * (lane >> 4) + r;
    frag[idx] = (row < N && col < N) ? (Real)sc[(size_t)row * N + col] : (Real)0;
}

// kHoist: let the compiler keep the whole fragment image in registers across
// the step loop (f32, 1 wave/SIMD); otherwise re-read it from LDS every step.
template <typename Real, int NT, bool kHoist>
__global__ void __launch_bounds__(kWaves * 64) wc_sde_kernel(const KArgs a) {
    typedef typename Tr<Real>::acc_t acc_t;
    typedef __attribute__((ext_vector_type(4))) Real real4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    real4* lfrag = reinterpret_cast<real4*>(smem);

    // stage the connectome fragment image in LDS (whole workgroup)
    {
        const real4* gfrag = reinterpret_cast<const real4*>(a.frag);
        for (int i = threadIdx.x; i < NT * NT * 64; i += blockDim.x) lfrag[i] = gfrag[i];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int j = lane & 15, g = lane >> 4;
    const int wave_sim0 = (blockIdx.x * kWaves + wave) * kSimsPerWave;
    if (wave_sim0 >= a.B) return;  // whole wave out of range (no barrier follows)
    const int b = wave_sim0 + j;
    const bool live = b < a.B;
    const int bb = live ? b : a.B - 1;  // tail lanes mirror the last sim, never store
    const int N = a.N;

    const uint64_t key = a.keys[bb];
    const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);

    // ---- load state and per-node parameters into registers ----
    // fp32 keeps G and sigmaE*log2(e) in registers; the fp64 parity path
    // re-reads them (L1/L2 resident) every step to stay out of scratch
    constexpr bool kParamRegs = sizeof(Real) == 4;
    constexpr int PT = kParamRegs ? NT : 1;
    Real E[NT][4], I[NT][4], Gc[PT][4], Sl[PT][4];
    double A[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = 16 * t + 4 * g + r;
            const bool ok = n < N;
            const size_t o = (size_t)bb * N + (ok ? n : 0);
            E[t][r] = ok ? (Real)a.E[o] : (Real)0;
            I[t][r] = ok ? (Real)a.I[o] : (Real)0;
            A[t][r] = ok ? a.A[o] : 0.0;
            if constexpr (kParamRegs) {
                Gc[t][r] = ok ? (Real)a.G[o] : (Real)0;
                Sl[t][r] = ok ? Tr<Real>::slope(a.sigmaE[o]) : (Real)0;
            }
        }

    const Real a_ee = (Real)a.a_ee, a_ei = (Real)a.a_ei, a_ii = (Real)a.a_ii;
    const Real P = (Real)a.P, rhoE = (Real)a.rhoE, rE = (Real)a.rE, rI = (Real)a.rI;
    const Real mu = (Real)a.mu, slI = Tr<Real>::slope(a.sigmaI), sqdtD = (Real)a.sqdtD;
    const Real dtE = (Real)(a.dtSim / a.tauE), dtI = (Real)(a.dtSim / a.tauI);
    const Real dt = (Real)a.dtSim;
    const double dtA = a.dtSim / a.tau_ip;
    // exact-division forms for the fp64 parity path
    const Real tauE = (Real)a.tauE, tauI = (Real)a.tauI, tau_ip = (Real)a.tau_ip;
    const size_t BN = (size_t)a.B * N;

    for (int s = 0; s < a.nsteps; ++s) {
        // ---- record the state before the update (wc:124-125) ----
        if (a.rec_every > 0 && (s % a.rec_every) == 0) {
            const size_t row = (size_t)(s / a.rec_every) * BN + (size_t)bb * N;
            if (live) {
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int n = 16 * t + 4 * g + r;
                        if (n < N) {
                            static_cast<Real*>(a.recE)[row + n] = E[t][r];
                            if (a.recI) static_cast<Real*>(a.recI)[row + n] = I[t][r];
                            if (a.recA) static_cast<Real*>(a.recA)[row + n] = (Real)A[t][r];
                        }
                    }
            }
        }

        // ---- coupling: acc[T][r] = sum_k CM[node(T,g,r)][k] * E[k]  (wc:81 np.dot) ----
        int fl = lane;
        if constexpr (!kHoist) asm volatile("" : "+v"(fl));  // opaque: no LICM of the LDS reads
        acc_t acc[NT];
#pragma unroll
        for (int T = 0; T < NT; ++T) acc[T] = acc_t{0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int T = 0; T < NT; ++T) {
                // bound how far ahead the fp64 path issues fragment reads
                if constexpr (!kHoist) if ((T & 1) == 0) __builtin_amdgcn_sched_barrier(0);
                const real4 f = lfrag[(T * NT + t) * 64 + fl];
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[T] = Tr<Real>::mfma(f[r], E[t][r], acc[T]);
            }

        // ---- elementwise update (wc:77-83), noise drawn inside the E sigmoid ----
        const uint64_t gstep = (uint64_t)(a.step0 + s);
        const uint32_t s_lo = (uint32_t)gstep, s_hi = (uint32_t)(gstep >> 32);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            // keep each tile's update (and its live range) in its own schedule region
            if constexpr (sizeof(Real) == 8) __builtin_amdgcn_sched_barrier(0);
            Real z[4];
            quad_normals(s_lo, s_hi, (uint32_t)(4 * t + g), k0, k1, z);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const Real e = E[t][r], in = I[t][r];
                const Real ai = (Real)A[t][r];
                Real gc, sl;
                if constexpr (kParamRegs) {
                    gc = Gc[t][r];
                    sl = Sl[t][r];
                } else {
                    const int n = 16 * t + 4 * g + r;
                    const size_t o = (size_t)bb * N + (n < N ? n : 0);
                    gc = n < N ? (Real)a.G[o] : (Real)0;
                    sl = n < N ? Tr<Real>::slope(a.sigmaE[o]) : (Real)0;
                }
                const Real xE = a_ee * e - ai * in + gc * acc[t][r] + P + sqdtD * z[r];
                const Real SE = Tr<Real>::sig(xE, mu, sl);
                const Real xI = a_ei * e - a_ii * in;
                const Real SI = Tr<Real>::sig(xI, mu, slI);
                if constexpr (sizeof(Real) == 8) {
                    const Real dE = (-e + (1 - rE * e) * SE) / tauE;
                    const Real dI = (-in + (1 - rI * in) * SI) / tauI;
                    const Real dA = (in * (e - rhoE)) / tau_ip;
                    E[t][r] = e + dt * dE;
                    I[t][r] = in + dt * dI;
                    A[t][r] = A[t][r] + dt * dA;
                } else {
                    E[t][r] = e + dtE * (-e + (1 - rE * e) * SE);
                    I[t][r] = in + dtI * (-in + (1 - rI * in) * SI);
                    A[t][r] = A[t][r] + dtA * (double)(in * (e - rhoE));
                }
            }
        }
    }

    // ---- write back the state ----
    if (live) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * t + 4 * g + r;
                if (n < N) {
                    const size_t o = (size_t)b * N + n;
                    a.E[o] = (double)E[t][r];
                    a.I[o] = (double)I[t][r];
                    a.A[o] = A[t][r];
                }
            }
    }
}

template <typename Real>
__global__ void noise_kernel(const uint64_t* __restrict__ keys, int B, int N, int64_t step, Real* out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int nq = (N + 3) / 4;
    if (idx >= B * nq) return;
    const int b = idx / nq, q = idx % nq;
    const uint64_t key = keys[b];
    Real z[4];
    quad_normals((uint32_t)(uint64_t)step, (uint32_t)((uint64_t)step >> 32), (uint32_t)q, (uint32_t)key,
                 (uint32_t)(key >> 32), z);
    for (int r = 0; r < 4; ++r)
        if (4 * q + r < N) out[(size_t)b * N + 4 * q + r] = z[r];
}

int tiles_for(int N) { return (N + 15) / 16; }

template <typename Real, int NT>
int launch_nt(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    const int total = NT * NT * 64 * 4;
    hipLaunchKernelGGL((build_frag<Real, NT>), dim3((total + 255) / 256), dim3(256), 0, st, sc, ka.N,
                       static_cast<Real*>(ws));
    const size_t lds = (size_t)NT * NT * 64 * 4 * sizeof(Real);
    const int blocks = (ka.B + kSimsPerBlock - 1) / kSimsPerBlock;
    constexpr bool hoist = sizeof(Real) == 4;
    auto kern = wc_sde_kernel<Real, NT, hoist>;
    if (lds > 65536) {
        hipError_t ea = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return set_err(WC_EHIP, hipGetErrorString(ea));
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kWaves * 64), lds, st, ka);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(WC_EHIP, hipGetErrorString(e));
    return WC_OK;
}

template <typename Real>
int launch(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    switch (tiles_for(ka.N)) {
        case 1: return launch_nt<Real, 1>(ka, sc, ws, st);
        case 2: return launch_nt<Real, 2>(ka, sc, ws, st);
        case 3: return launch_nt<Real, 3>(ka, sc, ws, st);
        case 4: return launch_nt<Real, 4>(ka, sc, ws, st);
        case 5: return launch_nt<Real, 5>(ka, sc, ws, st);
        case 6: return launch_nt<Real, 6>(ka, sc, ws, st);
        default: return set_err(WC_EUNSUPPORTED, "N > 96 not supported by the register-resident kernel");
    }
}

}  // namespace

extern "C" {

int wcsde_abi_version(void) { return WCSDE_ABI_VERSION; }

const char* wc_last_error(void) { return g_err; }

size_t wc_workspace_size(int N, int precision) {
    if (N <= 0) return 0;
    const int nt = tiles_for(N);
    return (size_t)nt * nt * 64 * 4 * (precision == WC_F64 ? 8 : 4);
}

int wc_integrate(const wc_params* p, int precision, int B, int N, const double* sc, const double* G,
                 const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A,
                 int64_t step0, int64_t nsteps, double tau_ip, int64_t rec_every, void* recE,
                 void* recI, void* recA, void* workspace, size_t ws_bytes, void* stream) {
    g_err[0] = 0;
    if (!p || B <= 0 || N <= 0 || nsteps < 0 || nsteps > INT32_MAX || step0 < 0 || rec_every < 0)
        return set_err(WC_EINVAL, "wc_integrate: invalid B/N/nsteps/step0/rec_every");
    if (!sc || !G || !sigmaE || !keys || !E || !I || !A)
        return set_err(WC_EINVAL, "wc_integrate: NULL array argument");
    if (precision != WC_F32 && precision != WC_F64) return set_err(WC_EINVAL, "wc_integrate: bad precision");
    if (rec_every > 0 && !recE) return set_err(WC_EINVAL, "wc_integrate: rec_every > 0 needs recE");
    if (tiles_for(N) > kMaxTiles) return set_err(WC_EUNSUPPORTED, "wc_integrate: N > 96 not supported");
    if (!workspace || ws_bytes < wc_workspace_size(N, precision))
        return set_err(WC_EWORKSPACE, "wc_integrate: workspace too small");
    if (nsteps == 0) return WC_OK;
    KArgs ka;
    ka.a_ee = p->a_ee; ka.a_ei = p->a_ei; ka.a_ii = p->a_ii;
    ka.tauE = p->tauE; ka.tauI = p->tauI; ka.P = p->P; ka.rhoE = p->rhoE;
    ka.rE = p->rE; ka.rI = p->rI; ka.mu = p->mu; ka.sigmaI = p->sigmaI;
    ka.sqdtD = p->sqdtD; ka.dtSim = p->dtSim; ka.tau_ip = tau_ip;
    ka.G = G; ka.sigmaE = sigmaE; ka.keys = keys; ka.E = E; ka.I = I; ka.A = A;
    ka.frag = workspace; ka.recE = recE; ka.recI = recI; ka.recA = recA;
    ka.step0 = step0; ka.rec_every = rec_every; ka.nsteps = (int)nsteps; ka.B = B; ka.N = N;
    hipStream_t st = static_cast<hipStream_t>(stream);
    return precision == WC_F64 ? launch<double>(ka, sc, workspace, st) : launch<float>(ka, sc, workspace, st);
}

int wc_noise(int precision, int B, int N, const uint64_t* keys, int64_t step, void* out, void* stream) {
    g_err[0] = 0;
    if (B <= 0 || N <= 0 || !keys || !out || step < 0) return set_err(WC_EINVAL, "wc_noise: bad arguments");
    const int nq = (N + 3) / 4;
    const int total = B * nq;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (precision == WC_F64)
        hipLaunchKernelGGL(noise_kernel<double>, dim3((total + 255) / 256), dim3(256), 0, st, keys, B, N, step,
                           static_cast<double*>(out));
    else
        hipLaunchKernelGGL(noise_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, st, keys, B, N, step,
                           static_cast<float*>(out));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(WC_EHIP, hipGetErrorString(e));
    return WC_OK;
}

}  // extern "C"
