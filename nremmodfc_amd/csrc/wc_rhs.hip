// wc_rhs.hip -- one evaluation of the Wilson-Cowan right-hand side, batched (fp64).
//
// netwWilsonCowanPlastic.wilsonCowan(t, X, sigmaE, mu, tau_ip, G) (wc:77-83) returns
//   [(-E + (1 - rE E) S(a_ee E - a_ie I + G CM@E + P + noise, sigmaE, mu)) / tauE,
//    (-I + (1 - rI I) S(a_ei E - a_ii I, sigmaI, mu)) / tauI,
//    I (E - rhoE) / tau_ip]
// with noise = np.random.normal(0, sqdtD, N) drawn inside the call.  The integrator fuses this
// into its step (wc_sde*.hip); this entry point exposes the single evaluation for callers that
// use the function on its own, drawing the noise of Philox step `step` of each key (the same
// normals the integrator uses at that global step).  One thread per (simulation, node); the
// dot product is summed in node order, the oracle's order (oracle/wc_oracle.c).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "wc_common.h"
#include "wc_device.h"

namespace {
using namespace wcdev;

__global__ void rhs_kernel(const wc_params p, int B, int N, const double* __restrict__ sc,
                           const double* __restrict__ G, const double* __restrict__ sigmaE,
                           const uint64_t* __restrict__ keys, int64_t step, double tau_ip,
                           const double* __restrict__ X, double* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)B * N) return;
    const int b = (int)(idx / N), i = (int)(idx % N);
    const double* E = X + (size_t)b * 3 * N;
    const double* I = E + N;
    const double* A = I + N;
    double acc = 0.0;  // np.dot(CM, E) row i
    for (int j = 0; j < N; ++j) acc += sc[(size_t)i * N + j] * E[j];
    double z[4];
    quad_normals((uint64_t)step, (uint32_t)(i / 4), keys[b], z);
    const double e = E[i], in = I[i], a = A[i];
    const size_t o = (size_t)b * N + i;
    const double noise = p.sqdtD * z[i % 4];
    const double xE = p.a_ee * e - a * in + G[o] * acc + p.P + noise;
    const double SE = 1.0 / (1.0 + exp(-(xE - p.mu) * sigmaE[o]));
    const double xI = p.a_ei * e - p.a_ii * in;
    const double SI = 1.0 / (1.0 + exp(-(xI - p.mu) * p.sigmaI));
    double* d = out + (size_t)b * 3 * N;
    d[i] = (-e + (1.0 - p.rE * e) * SE) / p.tauE;
    d[N + i] = (-in + (1.0 - p.rI * in) * SI) / p.tauI;
    d[2 * N + i] = (in * (e - p.rhoE)) / tau_ip;
}

}  // namespace

extern "C" int wc_rhs(const wc_params* p, int B, int N, const double* sc, const double* G, const double* sigmaE,
                      const uint64_t* keys, int64_t step, double tau_ip, const double* X, double* out, void* stream) {
    wc_clear_err();
    if (!p || B <= 0 || N <= 0 || !sc || !G || !sigmaE || !keys || !X || !out)
        return wc_set_err(WC_EINVAL, "wc_rhs: bad B/N or NULL argument");
    if (step < 0 || step >= (int64_t)1 << 48 || N > 4 * 65536)
        return wc_set_err(WC_EUNSUPPORTED, "wc_rhs: step >= 2^48 or N > 2^18 (Philox counter layout)");
    const int64_t n = (int64_t)B * N;
    hipLaunchKernelGGL(rhs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       *p, B, N, sc, G, sigmaE, keys, step, tau_ip, X, out);
    return wc_hip_check("wc_rhs");
}
