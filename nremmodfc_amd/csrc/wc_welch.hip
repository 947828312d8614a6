// wc_welch.hip -- Welch peak frequency of E_t for a batch of simulations (gfx950).
//
// Replaces whole_sweep_both.py:90-95:
//   freqs, fftPow = signal.welch(E_t.T, fs=1/wc.dt, nperseg=4000)
//   meanpow = fftPow.mean(axis=0); peakfreq = freqs[first argmax(meanpow)]
// scipy.signal.welch defaults: periodic Hann window, noverlap = nperseg/2,
// constant detrend per segment, density scaling, one-sided (bins 1..nperseg/2-1
// doubled), mean over segments.
//
// One workgroup per simulation and segment set: for each node, the 4000-sample
// segment is staged in LDS (node-major E: contiguous 4000-sample runs),
// mean-removed and windowed, packed as 2000 complex points z[n] = x[2n] +
// i x[2n+1], transformed by a Stockham FFT (radix 5, 5, 5, 4, 4) and unpacked
// to the 2001 real-FFT bins; |X_k|^2 is summed over nodes in registers and
// added to the simulation's fp64 accumulator row (single writer: deterministic).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>
#include "wc_common.h"

namespace {


constexpr int kSeg = 4000;     // nperseg (whole_sweep_both.py:90)
constexpr int kFFT = kSeg / 2; // packed complex length
constexpr int kBins = kFFT + 1;
constexpr int kThreads = 256;
constexpr int kBinsPerThread = (kBins + kThreads - 1) / kThreads;  // 8
#ifndef WC_WELCH_F64_THREADS
#define WC_WELCH_F64_THREADS 768  // (1024 spills at the 128-VGPR cap; 768: 100 VGPRs, 12 waves)
#endif
constexpr int kWelchF64Threads = WC_WELCH_F64_THREADS;
#ifndef WC_WELCH_W64
#define WC_WELCH_W64 1  // fp64 rings through welch_wave64_kernel (0: the LDS-Stockham welch_kernel<double>)
#endif

template <typename R> struct cx { R re, im; };
template <typename R> __device__ __forceinline__ cx<R> cmul(cx<R> a, cx<R> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename R> __device__ __forceinline__ cx<R> cadd(cx<R> a, cx<R> b) { return {a.re + b.re, a.im + b.im}; }
template <typename R> __device__ __forceinline__ cx<R> csub(cx<R> a, cx<R> b) { return {a.re - b.re, a.im - b.im}; }

// concurrent FFTs per workgroup: 2 x (ping + pong) x 2000 complex fits 64 KB (fp32) / 128 KB (fp64)
template <typename R> constexpr int kG = sizeof(R) == 4 ? 4 : 2;

// twiddle table T[m] = exp(-2 pi i m / 4000), m in [0, 4000): fp64 (tw) and its
// correctly rounded fp32 copy (tw32, right after the fp64 table)
__global__ void twiddle_kernel(double* tw) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= kSeg) return;
    double s, c;
    sincospi(2.0 * m / kSeg, &s, &c);
    tw[2 * m] = c;
    tw[2 * m + 1] = -s;
    float2* tw32 = reinterpret_cast<float2*>(tw + 2 * kSeg);
    // fp32 half turn by symmetry, T[m + 2000] = -T[m] exactly, so the product kernel can
    // keep only the first half in LDS
    if (m < kFFT) {
        tw32[m] = make_float2((float)c, (float)-s);
        tw32[m + kFFT] = make_float2(-(float)c, (float)s);
    }
    // periodic Hann pairs for the packed samples (2j, 2j+1): hann2[j] = (w(2j), w(2j+1))
    if ((m & 1) == 0) {
        double s1, c1;
        sincospi(2.0 * (m + 1) / kSeg, &s1, &c1);
        reinterpret_cast<float2*>(tw32 + kSeg)[m >> 1] = make_float2((float)(0.5 - 0.5 * c), (float)(0.5 - 0.5 * c1));
    }
}

template <typename R>
__device__ __forceinline__ cx<R> tw_at(const double* tw, int m) {  // exp(-2 pi i m / 4000), m mod 4000
#if defined(WC_W64_DIAG_NOTW)  // (ablation builds only: timing without the twiddle loads, wrong PSD)
    (void)tw;
    return {(R)1 + (R)(m & 1) * (R)1e-30, (R)0};
#else
    m %= kSeg;
    return {(R)tw[2 * m], (R)tw[2 * m + 1]};
#endif
}

// one Stockham stage of radix RAD over the 2000-point FFT, p = product of previous radices
template <typename R, int RAD>
__device__ __forceinline__ void stage(const cx<R>* __restrict__ x, cx<R>* __restrict__ y, int p, int i,
                                      const double* tw) {
    constexpr int S = kFFT / RAD;
    const int k = i % p;
    cx<R> u[RAD];
#pragma unroll
    for (int r = 0; r < RAD; ++r) u[r] = x[i + r * S];
    // twiddle exp(-2 pi i r k / (p RAD)) = T[2 * r * k * (kFFT / (p RAD))]
    const int step = 2 * (kFFT / (p * RAD));
#pragma unroll
    for (int r = 1; r < RAD; ++r) u[r] = cmul(u[r], tw_at<R>(tw, r * k * step));
    cx<R> U[RAD];
    if constexpr (RAD == 4) {
        const cx<R> a = cadd(u[0], u[2]), b = csub(u[0], u[2]);
        const cx<R> c = cadd(u[1], u[3]), d = csub(u[1], u[3]);
        U[0] = cadd(a, c);
        U[2] = csub(a, c);
        U[1] = {b.re + d.im, b.im - d.re};  // b - i d
        U[3] = {b.re - d.im, b.im + d.re};  // b + i d
    } else {  // RAD == 5
        const R c1 = (R)0.30901699437494742410, c2 = (R)-0.80901699437494742410;  // cos(2pi/5), cos(4pi/5)
        const R s1 = (R)0.95105651629515357212, s2 = (R)0.58778525229247312917;   // sin(2pi/5), sin(4pi/5)
        const cx<R> t1 = cadd(u[1], u[4]), t2 = cadd(u[2], u[3]);
        const cx<R> t3 = csub(u[1], u[4]), t4 = csub(u[2], u[3]);
        U[0] = {u[0].re + t1.re + t2.re, u[0].im + t1.im + t2.im};
        const cx<R> a1 = {u[0].re + c1 * t1.re + c2 * t2.re, u[0].im + c1 * t1.im + c2 * t2.im};
        const cx<R> a2 = {u[0].re + c2 * t1.re + c1 * t2.re, u[0].im + c2 * t1.im + c1 * t2.im};
        // -i (s1 t3 + s2 t4) and -i (s2 t3 - s1 t4)
        const cx<R> b1 = {s1 * t3.re + s2 * t4.re, s1 * t3.im + s2 * t4.im};
        const cx<R> b2 = {s2 * t3.re - s1 * t4.re, s2 * t3.im - s1 * t4.im};
        U[1] = {a1.re + b1.im, a1.im - b1.re};
        U[4] = {a1.re - b1.im, a1.im + b1.re};
        U[2] = {a2.re + b2.im, a2.im - b2.re};
        U[3] = {a2.re - b2.im, a2.im + b2.re};
    }
    const int j = (i - k) * RAD + k;
#pragma unroll
    for (int s = 0; s < RAD; ++s) y[j + s * p] = U[s];
}

template <typename R, int RAD, int T = kThreads>
__device__ __forceinline__ void run_stage(cx<R>* const* src, cx<R>* const* dst, int p, const double* tw) {
    constexpr int nb = kFFT / RAD;
    for (int idx = threadIdx.x; idx < kG<R> * nb; idx += T) {
        const int g = idx / nb, i = idx % nb;
        stage<R, RAD>(src[g], dst[g], p, i, tw);
    }
    __syncthreads();
}

struct WelchArgs {
    int B, N;
    const void* E;     // node-major ring: element (c, t) at c*ld + ((t/slot) % nslots)*slot + t % slot
    int64_t ld, slot, nslots;
    int64_t seg0;      // first sample of the (first) segment
    int nseg;          // consecutive segments (hop kSeg / 2) in this launch: 1, 2 or 4 (welch_wave_kernel)
    const double* tw;  // twiddle table
    double* acc;       // [B][kBins] running sum over nodes and segments of |X_k|^2
};

// T threads per workgroup: 256 for the fp32 fallback; 768 for fp64 (kWelchF64Threads), whose
// 128 KB of LDS allow one workgroup per CU -- 12 waves instead of 4 to hide its LDS and memory latency
template <typename R, int T = kThreads>
__global__ void __launch_bounds__(T) welch_kernel(const WelchArgs a) {
    constexpr int kW = T / 64, kBpt = (kBins + T - 1) / T;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cx<R>* base = reinterpret_cast<cx<R>*>(smem);  // [kG][2][kFFT]
    R* red = reinterpret_cast<R*>(base + 2 * kG<R> * kFFT);  // [kW waves][kG]
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const R* E = static_cast<const R*>(a.E);
    cx<R>* buf0[kG<R>];
    cx<R>* buf1[kG<R>];
#pragma unroll
    for (int g = 0; g < kG<R>; ++g) {
        buf0[g] = base + (2 * g) * kFFT;
        buf1[g] = base + (2 * g + 1) * kFFT;
    }
    double acc[kBpt];
#pragma unroll
    for (int j = 0; j < kBpt; ++j) acc[j] = 0.0;

    for (int n0 = 0; n0 < a.N; n0 += kG<R>) {
        // ---- stage the raw segments (as reals) and their sums ----
        R part[kG<R>];
#pragma unroll
        for (int g = 0; g < kG<R>; ++g) {
            part[g] = 0;
            const int n = n0 + g;
            R* xr = reinterpret_cast<R*>(buf0[g]);
            if (n < a.N) {
                const R* col = E + ((int64_t)b * a.N + n) * a.ld;
                // the segment is <= 5 contiguous runs of the ring (wave-uniform bookkeeping)
                for (int t = 0; t < kSeg;) {
                    const int64_t ts = a.seg0 + t;
                    const int64_t q = ts / a.slot, r = ts % a.slot;
                    const int len = (int)min((int64_t)(kSeg - t), a.slot - r);
                    const R* src = col + (q % a.nslots) * a.slot + r;
                    for (int i = tid; i < len; i += T) {
#if defined(WC_W64_DIAG_NOLOAD)  // (ablation builds only: timing without the segment loads, wrong PSD)
                        const R v = (R)(i & 7) + (R)(src == nullptr);
#else
                        const R v = src[i];
#endif
                        xr[t + i] = v;
                        part[g] += v;
                    }
                    t += len;
                }
            } else {
                for (int t = tid; t < kSeg; t += T) xr[t] = 0;
            }
        }
        // block reduction of the kG sums (wave shuffles, then 4 partials per g)
#pragma unroll
        for (int g = 0; g < kG<R>; ++g) {
            R v = part[g];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if ((tid & 63) == 0) red[(tid >> 6) * kG<R> + g] = v;
        }
        __syncthreads();
        R mean[kG<R>];
#pragma unroll
        for (int g = 0; g < kG<R>; ++g)
        {
            R sum = 0;
            for (int wv = 0; wv < kW; ++wv) sum += red[wv * kG<R> + g];  // (wave order: deterministic)
            mean[g] = sum / (R)kSeg;
        }
        // ---- detrend, periodic Hann window, pack z[n] = x[2n] + i x[2n+1] (in place) ----
#pragma unroll
        for (int g = 0; g < kG<R>; ++g) {
            cx<R>* z = buf0[g];
            for (int m = tid; m < kFFT; m += T) {
                const cx<R> v = z[m];
                const R w0 = (R)(0.5 - 0.5 * a.tw[2 * (2 * m)]);
                const R w1 = (R)(0.5 - 0.5 * a.tw[2 * (2 * m + 1)]);
                z[m] = {w0 * (v.re - mean[g]), w1 * (v.im - mean[g])};
            }
        }
        __syncthreads();
        // ---- Stockham 2000 = 5 * 5 * 5 * 4 * 4 ----
        run_stage<R, 5, T>(buf0, buf1, 1, a.tw);
        run_stage<R, 5, T>(buf1, buf0, 5, a.tw);
        run_stage<R, 5, T>(buf0, buf1, 25, a.tw);
        run_stage<R, 4, T>(buf1, buf0, 125, a.tw);
        run_stage<R, 4, T>(buf0, buf1, 500, a.tw);
        // ---- unpack X_k = (Z_k + conj Z_{-k})/2 - i/2 W^k (Z_k - conj Z_{-k}), |X_k|^2 ----
#pragma unroll
        for (int j = 0; j < kBpt; ++j) {
            const int k = tid + j * T;
            if (k < kBins) {
#pragma unroll
                for (int g = 0; g < kG<R>; ++g) {
                    if (n0 + g >= a.N) continue;
                    const cx<R> Zk = buf1[g][k % kFFT];
                    const cx<R> Zc = buf1[g][(kFFT - k) % kFFT];
                    const double er = 0.5 * ((double)Zk.re + Zc.re), ei = 0.5 * ((double)Zk.im - Zc.im);
                    const double dr = (double)Zk.re - Zc.re, di = (double)Zk.im + Zc.im;
                    const double wr = a.tw[2 * k], wi = a.tw[2 * k + 1];
                    // -i/2 * W * d
                    const double pr = wr * dr - wi * di, pi = wr * di + wi * dr;
                    const double xr = er + 0.5 * pi, xi = ei - 0.5 * pr;
                    acc[j] += xr * xr + xi * xi;
                }
            }
        }
        __syncthreads();  // buffers reused by the next node group
    }
#pragma unroll
    for (int j = 0; j < kBpt; ++j) {
        const int k = tid + j * T;
        if (k < kBins) a.acc[(int64_t)b * kBins + k] += acc[j];
    }
}

// ---------------- fp64 kernel: two waves per column ----------------
// The reference-precision pipeline's Welch (whole_sweep_both.py:90-95 with the fp64 ring).  The
// LDS-Stockham welch_kernel<double> above spends most of its time at workgroup barriers and on
// twiddle loads from memory (20% VALU issue, 58% of wave cycles waiting; profiles/r05/w64_ablation.log).
// Here a pair of waves (128 threads) owns one column's 2000-point packed FFT in 32 KB of LDS, four
// columns (eight waves, two per SIMD) per workgroup:
//   * the 4000-sample segment comes from HBM as 16-B sample pairs, thread t holding packed points
//     m = t + 128 j (j < 16); the next column's loads are issued as soon as the current one is in
//     LDS, so they run under its FFT;
//   * mean (block reduction over the pair) and the periodic Hann window, w(e) = 0.5 - 0.5 Re T^e with
//     T^(2m) = T^(256 j) T^(2t): the uniform factor an LDS broadcast, the thread's from registers;
//   * Stockham 2000 = 5 * 5 * 5 * 4 * 4 in place (every read of a stage into registers, a barrier,
//     every write, a barrier), twiddles from per-stage fp64 tables in LDS (1,995 entries, 31.9 KB);
//   * the real-FFT unpack with W^k = T^(128 j) T^t, |X_k|^2 summed per thread (bins k = t + 128 j)
//     over the pair's columns; at the end the four pairs (one simulation per workgroup) are combined
//     in a fixed order into its fp64 row (single writer, deterministic).
// Same radix order and butterflies as welch_kernel<double>; the mean and the window are summed /
// formed in another order (PSD within 1e-12 of it, 1e-9 of the oracle: test_signal_gpu.py).
constexpr int kW64Cols = 4, kW64Threads = kW64Cols * 128;
constexpr int kW64Tb2 = 0, kW64Tb3 = kW64Tb2 + 4 * 5, kW64Tb4 = kW64Tb3 + 4 * 25, kW64Tb5 = kW64Tb4 + 3 * 125;
constexpr int kW64StageTw = kW64Tb5 + 3 * 500;  // 1995
typedef double d2 __attribute__((ext_vector_type(2)));  // (re, im)
// LDS: the columns, the stage tables, T^(256 j) and T^(128 j) (j < 16), the pairs' partial sums
constexpr size_t kW64Lds = ((size_t)kW64Cols * kFFT + kW64StageTw + 32) * sizeof(d2) + kW64Cols * 2 * sizeof(double);

typedef const volatile __attribute__((address_space(3))) d2* lds_d2p;
__device__ __forceinline__ d2 ldsr64(const d2* p) { return *(lds_d2p)(p); }
__device__ __forceinline__ d2 cmul64(d2 a, d2 w) {
    return d2{__builtin_fma(a.x, w.x, -a.y * w.y), __builtin_fma(a.x, w.y, a.y * w.x)};
}

template <int RAD>
__device__ __forceinline__ void butterfly64(d2 (&u)[RAD]) {
    if constexpr (RAD == 4) {
        const d2 a = u[0] + u[2], b = u[0] - u[2];
        const d2 c = u[1] + u[3], d = u[1] - u[3];
        u[0] = a + c;
        u[2] = a - c;
        u[1] = d2{b.x + d.y, b.y - d.x};  // b - i d
        u[3] = d2{b.x - d.y, b.y + d.x};  // b + i d
    } else {
        const double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;  // cos(2pi/5), cos(4pi/5)
        const double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;   // sin(2pi/5), sin(4pi/5)
        const d2 t1 = u[1] + u[4], t2 = u[2] + u[3];
        const d2 t3 = u[1] - u[4], t4 = u[2] - u[3];
        const d2 a1 = u[0] + c1 * t1 + c2 * t2;
        const d2 a2 = u[0] + c2 * t1 + c1 * t2;
        const d2 b1 = s1 * t3 + s2 * t4, b2 = s2 * t3 - s1 * t4;
        u[0] = u[0] + t1 + t2;
        u[1] = d2{a1.x + b1.y, a1.y - b1.x};  // a1 - i b1
        u[4] = d2{a1.x - b1.y, a1.y + b1.x};
        u[2] = d2{a2.x + b2.y, a2.y - b2.x};  // a2 - i b2
        u[3] = d2{a2.x - b2.y, a2.y + b2.x};
    }
}

// one radix-RAD Stockham stage over a column's 2000 points, in place (P = product of the previous
// radices, TB its table base): butterfly i = t + 128 q of the pair's thread t; a partial last row
// re-reads the stage's last butterfly (clamped) and writes nothing.  Both barriers are workgroup
// barriers: the four columns of the workgroup step together.
template <int RAD, int P, int TB>
__device__ __forceinline__ void w64_stage(d2* z, const d2* Ts, int t) {
    constexpr int S = kFFT / RAD, NQ = (S + 127) / 128;
    d2 u[NQ][RAD];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {  // every point read first, back to back
        const int i = min(t + 128 * q, S - 1);
#pragma unroll
        for (int r = 0; r < RAD; ++r) u[q][r] = ldsr64(z + i + r * S);
    }
    if constexpr (P > 1) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int k = min(t + 128 * q, S - 1) % P;
            d2 tw[RAD - 1];  // (plain reads of the read-only table: one LDS wait per row)
#pragma unroll
            for (int r = 1; r < RAD; ++r) tw[r - 1] = Ts[TB + (r - 1) * P + k];
#pragma unroll
            for (int r = 1; r < RAD; ++r) u[q][r] = cmul64(u[q][r], tw[r - 1]);
            __builtin_amdgcn_sched_barrier(0);  // one row's twiddles live at a time
        }
    }
    __syncthreads();  // every read of the stage (both waves of the column) before any write
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = t + 128 * q, ic = min(i, S - 1), k = ic % P;
        butterfly64<RAD>(u[q]);
        if (128 * (q + 1) <= S || i < S) {
            const int j = (ic - k) * RAD + k;
#pragma unroll
            for (int s2i = 0; s2i < RAD; ++s2i) z[j + s2i * P] = u[q][s2i];
        }
    }
    __syncthreads();
}

__global__ void __launch_bounds__(kW64Threads, 1) welch_wave64_kernel(const WelchArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int c = threadIdx.x >> 7, t = threadIdx.x & 127;  // column slot of the workgroup, thread in the pair
    const int b = blockIdx.x;
    d2* z = reinterpret_cast<d2*>(smem) + c * kFFT;
    d2* Ts = reinterpret_cast<d2*>(smem) + kW64Cols * kFFT;
    d2* Tj = Ts + kW64StageTw;  // [0, 16): T^(256 j); [16, 32): T^(128 j)
    double* red = reinterpret_cast<double*>(Tj + 32);  // [column slot][wave of the pair]
    const d2* T = reinterpret_cast<const d2*>(a.tw);  // T^m = exp(-2 pi i m / 4000), m < 4000
    // per-stage tables: entry (r - 1) P + k of the stage with (P, RAD) is T^(r k 4000 / (P RAD))
    for (int e = threadIdx.x; e < kW64StageTw; e += kW64Threads) {
        int base, P, RAD;
        if (e < kW64Tb3) { base = kW64Tb2; P = 5; RAD = 5; }
        else if (e < kW64Tb4) { base = kW64Tb3; P = 25; RAD = 5; }
        else if (e < kW64Tb5) { base = kW64Tb4; P = 125; RAD = 4; }
        else { base = kW64Tb5; P = 500; RAD = 4; }
        const int k = (e - base) % P, r = (e - base) / P + 1;
        Ts[e] = T[(r * k * (kSeg / (P * RAD))) % kSeg];
    }
    if (threadIdx.x < 32) Tj[threadIdx.x] = T[threadIdx.x < 16 ? 256 * threadIdx.x : 128 * (threadIdx.x - 16)];
    // the thread's factors of the window (T^(2t), T^(2t + 1)) and of the unpack twiddle (T^t)
    const d2 tl0 = T[2 * t], tl1 = T[2 * t + 1], tu = T[t];
    const double* E = static_cast<const double*>(a.E);
    // circular ring per column: sample seg0 + s at (seg0 + s) mod L (byte offsets in 32 bits)
    const unsigned L = (unsigned)(a.slot * a.nslots);
    const unsigned baseB = (unsigned)(a.seg0 % L) * 8u, LB = L * 8u;
    const int64_t bc = (int64_t)b * a.N;
    double acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0;
    d2 x[16];  // samples (2m, 2m + 1) of packed point m = t + 128 j (row 15: threads < 80; others clamp)
    auto fetch = [&](int n, int tt) {
        const char* col = reinterpret_cast<const char*>(E + (bc + n) * a.ld);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            unsigned o = baseB + 16u * (unsigned)min(tt + 128 * j, kFFT - 1);
            o = min(o, o - LB);
            x[j] = *reinterpret_cast<const d2*>(col + o);
        }
    };
    // every column slot runs the same number of iterations (the stages' workgroup barriers); a slot
    // past the last column transforms the last one again and adds nothing
    const int iters = (a.N + kW64Cols - 1) / kW64Cols;
    fetch(min(c, a.N - 1), t);
    __syncthreads();  // stage tables in LDS
    for (int it = 0; it < iters; ++it) {
        const int n = c + kW64Cols * it;
        const bool live = n < a.N;
        // (the thread id laundered per column: hoisted out of the loop, the stages' loop-invariant
        // twiddle and point addresses would be held across it, i.e. spilled)
        int tt = t;
        asm volatile("" : "+v"(tt));
        tt &= 127;
        // ---- mean over the 4000 samples (thread partials, each wave, then the pair) ----
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < 15 || tt < 80) sum += x[j].x + x[j].y;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        if ((tt & 63) == 0) red[c * 2 + (tt >> 6)] = sum;
        __syncthreads();
        const double mean = (red[c * 2] + red[c * 2 + 1]) / (double)kSeg;
        // ---- detrend and window into LDS: w(2m) = 0.5 - 0.5 Re(T^(256 j) T^(2t)) ----
#pragma unroll
        for (int jb = 0; jb < 16; jb += 8) {  // (the factors read eight at a time: one LDS wait per batch)
            d2 tj[8];
#pragma unroll
            for (int u8 = 0; u8 < 8; ++u8) tj[u8] = ldsr64(Tj + jb + u8);  // (uniform address: an LDS broadcast)
#pragma unroll
            for (int u8 = 0; u8 < 8; ++u8) {
                const int j = jb + u8;
                const double c0 = __builtin_fma(tj[u8].x, tl0.x, -tj[u8].y * tl0.y);
                const double c1 = __builtin_fma(tj[u8].x, tl1.x, -tj[u8].y * tl1.y);
                const d2 v = d2{__builtin_fma(-0.5, c0, 0.5) * (x[j].x - mean), __builtin_fma(-0.5, c1, 0.5) * (x[j].y - mean)};
                if (j < 15 || tt < 80) z[tt + 128 * j] = v;
            }
        }
        __syncthreads();
        // the registers are free: the next column's loads run under this one's FFT
        if (it + 1 < iters) fetch(min(n + kW64Cols, a.N - 1), tt);
        w64_stage<5, 1, 0>(z, Ts, tt);
        w64_stage<5, 5, kW64Tb2>(z, Ts, tt);
        w64_stage<5, 25, kW64Tb3>(z, Ts, tt);
        w64_stage<4, 125, kW64Tb4>(z, Ts, tt);
        w64_stage<4, 500, kW64Tb5>(z, Ts, tt);
        // ---- unpack X_k = (Z_k + conj Z_{-k})/2 - i/2 W^k (Z_k - conj Z_{-k}), |X_k|^2 ----
#pragma unroll
        for (int jb = 0; jb < 16; jb += 4) {  // (four bins read ahead: one LDS wait per batch)
            d2 Zk4[4], Zc4[4], tj4[4];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                const int k = min(tt + 128 * (jb + u4), kFFT);
                Zk4[u4] = ldsr64(z + (k == kFFT ? 0 : k));
                Zc4[u4] = ldsr64(z + (k == 0 ? 0 : kFFT - k));
                tj4[u4] = ldsr64(Tj + 16 + jb + u4);
            }
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                const int j = jb + u4;
                const d2 Zk = Zk4[u4], Zc = Zc4[u4], tj = tj4[u4];
                const d2 W = d2{__builtin_fma(tj.x, tu.x, -tj.y * tu.y), __builtin_fma(tj.x, tu.y, tj.y * tu.x)};
                const double er = 0.5 * (Zk.x + Zc.x), ei = 0.5 * (Zk.y - Zc.y);
                const double dr = Zk.x - Zc.x, di = Zk.y + Zc.y;
                const double pr = W.x * dr - W.y * di, pi = W.x * di + W.y * dr;
                const double xr = er + 0.5 * pi, xi = ei - 0.5 * pr;
                if (live && (j < 15 || tt <= 80)) acc[j] += xr * xr + xi * xi;
            }
        }
        __syncthreads();  // the unpack's reads before the next column's window writes
    }
    // ---- the four column slots' sums into the simulation's row (fixed order: single writer) ----
    double* part = reinterpret_cast<double*>(smem);  // [column slot][16 rows][128 threads]
#pragma unroll
    for (int j = 0; j < 16; ++j) part[(c * 16 + j) * 128 + t] = acc[j];
    __syncthreads();
    for (int k = threadIdx.x; k < kBins; k += kW64Threads) {
        const int j = k >> 7, l = k & 127;
        double s2 = 0.0;
#pragma unroll
        for (int v = 0; v < kW64Cols; ++v) s2 += part[(v * 16 + j) * 128 + l];
        a.acc[(int64_t)b * kBins + k] += s2;
    }
}

// ---------------- fp32 product kernel: one wave per column ----------------
// Each wave owns one column's 2000-point packed FFT in its own 16 KB of LDS and
// runs it with no workgroup barrier: every radix stage reads all of the wave's
// butterfly inputs into registers, then writes the outputs in place (the wave
// owns every point).  Eight waves per workgroup, four per simulation (two
// simulations per workgroup), one workgroup per CU: 8 x 16 KB of columns plus
// 32 KB of twiddle tables shared by the eight waves (per-stage tables laid out
// [r][k], so a row's lanes read consecutive entries and need no index arithmetic
// beyond k).  While a column is transformed, the wave's next column
// is already on its way from HBM into registers, so the FFT never waits on
// memory.  fp32 arithmetic with the correctly rounded fp32 twiddle table;
// |X_k|^2 summed per lane in fp32 over the wave's ~N/4 columns, then the four
// waves of a simulation are combined in fp64 and added to its fp64 row.
constexpr int kWv = 4;       // waves (columns in flight) per simulation
constexpr int kSimsWg = 2;   // simulations per workgroup
constexpr int kLaneBins = (kBins + 63) / 64;  // 32
#ifndef WC_WELCH_PF_EARLY
#define WC_WELCH_PF_EARLY 8  // (all of them; clipped to the row count, and even under WC_WELCH_X4)
#endif
constexpr int kPfEarly = WC_WELCH_PF_EARLY;  // rows of the next column fetched right after stage 1 (min'd with kXR below)
// per-stage twiddle tables: entry (k, r) = T^(r k TS) at base + (r - 1) P + k (r-major: the
// lanes of a row read consecutive k, conflict-free; r is an immediate offset)
// (stages 5 x 5 x 5 x 16; the first has no twiddles)
constexpr int kTb2 = 0, kTb3 = kTb2 + 5 * 4, kTb4 = kTb3 + 25 * 4;
constexpr int kStageTw = kTb4 + 125 * 15;  // 1995
constexpr int kUnpTw = kBins + 1;         // T^k, k in [0, 2000] (+1 pad: 16-B aligned stage tables)
constexpr size_t kWelchLds = (size_t)kWv * kSimsWg * kFFT * 8 + (size_t)(kUnpTw + kStageTw) * 8;  // 159,976 B

typedef float f2 __attribute__((ext_vector_type(2)));

// stage tables from the fp32 turn (run after twiddle_kernel): entry (k, r) of the
// stage with (P, RAD) is T^(r k TS), TS = 2 kFFT / (P RAD), r k TS < 4000
__global__ void stage_twiddle_kernel(double* tw) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= kStageTw) return;
    const float2* tw32 = reinterpret_cast<const float2*>(tw + 2 * kSeg);
    float2* st = const_cast<float2*>(tw32) + kSeg + kFFT;
    int base, P, RAD;
    if (m < kTb3) { base = kTb2; P = 5; RAD = 5; }
    else if (m < kTb4) { base = kTb3; P = 25; RAD = 5; }
    else { base = kTb4; P = 125; RAD = 16; }
    const int k = (m - base) % P, r = (m - base) / P + 1;
    st[m] = tw32[r * k * (2 * kFFT / (P * RAD))];
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Packed complex helpers written with explicit VOP3P modifiers (op_sel picks the
// register half each result lane reads, neg_lo/neg_hi negate per lane): the compiler
// does not fold a one-lane negation into the modifiers and would emit xor + mov pairs.
__device__ __forceinline__ f2 cmulv(f2 u, f2 w) {  // u * w in two packed ops
    f2 t, r;
    // t = (u.x w.x, u.x w.y)
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(u), "v"(w));
    // r = (-u.y w.y + t.x, u.y w.x + t.y)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(u), "v"(w), "v"(t));
    return r;
}
// two independent products with their instructions interleaved: a v_pk_* op that reads the result of
// the one right before it needs a wait state on gfx950 (an s_nop when nothing independent sits between)
__device__ __forceinline__ void cmulv2(f2& u0, f2 w0, f2& u1, f2 w1) {
    f2 t0, t1, r0, r1;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t0) : "v"(u0), "v"(w0));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t1) : "v"(u1), "v"(w1));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r0) : "v"(u0), "v"(w0), "v"(t0));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r1) : "v"(u1), "v"(w1), "v"(t1));
    u0 = r0;
    u1 = r1;
}
// u[r] *= w[r - 1] for r = 1 .. K - 1, two products at a time
template <int K>
__device__ __forceinline__ void cmul_rows(f2 (&u)[K], const f2 (&w)[K - 1]) {
#pragma unroll
    for (int r = 1; r + 1 < K; r += 2) cmulv2(u[r], w[r - 1], u[r + 1], w[r]);
    if constexpr ((K - 1) % 2) u[K - 1] = cmulv(u[K - 1], w[K - 2]);
}
__device__ __forceinline__ f2 add_mi(f2 a, f2 d) {  // a - i d = (a.x + d.y, a.y - d.x)
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(d));
    return r;
}
__device__ __forceinline__ f2 sub_mi(f2 a, f2 d) {  // a + i d = (a.x - d.y, a.y + d.x)
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(d));
    return r;
}

// LDS reads one wave-instruction per access: volatile keeps the compiler from pairing
// them into ds_read2_b64, which costs 8 LDS cycles against 2 x 2 for two ds_read_b64
typedef const volatile __attribute__((address_space(3))) f2* lds_f2p;
__device__ __forceinline__ f2 ldsr(const f2* p) { return *(lds_f2p)(p); }

// Radix-RAD Stockham stage, in place (P = product of the previous radices, TB its
// twiddle table base).  Every read is unconditional (the lanes of a partial last row
// re-read the row's last butterfly, index clamped); only that row's writes are masked.
template <int RAD, int P> struct Rows {
    static constexpr int S = kFFT / RAD, NB = (S + 63) / 64;
    __device__ static int idx(int lane, int q) { return 64 * (q + 1) <= S ? lane + 64 * q : min(lane + 64 * q, S - 1); }
    __device__ static bool own(int lane, int q) { return 64 * (q + 1) <= S || lane + 64 * q < S; }
};

template <int RAD>
__device__ __forceinline__ void butterfly(const f2 (&u)[RAD], f2 (&U)[RAD]) {
    if constexpr (RAD == 4) {
        const f2 a = u[0] + u[2], b = u[0] - u[2];
        const f2 c = u[1] + u[3], d = u[1] - u[3];
        U[0] = a + c;
        U[2] = a - c;
        U[1] = add_mi(b, d);  // b - i d
        U[3] = sub_mi(b, d);  // b + i d
    } else {
        const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
        const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
        const f2 t1 = u[1] + u[4], t2 = u[2] + u[3];
        const f2 t3 = u[1] - u[4], t4 = u[2] - u[3];
        U[0] = u[0] + t1 + t2;
        const f2 a1 = u[0] + c1 * t1 + c2 * t2;
        const f2 a2 = u[0] + c2 * t1 + c1 * t2;
        const f2 b1 = s1 * t3 + s2 * t4, b2 = s2 * t3 - s1 * t4;
        U[1] = add_mi(a1, b1);  // a1 - i b1
        U[4] = sub_mi(a1, b1);
        U[2] = add_mi(a2, b2);
        U[3] = sub_mi(a2, b2);
    }
}

#ifndef WC_WELCH_X4
#define WC_WELCH_X4 1  // stage-1 points fetched as 16-B pairs (two butterflies per lane and load)
#endif
// stage 1 under WC_WELCH_X4: lane l holds butterflies 2l + j + 128 p (rows q = 2p + j, p < 4), so
// one 16-B load brings the points of rows 2p and 2p + 1; rows 6 and 7 are owned by lanes 0..7
// only (the others re-read points 398, 399 and write nothing)
struct Rows1x4 {
    static constexpr int S = kFFT / 5, NB = 8;
    __device__ static int idx(int lane, int q) { return min(2 * lane + (q & 1) + 128 * (q >> 1), S - 1); }
    __device__ static bool own(int lane, int q) { return q < 6 || 2 * lane + (q & 1) + 128 * (q >> 1) < S; }
    __device__ static int pair_base(int lane, int p) { return min(2 * lane + 128 * p, S - 2); }  // even
};

template <typename R, int RAD, int P>
__device__ __forceinline__ void write_rows_t(f2* z, f2 (&u)[R::NB][RAD], int lane) {
#pragma unroll
    for (int q = 0; q < R::NB; ++q) {
        const int i = R::idx(lane, q), k = i % P;
        f2 U[RAD];
        butterfly<RAD>(u[q], U);
        const int j = (i - k) * RAD + k;
        if (R::own(lane, q)) {
#pragma unroll
            for (int s2i = 0; s2i < RAD; ++s2i) z[j + s2i * P] = U[s2i];
        }
    }
}

template <int RAD, int P>
__device__ __forceinline__ void write_rows(f2* z, f2 (&u)[Rows<RAD, P>::NB][RAD], int lane) {
    write_rows_t<Rows<RAD, P>, RAD, P>(z, u, lane);
}

// stage 1 (radix 5, no twiddles) fed from registers: x[q][r] = packed point i + 400 r of
// the raw column; the column mean (constant detrend) and the periodic Hann window
// w(t) = 0.5 - 0.5 cos(2 pi t / 4000) are applied on the way in
using Rows1 = std::conditional_t<WC_WELCH_X4 != 0, Rows1x4, Rows<5, 1>>;
constexpr int kXR = Rows1::NB;  // stage-1 rows per lane: 8 (16-B pairs) or 7
constexpr int kPf = kPfEarly < kXR ? kPfEarly : kXR;
static_assert(!WC_WELCH_X4 || kPf % 2 == 0, "16-B pair fetch: an even number of early rows");
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wstage1(f2* z, f2 (&x)[kXR][5], const f2* __restrict__ hann, int lane) {
    using R = Rows1;
    float part = 0.f;
    f2 hw[kXR][5];
#pragma unroll
    for (int q = 0; q < kXR; ++q) {
        const int i = R::idx(lane, q);
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            part += R::own(lane, q) ? x[q][r].x + x[q][r].y : 0.f;
            // (w(2m), w(2m+1)); unsigned byte offset: the saddr form of the load
#if defined(WC_WELCH_DIAG_NOHANN)  // (ablation builds only: timing without the window loads, wrong PSD)
            hw[q][r] = (f2){1.0f, 1.0f};
            (void)i;
#elif WC_WELCH_X4
            if ((q & 1) == 0) {  // the window of rows q, q + 1 in one 16-B load
                const f4v w4 = *reinterpret_cast<const f4v*>(
                    reinterpret_cast<const char*>(hann) + (unsigned)(R::pair_base(lane, q >> 1) + r * R::S) * 8u);
                hw[q][r] = (f2){w4.x, w4.y};
                hw[q + 1][r] = (f2){w4.z, w4.w};
            }
            (void)i;
#else
            hw[q][r] = *reinterpret_cast<const f2*>(reinterpret_cast<const char*>(hann) + (unsigned)(i + r * R::S) * 8u);
#endif
        }
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    const float mean = part / (float)kSeg;
#pragma unroll
    for (int q = 0; q < kXR; ++q)
#pragma unroll
        for (int r = 0; r < 5; ++r) x[q][r] = (x[q][r] - mean) * hw[q][r];
#if WC_WELCH_X4
    // butterflies i0, i0 + 1 write z[5 i0 .. 5 i0 + 9], 80 contiguous bytes per lane: five 16-B writes,
    // conflict-free (lane stride 20 dwords) where ten 8-B ones at that stride met in pairs of lanes
#pragma unroll
    for (int p = 0; p < kXR / 2; ++p) {
        f2 Ua[5], Ub[5];
        butterfly<5>(x[2 * p], Ua);
        butterfly<5>(x[2 * p + 1], Ub);
        if (R::own(lane, 2 * p)) {
            f4v* zz = reinterpret_cast<f4v*>(z + 5 * R::pair_base(lane, p));
            zz[0] = (f4v){Ua[0].x, Ua[0].y, Ua[1].x, Ua[1].y};
            zz[1] = (f4v){Ua[2].x, Ua[2].y, Ua[3].x, Ua[3].y};
            zz[2] = (f4v){Ua[4].x, Ua[4].y, Ub[0].x, Ub[0].y};
            zz[3] = (f4v){Ub[1].x, Ub[1].y, Ub[2].x, Ub[2].y};
            zz[4] = (f4v){Ub[3].x, Ub[3].y, Ub[4].x, Ub[4].y};
        }
    }
#else
    write_rows_t<R, 5, 1>(z, x, lane);
#endif
    wave_sync();
}

template <int RAD, int P, int TB>
__device__ __forceinline__ void wstage(f2* z, const f2* Ts, int lane) {
    using R = Rows<RAD, P>;
    f2 u[R::NB][RAD];
#pragma unroll
    for (int q = 0; q < R::NB; ++q) {
        const int i = R::idx(lane, q);
#pragma unroll
        for (int r = 0; r < RAD; ++r) u[q][r] = ldsr(z + i + r * R::S);
    }
    wave_sync();
    // twiddles one row ahead: the volatile LDS reads are scheduling barriers, so a row's
    // reads issued right before its own products were each waited on (one exposed LDS
    // round trip per twiddle); issuing row q+1's reads before row q's products keeps
    // them in flight behind that work
    f2 tw[2][RAD - 1];
#pragma unroll
    for (int r = 1; r < RAD; ++r) tw[0][r - 1] = ldsr(Ts + TB + R::idx(lane, 0) % P + (r - 1) * P);
#pragma unroll
    for (int q = 0; q < R::NB; ++q) {
        if (q + 1 < R::NB) {
#pragma unroll
            for (int r = 1; r < RAD; ++r)
                tw[(q + 1) & 1][r - 1] = ldsr(Ts + TB + R::idx(lane, q + 1) % P + (r - 1) * P);
        }
        cmul_rows<RAD>(u[q], tw[q & 1]);
    }
    write_rows<RAD, P>(z, u, lane);
    wave_sync();
}

// 16-point DFT U[s] = sum_r u[r] W16^(r s) as 4 x 4 (r = 4 r1 + r2, s = s1 + 4 s2):
// radix-4 over r1, twiddle W16^(r2 s1), radix-4 over r2
__device__ __forceinline__ void dft16(f2 (&u)[16]) {
    constexpr float h = 0.70710678118654752440f, c = 0.92387953251128675613f, d = 0.38268343236508977173f;
    f2 v[4][4];  // v[r2][s1]
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) {
        const f2 in[4] = {u[r2], u[4 + r2], u[8 + r2], u[12 + r2]};
        butterfly<4>(in, v[r2]);
    }
    // W16^j = (cos, -sin)(2 pi j / 16): j = r2 s1 in {1, 2, 3, 4, 6, 9}
    cmulv2(v[1][1], (f2){c, -d}, v[1][2], (f2){h, -h});
    cmulv2(v[1][3], (f2){d, -c}, v[2][1], (f2){h, -h});
    cmulv2(v[2][2], (f2){0.f, -1.f}, v[2][3], (f2){-h, -h});
    cmulv2(v[3][1], (f2){d, -c}, v[3][2], (f2){-h, -h});
    v[3][3] = cmulv(v[3][3], (f2){-c, d});
#pragma unroll
    for (int s1 = 0; s1 < 4; ++s1) {
        const f2 in[4] = {v[0][s1], v[1][s1], v[2][s1], v[3][s1]};
        f2 o[4];
        butterfly<4>(in, o);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) u[s1 + 4 * s2] = o[s2];
    }
}

// acc + v * v as one v_fma_f32 (written out: the compiler pairs the two bins' accumulators into
// v_pk_fma_f32 and transposes their operands with three v_mov per pair, 5 VALU for 4 fmas)
__device__ __forceinline__ float sq_acc(float v, float acc) {
    float r;
    asm("v_fma_f32 %0, %1, %1, %2" : "=v"(r) : "v"(v), "v"(acc));
    return r;
}

// Last stage (radix 16, P = 125) fused with the real-FFT unpack, all in registers.
// Butterfly i produces Z_{i + 125 s}, s = 0..15; bin k pairs Z_k with Z_{2000-k}, and
// Z_{2000 - (i + 125 s)} is slot 15 - s of butterfly 125 - i.  Row 0 of a lane holds
// butterfly m = lane (m <= 62) and row 1 its partner 125 - m, so every pair meets in
// one lane: 2 X_k = s - i p and 2 X_{2000-k} = conj(s + i p), with s = Z_k + conj Z_c,
// d = Z_k - conj Z_c, p = T^k d.  Butterfly 0 is its own partner (Z_c = slot
// (16 - s) % 16 of the same row).  acc[s][0] collects bin m + 125 s, acc[s][1] bin
// 2000 - m - 125 s (times 4).
__device__ __forceinline__ void wstage_last_unpack(const f2* z, const f2* Ts, const f2* Tu, float (&acc)[16][2],
                                                   int lane) {
    const int m = min(lane, 62);
    const int rows[2] = {m, 125 - max(m, 1)};
    f2 u[2][16];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) u[q][r] = ldsr(z + rows[q] + 125 * r);
    wave_sync();  // (the next column's stage 1 overwrites z)
    // twiddle reads batched ahead of the work that needs them (see wstage): row 0's before
    // its products, row 1's before row 0's DFT, the unpack's before row 1's DFT
    f2 tw[2][15], tu[16];
#pragma unroll
    for (int r = 1; r < 16; ++r) tw[0][r - 1] = ldsr(Ts + kTb4 + (r - 1) * 125 + rows[0]);
    cmul_rows<16>(u[0], tw[0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) tw[1][r - 1] = ldsr(Ts + kTb4 + (r - 1) * 125 + rows[1]);
    dft16(u[0]);
    cmul_rows<16>(u[1], tw[1]);
#pragma unroll
    for (int s2i = 0; s2i < 16; ++s2i) tu[s2i] = ldsr(Tu + m + 125 * s2i);
    dft16(u[1]);
    // two bins at a time, their instructions interleaved (no v_pk_* right behind its producer; the
    // same operations on every value)
#pragma unroll
    for (int s2i = 0; s2i < 16; s2i += 2) {
        f2 sv[2], dv[2], pv[2], xa[2], xb[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int si = s2i + k;
            const f2 Zk = u[0][si];
            const f2 Zc = m == 0 ? u[0][(16 - si) & 15] : u[1][15 - si];
            asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(sv[k]) : "v"(Zk), "v"(Zc));
            asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(dv[k]) : "v"(Zk), "v"(Zc));
        }
        pv[0] = dv[0];
        pv[1] = dv[1];
        cmulv2(pv[0], tu[s2i], pv[1], tu[s2i + 1]);
#pragma unroll
        for (int k = 0; k < 2; ++k) xa[k] = add_mi(sv[k], pv[k]);
#pragma unroll
        for (int k = 0; k < 2; ++k) xb[k] = sub_mi(sv[k], pv[k]);
        float t[2][2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            t[k][0] = sq_acc(xa[k].y, acc[s2i + k][0]);
            t[k][1] = sq_acc(xb[k].y, acc[s2i + k][1]);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            acc[s2i + k][0] = sq_acc(xa[k].x, t[k][0]);
            acc[s2i + k][1] = sq_acc(xb[k].x, t[k][1]);
        }
    }
}

__global__ void __launch_bounds__(kWv * kSimsWg * 64, 1) welch_wave_kernel(const WelchArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // (the wave index through readfirstlane: the column base is then scalar and every load the
    // saddr form, an SGPR base plus a 32-bit lane offset, instead of a 64-bit VGPR address each)
    const int wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int w = wg & (kWv - 1);                         // column slot within the simulation
    // nseg == 2: waves w and w ^ 1 take segments 0 and 1 of the same column at the same time (the
    // half they share is read once from HBM, once from the caches), each wave every other column;
    // nseg == 4: wave w takes segment w of every column
    const int sgi = w % a.nseg, cstep = kWv / a.nseg, c0 = w / a.nseg;
    const int b = blockIdx.x * kSimsWg + wg / kWv;        // this wave's simulation
    const int ncol = b < a.B ? a.N : 0;
    f2* z = reinterpret_cast<f2*>(smem) + wg * kFFT;
    f2* Tu = reinterpret_cast<f2*>(smem) + kWv * kSimsWg * kFFT;  // T^k for the unpack
    f2* Ts = Tu + kUnpTw;                                          // per-stage tables
    const float* twg = reinterpret_cast<const float*>(a.tw + 2 * kSeg);  // fp32 tables: T, Hann, stage
    const f2* hann = reinterpret_cast<const f2*>(twg) + kSeg;
    const float* E = static_cast<const float*>(a.E);
    float acc[16][2];
#pragma unroll
    for (int s2i = 0; s2i < 16; ++s2i) acc[s2i][0] = acc[s2i][1] = 0.f;
    // the ring is circular per column: sample seg0 + t sits at (seg0 + t) mod L, L = slot * nslots
    // (byte offsets in 32 bits: the host admits ld < INT32_MAX / 2 - 8192, so 4 (L + 4000) < 2^32)
    const unsigned L = (unsigned)(a.slot * a.nslots);
    const unsigned baseB = (unsigned)((a.seg0 + (int64_t)sgi * (kSeg / 2)) % L) * 4u, LB = L * 4u;
    // stage-1 inputs come straight from HBM into registers, in the butterfly layout
    // (x[q][r] = packed point i + 400 r, i = lane + 64 q); the next column is fetched
    // while the current one is transformed (branch-free: the clamped lanes of row 6
    // re-read a valid point, and a wave's last column re-fetches itself, an L2 hit)
    f2 x[kXR][5];
    const int64_t bc = (int64_t)min(b, a.B - 1) * a.N;
    // (uniform column base + 32-bit unsigned lane offset: the saddr form of global_load)
#if WC_WELCH_X4
    // rows 2p, 2p + 1 from one 16-B load of points i0, i0 + 1 (i0 even: the four samples sit in one
    // aligned group, which the ring's wrap never splits: seg0, L and the slot length are multiples of 4)
#define WELCH_FETCH(n, Q0, Q1, LN)                                                             \
    {                                                                                          \
        const float* col_ = E + (bc + (n)) * a.ld;                                             \
        _Pragma("unroll") for (int p = (Q0) / 2; p < (Q1) / 2; ++p) {                          \
            const int i_ = Rows1x4::pair_base(LN, p);                                          \
            _Pragma("unroll") for (int r = 0; r < 5; ++r) {                                    \
                unsigned o_ = baseB + 8u * (unsigned)(i_ + 400 * r);                           \
                o_ = min(o_, o_ - LB);                                                         \
                const f4v v_ = *reinterpret_cast<const f4v*>(reinterpret_cast<const char*>(col_) + o_); \
                x[2 * p][r] = (f2){v_.x, v_.y};                                                \
                x[2 * p + 1][r] = (f2){v_.z, v_.w};                                            \
            }                                                                                  \
        }                                                                                      \
    }
#else
#define WELCH_FETCH(n, Q0, Q1, LN)                                                             \
    {                                                                                          \
        const float* col_ = E + (bc + (n)) * a.ld;                                             \
        _Pragma("unroll") for (int q = Q0; q < Q1; ++q) {                                      \
            const int i_ = Rows<5, 1>::idx(LN, q);                                            \
            _Pragma("unroll") for (int r = 0; r < 5; ++r) {                                    \
                unsigned o_ = baseB + 8u * (unsigned)(i_ + 400 * r);                           \
                o_ = min(o_, o_ - LB);                                                         \
                x[q][r] = *reinterpret_cast<const f2*>(reinterpret_cast<const char*>(col_) + o_); \
            }                                                                                  \
        }                                                                                      \
    }
#endif
    WELCH_FETCH(min(c0, a.N - 1), 0, kXR, lane);
    {  // twiddle tables into LDS: T^0..T^2000 and the stage tables (the pad entry is never read)
        const f2* src = reinterpret_cast<const f2*>(twg);
        const f2* sst = reinterpret_cast<const f2*>(twg) + kSeg + kFFT;
        for (int i = threadIdx.x; i < kUnpTw + kStageTw; i += kWv * kSimsWg * 64)
            Tu[i] = i < kBins ? src[i] : i < kUnpTw ? (f2){0.f, 0.f} : sst[i - kUnpTw];
    }
    __syncthreads();

    for (int n = c0; n < ncol; n += cstep) {
        // (the lane id is laundered per column so the compiler does not hoist hundreds
        // of loop-invariant twiddle offsets out of the column loop)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        ln &= 63;  // (range-known again: unsigned index arithmetic, static masks)
        // ---- Stockham 2000 = 5 * 5 * 5 * 16, window fused into the first stage,
        //      the real-FFT unpack into the last ----
        wstage1(z, x, hann, ln);
        // the Hann loads have retired: the next column's loads are the only VMEM in flight
        const int nn = n + cstep < ncol ? n + cstep : n;
#if defined(WC_WELCH_DIAG_NOLOAD)  // (ablation builds only: tools/dbg/welch_variants.sh)
        (void)nn;
#else
        WELCH_FETCH(nn, 0, kPf, ln);
#endif
#if defined(WC_WELCH_DIAG_NOFFT)
        {
            const f2 v = ldsr(z + ln);
            acc[0][0] += v.x;
            acc[0][1] += v.y;
        }
        WELCH_FETCH(nn, kPf, kXR, ln);
#else
        wstage<5, 5, kTb2>(z, Ts, ln);
        wstage<5, 25, kTb3>(z, Ts, ln);
#if !defined(WC_WELCH_DIAG_NOLOAD)
        WELCH_FETCH(nn, kPf, kXR, ln);  // (the rest of the next column: fewer live registers through the stages)
#endif
        wstage_last_unpack(z, Ts, Tu, acc, ln);
#endif
    }
#undef WELCH_FETCH
    // ---- combine each simulation's four waves (fp64) into its accumulator row (single writer) ----
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [kSimsWg][kWv][kBins]
#pragma unroll
    for (int s2i = 0; s2i < 16; ++s2i) {
        // each bin once: lane 63 repeats lane 62; butterfly 0 pairs with itself, so its
        // slots past 8 repeat earlier bins and slot 8 is bin 1000 twice
        const bool ok = lane < 63 && !(lane == 0 && s2i > 8);
        const int k = lane + 125 * s2i;
        if (ok) red[wg * kBins + k] = acc[s2i][0];
        if (ok && !(lane == 0 && s2i == 8)) red[wg * kBins + kFFT - k] = acc[s2i][1];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < kSimsWg * kBins; idx += kWv * kSimsWg * 64) {
        const int sw = idx / kBins, k = idx % kBins;
        const int bs = blockIdx.x * kSimsWg + sw;
        if (bs >= a.B) continue;
        double sacc = 0.0;
#pragma unroll
        for (int v = 0; v < kWv; ++v) sacc += (double)red[(sw * kWv + v) * kBins + k];
        a.acc[(int64_t)bs * kBins + k] += 0.25 * sacc;
    }
}

// ---------------- fp32 product kernel, two waves per column ----------------
// The one-wave kernel above holds 16 KB of LDS per column in flight and 232 VGPRs, so a CU
// runs 8 columns on 8 waves, two per SIMD, and each column's stages are one wave's serial
// chain of LDS round trips (latency-bound, PMC: VALU issue 55% busy).  Here a PAIR of waves
// shares a column: stages 1-3 split the 7 butterfly rows 4 + 3 between them, and the radix-16
// last stage gives each lane ONE butterfly b: the lower half-wave holds b = m, the upper
// half-wave its unpack partner b = 125 - m in the same lane pair (m = 0 pairs with a virtual
// butterfly 125: butterfly 0 read with twiddles T^(250 r) = W16^r, i.e. its outputs rotated by
// one slot, Z_{125 (s + 1)}).  Two half-exchanges per slot pair (v_permlane32_swap) hand each
// lane its partner's slots 8..15, so every lane unpacks 8 bin pairs with no select.  Workgroup
// = one simulation, 4 column pairs (8 waves, 80 KB of LDS), two workgroups per CU: 16 waves at
// <= 128 VGPRs.  Six workgroup barriers per column (the pair's in-place stages need
// read -> barrier -> write -> barrier); the other workgroup on the CU runs between them.
#ifndef WC_WELCH_PAIR
#define WC_WELCH_PAIR 0  // 1: build the two-waves-per-column kernel and launch it (ablation)
#endif
#if WC_WELCH_PAIR
constexpr int kPairCols = 4;                       // column pairs per workgroup
constexpr int kPairThreads = kPairCols * 2 * 64;   // 512
constexpr int kP4 = 126;                           // last-stage table width: butterflies 0..125
constexpr int kPTs2 = 0, kPTs3 = kPTs2 + 4 * 5, kPTs4 = kPTs3 + 4 * 25;
constexpr int kPTw = kPTs4 + 15 * kP4;             // 2010 stage twiddles
constexpr size_t kPairLds = (size_t)kPairCols * kFFT * 8 + (size_t)kPTw * 8 + 2 * kPairCols * 4;  // 80,112 B

// one radix-5 stage over rows q0 .. q0 + NQ - 1 of the 7 (P = 1: the windowed stage 1 from
// registers; else in place from LDS with the table at TB): reads, barrier, products, writes
template <int P, int NQ, int Q0>
__device__ __forceinline__ void pstage_rw(f2* z, const f2* Ts, int TB, int lane) {
    using R = Rows<5, P>;
    f2 u[NQ][5];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = R::idx(lane, Q0 + q);
#pragma unroll
        for (int r = 0; r < 5; ++r) u[q][r] = ldsr(z + i + r * R::S);
    }
    __syncthreads();  // both waves' reads of the column precede either's in-place writes
    f2 tw[2][4];
#pragma unroll
    for (int r = 1; r < 5; ++r) tw[0][r - 1] = ldsr(Ts + TB + R::idx(lane, Q0) % P + (r - 1) * P);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) {
#pragma unroll
            for (int r = 1; r < 5; ++r) tw[(q + 1) & 1][r - 1] = ldsr(Ts + TB + R::idx(lane, Q0 + q + 1) % P + (r - 1) * P);
        }
#pragma unroll
        for (int r = 1; r < 5; ++r) u[q][r] = cmulv(u[q][r], tw[q & 1][r - 1]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = R::idx(lane, Q0 + q), k = i % P;
        f2 U[5];
        butterfly<5>(u[q], U);
        const int j = (i - k) * 5 + k;
        if (R::own(lane, Q0 + q)) {
#pragma unroll
            for (int s = 0; s < 5; ++s) z[j + s * P] = U[s];
        }
    }
    __syncthreads();
}

// half-exchange between the wave's lane halves: afterwards a holds the partner lane's b and
// b the partner's a (lanes l and l ^ 32), two v_permlane32_swap per dword
__device__ __forceinline__ float2 swap_halves(float a, float b) {
    const auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const auto r2 = __builtin_amdgcn_permlane32_swap(r1[1], r1[0], false, false);
    return make_float2(__uint_as_float(r2[1]), __uint_as_float(r2[0]));
}
__device__ __forceinline__ void swap_pair(f2& a, f2& b) {
    const float2 x = swap_halves(a.x, b.x), y = swap_halves(a.y, b.y);
    a = (f2){x.x, y.x};
    b = (f2){x.y, y.y};
}

template <int H>
__device__ __forceinline__ void pair_columns(const WelchArgs& a, f2* z, const f2* Ts, float* red, float* redf, int c,
                                             int lane) {
    constexpr int NQ = H == 0 ? 4 : 3, Q0 = H == 0 ? 0 : 4;  // stage 1-3 rows of this wave
    const int b = blockIdx.x;
    const int ncol = a.N;
    const float* twg = reinterpret_cast<const float*>(a.tw + 2 * kSeg);
    const f2* tw32 = reinterpret_cast<const f2*>(twg);
    const f2* hann = tw32 + kSeg;
    const float* E = static_cast<const float*>(a.E);
    // last-stage butterfly of this lane: pair p = 32 H + lane % 32 (m = min(p, 62)), lower
    // half b = m, upper half its partner 125 - m; valid pairs p <= 62
    const int p = 32 * H + (lane & 31);
    const int m = min(p, 62);
    const int bl = lane < 32 ? m : 125 - m;
    const int brd = bl == 125 ? 0 : bl;  // the virtual butterfly 125 reads butterfly 0
    const f2 tb = tw32[bl];              // T^b: the unpack twiddles T^(b + 125 s) = T^b W32^s
    float acc[8][2];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s][0] = acc[s][1] = 0.f;
    const unsigned L = (unsigned)(a.slot * a.nslots);
    const unsigned baseB = (unsigned)(a.seg0 % L) * 4u, LB = L * 4u;
    const int64_t bc = (int64_t)b * ncol;
    f2 x[NQ][5];
#define PAIR_FETCH(n, QA, QB, LN)                                                              \
    {                                                                                          \
        const float* col_ = E + (bc + (n)) * a.ld;                                             \
        _Pragma("unroll") for (int q = QA; q < QB; ++q) {                                      \
            const int i_ = Rows<5, 1>::idx(LN, Q0 + q);                                       \
            _Pragma("unroll") for (int r = 0; r < 5; ++r) {                                    \
                unsigned o_ = baseB + 8u * (unsigned)(i_ + 400 * r);                           \
                o_ = min(o_, o_ - LB);                                                         \
                x[q][r] = *reinterpret_cast<const f2*>(reinterpret_cast<const char*>(col_) + o_); \
            }                                                                                  \
        }                                                                                      \
    }
    PAIR_FETCH(min(c, ncol - 1), 0, NQ, lane);
    // every pair runs the same number of columns (barriers): the last round's missing columns
    // repeat column ncol - 1 and are not accumulated
    for (int n0 = 0; n0 < ncol; n0 += kPairCols) {
        const int n = n0 + c;
        const bool live = n < ncol;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        ln &= 63;
        // ---- column mean (constant detrend): the pair's two partial sums ----
        float part = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int r = 0; r < 5; ++r) part += Rows<5, 1>::own(ln, Q0 + q) ? x[q][r].x + x[q][r].y : 0.f;
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
        if (ln == 0) red[2 * c + H] = part;
        __syncthreads();  // (B1: also every wave's last-stage reads of the previous column are done)
        const float mean = (red[2 * c] + red[2 * c + 1]) / (float)kSeg;
        // ---- stage 1 (radix 5, no twiddles): detrend, periodic Hann window, butterflies ----
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = Rows<5, 1>::idx(ln, Q0 + q);
            f2 U[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                const f2 hw = *reinterpret_cast<const f2*>(reinterpret_cast<const char*>(hann) + (unsigned)(i + r * 400) * 8u);
                x[q][r] = (x[q][r] - mean) * hw;
            }
            butterfly<5>(x[q], U);
            if (Rows<5, 1>::own(ln, Q0 + q)) {
#pragma unroll
                for (int s = 0; s < 5; ++s) z[5 * i + s] = U[s];
            }
        }
        const int nn = min(n + kPairCols, ncol - 1);
        PAIR_FETCH(nn, 0, NQ - 1, ln);
        __syncthreads();  // B2
        pstage_rw<5, NQ, Q0>(z, Ts, kPTs2, ln);   // B3, B4
        pstage_rw<25, NQ, Q0>(z, Ts, kPTs3, ln);  // B5, B6
        PAIR_FETCH(nn, NQ - 1, NQ, ln);
        // ---- last stage (radix 16, P = 125): one butterfly per lane, then the unpack ----
        f2 u[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) u[r] = ldsr(z + brd + 125 * r);
        f2 tw[15];
#pragma unroll
        for (int r = 1; r < 16; ++r) tw[r - 1] = ldsr(Ts + kPTs4 + (r - 1) * kP4 + bl);
#pragma unroll
        for (int r = 1; r < 16; ++r) u[r] = cmulv(u[r], tw[r - 1]);
        dft16(u);
        // partner's slots 8..15: afterwards slot 8 + t holds the partner's 15 - t and v.v.
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            swap_pair(u[8 + t], u[15 - t]);
        }
        if (live) {
            f2 tu = tb;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                // W32^s = exp(-2 pi i s / 32)
                constexpr float w32c[8] = {1.f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                                           0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                                           0.19509032201612826785f};
                constexpr float w32s[8] = {0.f, 0.19509032201612826785f, 0.38268343236508977173f, 0.55557023301960222474f,
                                           0.70710678118654752440f, 0.83146961230254523708f, 0.92387953251128675613f,
                                           0.98078528040323044913f};
                if (s > 0) tu = cmulv(tb, (f2){w32c[s], -w32s[s]});
                const f2 Zk = u[s], Zc = u[8 + s];
                f2 sv, dv;
                asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(sv) : "v"(Zk), "v"(Zc));
                asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(dv) : "v"(Zk), "v"(Zc));
                const f2 pv = cmulv(dv, tu);
                const f2 xa = add_mi(sv, pv), xb = sub_mi(sv, pv);
                acc[s][0] = sq_acc(xa.x, sq_acc(xa.y, acc[s][0]));
                acc[s][1] = sq_acc(xb.x, sq_acc(xb.y, acc[s][1]));
            }
        }
    }
#undef PAIR_FETCH
    __syncthreads();  // the column buffers become the reduction area
    // bins once each: pairs p <= 62; of the pair (0, 125) the virtual butterfly gives bin 1000 only
    const bool okp = p <= 62;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int k0 = bl + 125 * s, k1 = kFFT - bl - 125 * s;
        const bool virt = bl == 125;
        if (okp && (!virt || s == 7)) redf[c * kBins + k0] = acc[s][0];
        if (okp && !virt) redf[c * kBins + k1] = acc[s][1];
    }
}

__global__ void __launch_bounds__(kPairThreads, 4) welch_pair_kernel(const WelchArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = wg >> 1, h = wg & 1;
    f2* z = reinterpret_cast<f2*>(smem) + c * kFFT;
    f2* Ts = reinterpret_cast<f2*>(smem) + kPairCols * kFFT;
    float* red = reinterpret_cast<float*>(Ts + kPTw);
    float* redf = reinterpret_cast<float*>(smem);  // [kPairCols][kBins] after the column loop
    {  // stage tables from the fp32 turn: entry (k, r) of the stage (P, RAD) = T^(r k 4000 / (P RAD))
        const f2* tw32 = reinterpret_cast<const f2*>(a.tw + 2 * kSeg);
        for (int i = threadIdx.x; i < kPTw; i += kPairThreads) {
            int P, RAD, base, W;
            if (i < kPTs3) { base = kPTs2; P = 5; RAD = 5; W = 5; }
            else if (i < kPTs4) { base = kPTs3; P = 25; RAD = 5; W = 25; }
            else { base = kPTs4; P = 125; RAD = 16; W = kP4; }
            const int k = (i - base) % W, r = (i - base) / W + 1;
            Ts[i] = tw32[(r * k * (kSeg / (P * RAD))) % kSeg];
        }
    }
    __syncthreads();
    if (h == 0) pair_columns<0>(a, z, Ts, red, redf, c, lane);
    else pair_columns<1>(a, z, Ts, red, redf, c, lane);
    __syncthreads();
    for (int k = threadIdx.x; k < kBins; k += kPairThreads) {
        double sacc = 0.0;
#pragma unroll
        for (int v = 0; v < kPairCols; ++v) sacc += (double)redf[v * kBins + k];
        a.acc[(int64_t)blockIdx.x * kBins + k] += 0.25 * sacc;
    }
}

#endif  // WC_WELCH_PAIR

// mean PSD (density scaling, one-sided) and the first argmax -> peak frequency
__global__ void welch_peak_kernel(int B, int N, int nseg, double fs, const double* __restrict__ acc,
                                  double* __restrict__ peak, double* __restrict__ psd) {
    __shared__ double bv[kThreads];
    __shared__ int bi[kThreads];
    const int b = blockIdx.x, tid = threadIdx.x;
    // scale = 1/(fs * sum(w^2)); sum of the periodic Hann squared = 3/8 * nperseg
    const double scale = 1.0 / (fs * (3.0 / 8.0) * kSeg) / ((double)nseg * N);
    double best = -1.0;
    int besti = 0;
    for (int k = tid; k < kBins; k += kThreads) {
        double v = acc[(int64_t)b * kBins + k] * scale;
        if (k > 0 && k < kBins - 1) v *= 2.0;
        if (psd) psd[(int64_t)b * kBins + k] = v;
        if (v > best) { best = v; besti = k; }
    }
    bv[tid] = best;
    bi[tid] = besti;
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if (tid < s) {
            if (bv[tid + s] > bv[tid] || (bv[tid + s] == bv[tid] && bi[tid + s] < bi[tid])) {
                bv[tid] = bv[tid + s];
                bi[tid] = bi[tid + s];
            }
        }
        __syncthreads();
    }
    if (tid == 0) peak[b] = bi[0] * fs / kSeg;
}

}  // namespace

extern "C" {

size_t wc_welch_workspace_size(void) {
    // fp64 turn, fp32 turn, fp32 Hann pairs, fp32 stage tables
    return (size_t)kSeg * 2 * sizeof(double) + (size_t)kSeg * sizeof(float2) + (size_t)kFFT * sizeof(float2) +
           (size_t)kStageTw * sizeof(float2);
}
int wc_welch_bins(void) { return kBins; }

int wc_welch_prepare(void* workspace, size_t ws_bytes, void* stream) {
    wc_clear_err();
    if (!workspace || ws_bytes < wc_welch_workspace_size()) return wc_set_err(WC_EWORKSPACE, "wc_welch_prepare");
    hipLaunchKernelGGL(twiddle_kernel, dim3((kSeg + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<double*>(workspace));
    hipLaunchKernelGGL(stage_twiddle_kernel, dim3((kStageTw + 255) / 256), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<double*>(workspace));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}

int wc_welch_accumulate(int B, int N, const void* E, int e_f64, int64_t ld, int64_t slot, int64_t nslots,
                        int64_t seg0, int nseg, const void* workspace, double* acc, void* stream) {
    wc_clear_err();
    if (B <= 0 || N <= 0 || !E || !acc || !workspace || slot <= 0 || nslots <= 0 || seg0 < 0 || ld < slot * nslots ||
        (nseg != 1 && nseg != 2 && nseg != 4) || kSeg + (int64_t)(nseg - 1) * (kSeg / 2) > slot * nslots)
        return wc_set_err(WC_EINVAL, "wc_welch_accumulate: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const bool wave = !e_f64 && ld % 4 == 0 && slot % 4 == 0 && seg0 % 4 == 0 && ((uintptr_t)E & 15) == 0 &&
                      ld < INT32_MAX / 2 - 8192;
    // fp64 rings: the wave-per-column kernel when sample pairs are 16-B aligned and never split by
    // the ring's wrap (even seg0, slot * nslots and ld; byte offsets within 32 bits)
    bool w64 = WC_WELCH_W64 && e_f64 && seg0 % 2 == 0 && (slot * nslots) % 2 == 0 && ld % 2 == 0 &&
               ((uintptr_t)E & 15) == 0 && slot * nslots < INT32_MAX / 8 - 8192;
    // it needs ~160.5 KB of dynamic LDS: if the runtime refuses that, the LDS-Stockham kernel takes the
    // same inputs (one segment per launch, the same PSD to 3e-16)
    if (w64 && hipFuncSetAttribute((const void*)welch_wave64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kW64Lds) != hipSuccess) {
        (void)hipGetLastError();
        w64 = false;
    }
    // the LDS-Stockham kernels (fp64 input, unaligned rings) take one segment per launch
    for (int sg = 0; sg < (wave ? 1 : nseg); ++sg) {
        WelchArgs a{B, N, E, ld, slot, nslots, seg0 + (int64_t)sg * (kSeg / 2), wave ? nseg : 1,
                    static_cast<const double*>(workspace), acc};
        if (e_f64 && w64) {
            hipLaunchKernelGGL(welch_wave64_kernel, dim3(B), dim3(kW64Threads), kW64Lds, st, a);
        } else if (e_f64) {
            constexpr int T = kWelchF64Threads;
            const size_t lds = (size_t)2 * kG<double> * kFFT * sizeof(cx<double>) + (T / 64) * kG<double> * sizeof(double);
            hipError_t ea = hipFuncSetAttribute((const void*)welch_kernel<double, T>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (ea != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(ea));
            hipLaunchKernelGGL((welch_kernel<double, T>), dim3(B), dim3(T), lds, st, a);
        } else if (wave) {
#if WC_WELCH_PAIR
            if (nseg != 1) return wc_set_err(WC_EINVAL, "wc_welch_accumulate: the pair build takes one segment");
            hipError_t ea = hipFuncSetAttribute((const void*)welch_pair_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPairLds);
            if (ea != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(ea));
            hipLaunchKernelGGL(welch_pair_kernel, dim3(B), dim3(kPairThreads), kPairLds, st, a);
#else
            hipError_t ea = hipFuncSetAttribute((const void*)welch_wave_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWelchLds);
            if (ea != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(ea));
            hipLaunchKernelGGL(welch_wave_kernel, dim3((B + kSimsWg - 1) / kSimsWg), dim3(kWv * kSimsWg * 64),
                               kWelchLds, st, a);
#endif
        } else {  // unaligned rings (e.g. odd lengths): the LDS-Stockham kernel, scalar loads
            const size_t lds = (size_t)2 * kG<float> * kFFT * sizeof(cx<float>) + 4 * kG<float> * sizeof(float);
            hipError_t ea = hipFuncSetAttribute((const void*)welch_kernel<float>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (ea != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(ea));
            hipLaunchKernelGGL(welch_kernel<float>, dim3(B), dim3(kThreads), lds, st, a);
        }
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}

int wc_welch_peak(int B, int N, int nseg, double fs, const double* acc, double* peak, double* psd, void* stream) {
    wc_clear_err();
    if (B <= 0 || N <= 0 || nseg <= 0 || !acc || !peak) return wc_set_err(WC_EINVAL, "wc_welch_peak: bad arguments");
    hipLaunchKernelGGL(welch_peak_kernel, dim3(B), dim3(kThreads), 0, static_cast<hipStream_t>(stream), B, N, nseg,
                       fs, acc, peak, psd);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}

}  // extern "C"
