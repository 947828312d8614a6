// wc_signal.hip -- the per-simulation signal chain after the integrator, on gfx950.
//
// Replaces, for a whole batch of simulations at once:
//   simBOLD  (netwWilsonCowanPlastic.py:140-158): BD.Sim -> drop Neq -> Bessel
//            band-pass filtfilt (axis 0) -> [::BOLD_downsamp]
//   sFC = np.corrcoef(BOLD.T)                   (whole_sweep_both.py:81)
//   utils.get_all_metrics(sFC, empFC, 1) x K    (utils.py:42-50, whole_sweep_both.py:83-86)
//   utils.kuramoto(BOLD), np.mean(sFC)          (utils.py:34-40, whole_sweep_both.py:93-94)
//
// Columns: one (simulation, node) time series = column c = b*N + n; every
// trajectory array is time-major [t][C] so consecutive threads read
// consecutive addresses at every time step (HBM-coalesced).
//
// filtfilt without the trajectory: the forward IIR is causal
// and streams with the BOLD ODE.  The backward IIR is linear, so over a
// decimation block of L samples its state obeys z_out = A^L z_in + u and the
// decimated output is y_zs + c A^(L-1) z_in, where (y_zs, u) -- the zero-state
// backward pass over the block alone -- are fixed linear functionals of the
// block: y_zs = sum_k h[k] y[k], u = sum_k G[k] y[k], with h / G the filter's
// impulse response / state response at lag k (position k from the block
// START: independent of the block length).  wc_bold_init tabulates (h, G) in
// double-double; wc_bold_chunk accumulates the five sums as the forward output
// is produced (no block buffer at all); wc_bold_finish runs the 298-step
// backward recursion over blocks from the end state of the odd-extended tail.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <complex>
#include <cstdlib>
#include "wc_common.h"

// N > 96: wc_fc_large.hip
size_t wc_large_fc_metrics_workspace_size(int B, int N, int K, int own_fc);
int wc_large_fc_metrics(int B, int N, int M, const double* bold, const double* fc_in, const double* empfc, int K,
                        double data_range, const double* kur, double* fc_out, double* metrics, double* extra,
                        void* workspace, size_t ws_bytes, hipStream_t st);

namespace {


constexpr int kPad = 15;  // filtfilt padlen = 3*max(len(a), len(b)) for an order-4 filter

// state layout (doubles), all [k][C] planes, then the (h, G) table [dec][5]
struct BoldLayout {
    int64_t C, M;
    int64_t bal, zf, head, x16, acc, yzs, u, zend, tab, total;
    __host__ __device__ BoldLayout(int64_t C_, int64_t M_, int64_t dec) : C(C_), M(M_) {
        bal = 0;                 // 4: s, f, v, q
        zf = bal + 4 * C;        // 4: forward IIR state
        head = zf + 4 * C;       // 16: x[0..15]
        x16 = head + 16 * C;     // 16: x[n-16..n-1]
        acc = x16 + 16 * C;      // 5: running (y_zs, u) sums of the current block
        yzs = acc + 5 * C;       // M: zero-state backward output at each block start
        u = yzs + M * C;         // 4M: zero-state backward state after each block
        zend = u + 4 * M * C;    // 4: backward state entering the last sample
        tab = zend + 4 * C;      // dec x 5: h[k], G[k][0..3]
        total = tab + 5 * dec;
    }
};

// scipy lfilter (DF2T), one step, with fused multiply-adds (z + x b - y a as two fmas): the
// oracle (oracle/sigchain.py) keeps scipy's unfused order and is bit-exact with scipy; the
// device differs from it by rounding only (~1e-16 relative per step; the BOLD tests compare
// at 1e-7 of max|BOLD| after the whole filtfilt), 6 fp64 operations fewer per sample
__device__ __forceinline__ double iir_step(double z[4], double x, const double* b, const double* a) {
    const double y = fma(x, b[0], z[0]);
    z[0] = fma(x, b[1], fma(-y, a[1], z[1]));
    z[1] = fma(x, b[2], fma(-y, a[2], z[2]));
    z[2] = fma(x, b[3], fma(-y, a[3], z[3]));
    z[3] = fma(x, b[4], -y * a[4]);
    return y;
}
// the same step for b[1] == b[3] == 0 (the Bessel band-pass): fma(x, 0, t) == t exactly
// for finite x, so the result is bit-identical with two fmas fewer
__device__ __forceinline__ double iir_step_bp(double z[4], double x, const double* b, const double* a) {
    const double y = fma(x, b[0], z[0]);
    z[0] = fma(-y, a[1], z[1]);
    z[1] = fma(x, b[2], fma(-y, a[2], z[2]));
    z[2] = fma(-y, a[3], z[3]);
    z[3] = fma(x, b[4], -y * a[4]);
    return y;
}

// e^x for the Balloon's (1 - E0)^(1/f) (|x| < 700): x = k ln2 + r, |r| <= ln2/2,
// e^r by its degree-11 Taylor polynomial (truncation < 7e-15 relative), 2^k by
// ldexp.  Straight-line, no special cases (ocml's exp spends ~20 more instructions
// on range checks and coefficient moves).
// Horner steps as three-address v_fma_f64: with the coefficients hoisted into VGPRs the
// compiler otherwise emits v_mov_b64 (copy the coefficient into the destination) +
// v_fmac_f64 per step, 8 extra moves per sample in the BOLD loop.  Same fused operation,
// same bits.
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// 2^y for the Balloon's (1 - E0)^(1/f) = 2^(log2(1 - E0) / f) (|y| < 1000): y = k + r, k = rint(y),
// r = y - k exact (|r| <= 1/2), 2^r = e^(r ln2) by its degree-11 Taylor polynomial in r with the
// ln2^n/n! folded into the coefficients (truncation < 7e-15 relative), 2^k by ldexp.  In base 2
// the reduction is one exact subtraction (base e needed x log2e and a two-part ln2).
__device__ __forceinline__ double exp2_rr(double y) {
    const double k = __builtin_rint(y);
    const double r = y - k;
    double p = 4.4455382718708116e-10;  // ln2^11 / 11!
    p = fma3(p, r, 7.054911620801123e-09);
    p = fma3(p, r, 1.01780860092397e-07);
    p = fma3(p, r, 1.321548679014431e-06);
    p = fma3(p, r, 1.5252733804059841e-05);
    p = fma3(p, r, 0.0001540353039338161);
    p = fma3(p, r, 0.0013333558146428443);
    p = fma3(p, r, 0.009618129107628477);
    p = fma3(p, r, 0.05550410866482158);
    p = fma3(p, r, 0.24022650695910072);
    p = fma3(p, r, 0.6931471805599453);
    p = fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)k);
}

struct BoldArgs {
    wc_bold_cfg cfg;
    int64_t C, n, M;
    double itaus, itauf, itauo, ialpha, iEo, vo, k1, k2, k3, log2_1mEo;
    double dq_a, dq_b;  // q += dq_a f (1 - fpow) - dq_b q v^(1/alpha - 1): dt itauo iEo, dt itauo
    double bc0, bc1, bc2, bc3;  // BOLD = vo (k1 (1-q) + k2 (1-q/v) + k3 (1-v)) = bc0 - bc1 q - bc2 q/v - bc3 v
    int alpha_3125;  // 1/alpha == 3.125: v^(1/alpha) = v^3 * v^(1/8) by square roots
};

// The (h, G) table is read-only inside wc_bold_chunk, and its row r is wave-uniform.  Read
// through the constant address space it becomes scalar loads (lgkmcnt).  Through the state
// pointer, which the kernel also stores to, it was a vector load issued a few instructions
// before its use.  That load is the youngest in vmcnt, so each sample's wait for it also
// waited for the next batch's prefetched E loads.
typedef const __attribute__((address_space(4))) double* tab_ptr;
__device__ __forceinline__ tab_ptr tab_row(const double* st, const BoldLayout& L, int64_t r) {
    return (tab_ptr)(st + L.tab) + 5 * r;
}

// forward output y of data sample k: accumulate the block's zero-state backward
// summaries; at the block's last sample store them (block m = k / dec)
// (r, m) = (k % dec, k / dec), passed in by the caller's running counters
__device__ __forceinline__ void emit_rm(const BoldArgs& a, const BoldLayout& L, double* st, int64_t c, int64_t k,
                                        int64_t r, int64_t m, double y, double acc[5]) {
    const int64_t dec = a.cfg.dec;
    const tab_ptr tab = tab_row(st, L, r);  // wave-uniform row: scalar loads
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[j] += tab[j] * y;
    if (r == dec - 1 || k == a.n - 1) {
        st[L.yzs + m * L.C + c] = acc[0];
#pragma unroll
        for (int j = 0; j < 4; ++j) st[L.u + (m * 4 + j) * L.C + c] = acc[1 + j];
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[j] = 0.0;
    }
}

__device__ __forceinline__ void emit(const BoldArgs& a, const BoldLayout& L, double* st, int64_t c, int64_t k,
                                     double y, double acc[5]) {
    const int64_t dec = a.cfg.dec;
    const int64_t r = k % dec;
    const tab_ptr tab = tab_row(st, L, r);  // wave-uniform row: scalar loads
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[j] += tab[j] * y;
    if (r == dec - 1 || k == a.n - 1) {
        const int64_t m = k / dec;
        st[L.yzs + m * L.C + c] = acc[0];
#pragma unroll
        for (int j = 0; j < 4; ++j) st[L.u + (m * 4 + j) * L.C + c] = acc[1 + j];
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[j] = 0.0;
    }
}

// E layout: e_ld == 0 -> time-major [Tc][C]; e_ld > 0 -> node-major, sample tt of
// column c at c*e_ld + tt (a slot of the integrator's recording ring)
// One thread per column (the kernel is bound by its fp64 Balloon arithmetic;
// staging a node-major input through LDS for coalescing measured 10% slower).
// COPY: time-major fp32 input, also written out node-major (copy[c*copy_ld + tt])
// through a 256-column x 32-sample LDS tile flushed as 128-B rows.
constexpr int kCopyT = 32;
#ifndef WC_BOLD_PINGPONG
#define WC_BOLD_PINGPONG 1  // the steady loop's two sample batches in static ping-pong buffers (0: one
                            // buffer copied per batch; 1.3% slower, profiles/r03_ab_bold_pp.log)
#endif
#ifndef WC_BOLD_BATCH
#define WC_BOLD_BATCH 16    // samples per load batch (divides kCopyT)
#endif
constexpr int kBat = WC_BOLD_BATCH;
#ifndef WC_BOLD_COPY_WPS
#define WC_BOLD_COPY_WPS 4  // workgroups (of 4 waves) per CU for the steady copy instantiation: 128 VGPRs,
                            // 8 spilled, 6% faster than 3 (tools/ab_multi.sh, profiles/r03_ab_bold.log)
#endif
template <typename ET, bool COPY, bool STEADY, bool BP = false>
__global__ void __launch_bounds__(256, (STEADY && sizeof(ET) == 4) ? (COPY ? WC_BOLD_COPY_WPS : 4) : 1) bold_chunk_kernel(const BoldArgs a, const ET* __restrict__ E, int64_t e_ld,
                                                         int64_t t0, int64_t Tc, double* __restrict__ st,
                                                         float* __restrict__ copy, int64_t copy_ld) {
    const int64_t c0 = (int64_t)blockIdx.x * blockDim.x;
    const int64_t c = c0 + threadIdx.x;
    if (!COPY && c >= a.C) return;
    const bool live = c < a.C;
    const int64_t cc = live ? c : a.C - 1;  // COPY tail threads shadow the last column and never store
    const BoldLayout L(a.C, a.M, a.cfg.dec);
    // per-wave tile (64 columns x 32 samples): each wave transposes its own columns,
    // so the only synchronisation is the wave's own (no workgroup barrier)
    __shared__ float tiles[COPY ? 4 * 64 * (kCopyT + 1) : 1];
    float* tile = tiles + (threadIdx.x >> 6) * 64 * (kCopyT + 1);
    const int lane = threadIdx.x & 63;
    const int64_t w0 = c0 + (threadIdx.x & ~63);  // first column of this wave
    // 16-B row stores when every row start is 16-B aligned, else scalar stores
    const bool vec = COPY && ((uintptr_t)copy & 15) == 0 && copy_ld % 4 == 0;
    // LDS operations of one wave complete in order: a compiler barrier plus an
    // lgkmcnt drain orders the tile's writes and reads (a wavefront-scope release
    // fence would also drain the in-flight row stores: 7 ms per chunk at C3)
    auto wsync = []() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // the wave's rows of the copy through one buffer descriptor (wave-uniform base,
    // 32-bit per-lane offsets): columns past C fall outside its range and the
    // hardware drops their stores, so the row loop carries no column test and no
    // 64-bit addresses (hoisted 64-bit row addresses cost ~100 VGPRs)
    const int64_t w0u = ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)(w0 >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)w0);
    const int64_t ncol = COPY ? (a.C - w0u < 64 ? (a.C > w0u ? a.C - w0u : 0) : 64) : 0;  // 0: no stores
    const __amdgpu_buffer_rsrc_t crs =
        __builtin_amdgcn_make_buffer_rsrc(COPY ? copy + w0u * copy_ld : nullptr, 0, (int)(ncol * copy_ld * 4),
                                          0x00020000);
    auto flush = [&](int64_t tt0, int len) {  // tile samples [tt0, tt0+len) of the wave's columns
        wsync();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = lane + 64 * i, col = q >> 3, part = q & 7;
            const float* srow = tile + col * (kCopyT + 1) + 4 * part;
            const int off = (int)(((int64_t)col * copy_ld + tt0 + 4 * part) * 4);
            if (vec && len == kCopyT) {
                typedef unsigned u4 __attribute__((ext_vector_type(4)));
                const u4 v = {__float_as_uint(srow[0]), __float_as_uint(srow[1]), __float_as_uint(srow[2]),
                              __float_as_uint(srow[3])};
                __builtin_amdgcn_raw_buffer_store_b128(v, crs, off, 0, 0);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * part + k < len) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(srow[k]), crs,
                                                                                   off + 4 * k, 0, 0);
            }
        }
        wsync();
    };
    const double* b = a.cfg.b;
    const double* fa = a.cfg.a;
    double s = st[L.bal + cc], f = st[L.bal + a.C + cc], v = st[L.bal + 2 * a.C + cc], q = st[L.bal + 3 * a.C + cc];
    const int64_t ce = live ? c : a.C - 1;
    double zf[4], acc[5];
#pragma unroll
    for (int k = 0; k < 4; ++k) zf[k] = st[L.zf + k * a.C + cc];
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = st[L.acc + k * a.C + cc];
    const int64_t neq = a.cfg.neq, n = a.n;
    const double dt = a.cfg.dt;
    // (r_blk, m_blk) = ((t - neq) % dec, (t - neq) / dec) of the next sample with
    // t >= neq, advanced by one per sample (no 64-bit division in the loop)
    int64_t r_blk = 0, m_blk = 0;
    {
        const int64_t i0 = t0 - neq;
        if (i0 > 0) {
            r_blk = i0 % a.cfg.dec;
            m_blk = i0 / a.cfg.dec;
        }
    }
    // Balloon-Windkessel: BOLD[t] from the state after t steps, then one Euler step
    // driven by x (see oracle/wc_oracle.c orc_bold)
    auto balloon = [&](double x) -> double {
        double iv, vpow_iv;
        if (STEADY || a.alpha_3125) {  // the host launches STEADY only when 1/alpha == 3.125
            // w = v^(-1/8) from an fp32 seed z (hardware sqrt/rsq, relative error ~3e-7) without
            // a Newton update: with 1 - t = v z^8 (t = O(1e-6)),
            //   1/v     = w^8 = z^8 / (1 - t)       = z^8 (1 + t + t^2 + O(t^3)),
            //   v^(-7/8) = w^7 = z^7 (1 - t)^(-7/8) = z^7 (1 + 7t/8 + 105t^2/128 + O(t^3)),
            // (relative error ~1e-17), v^2.125 = v^3 w^7 and v^3.125 = v v^2.125
            const double z = (double)__builtin_amdgcn_rsqf(__builtin_amdgcn_sqrtf(__builtin_amdgcn_sqrtf((float)v)));
            const double z2 = z * z, z4 = z2 * z2, z8 = z4 * z4;
            const double t = fma(-v, z8, 1.0);
            iv = fma(z8, fma(t, t, t), z8);
            const double z7 = z4 * z2 * z;
            const double w7 = fma(z7, fma(t, 0.8203125, 0.875) * t, z7);
            vpow_iv = v * v * v * w7;  // v^2.125
        } else {
            iv = 1.0 / v;
            vpow_iv = exp(log(v) * a.ialpha) * iv;
        }
        // bc0 - (bc1 q + bc2 q/v + bc3 v): every fma takes ONE uniform (SGPR) operand, so no
        // constant is copied into a VGPR per sample (gfx950 VALU reads one scalar per instruction)
        const double bold = a.bc0 - fma(a.bc1, q, fma(a.bc2, q * iv, a.bc3 * v));
        double rf = (double)__builtin_amdgcn_rcpf((float)f);  // 1/f: fp32 seed + one Newton step (~1e-14)
        rf = fma(rf, fma(-f, rf, 1.0), rf);
        const double fpow = exp2_rr(a.log2_1mEo * rf);  // (1 - E0)^(1/f)
        const double ds = x - a.itaus * s - a.itauf * (f - 1.0);
        // Euler steps with dt folded into the constants (dt itauo, dt itauo iEo):
        //   v += dt (f - v^(1/alpha)) itauo;  q += dt (f (1 - fpow) iEo - q v^(1/alpha - 1)) itauo
        const double vn = fma(a.dq_b, fma(-v, vpow_iv, f), v);
        q = fma(a.dq_a, f * (1.0 - fpow), fma(-a.dq_b, q * vpow_iv, q));
        f += dt * s;  // df = s (the state at the step's start)
        s += dt * ds;
        v = vn;
        return bold;
    };
    // one sample of the stream (x = E at sample tt of this chunk), every case
    auto sample = [&](double x, int64_t tt) {
        const int64_t t = t0 + tt;
        const double bold = balloon(x);
        if (t < neq) return;
        const int64_t i = t - neq;  // data index of this BOLD sample
        const int64_t r_cur = r_blk, m_cur = m_blk;
        if (++r_blk == a.cfg.dec) {
            r_blk = 0;
            ++m_blk;
        }
        if (i >= n) return;
        if (i >= n - 16) st[L.x16 + (i - (n - 16)) * a.C + c] = bold;
        if (i < 16) st[L.head + i * a.C + c] = bold;
        if (i < kPad) return;
        if (i == kPad) {
            // odd extension in front: ext = 2 x0 - x[15..1], then x[0..15]; zi * ext[0]
            const double x0 = st[L.head + c];
            const double e0 = 2.0 * x0 - st[L.head + 15 * a.C + c];
#pragma unroll
            for (int k = 0; k < 4; ++k) zf[k] = a.cfg.zi[k] * e0;
            for (int k = 15; k >= 1; --k) iir_step(zf, 2.0 * x0 - st[L.head + k * a.C + c], b, fa);
            for (int k = 0; k <= 15; ++k) emit(a, L, st, c, k, iir_step(zf, st[L.head + k * a.C + c], b, fa), acc);
        } else {
            emit_rm(a, L, st, c, i, r_cur, m_cur, iir_step(zf, bold, b, fa), acc);
        }
        if (i == n - 1) {
            // odd extension at the end: 2 x[n-1] - x[n-2..n-16]; backward pass starts there
            const double xl = st[L.x16 + 15 * a.C + c];
            double yext[kPad];
#pragma unroll
            for (int k = 0; k < kPad; ++k) yext[k] = iir_step(zf, 2.0 * xl - st[L.x16 + (14 - k) * a.C + c], b, fa);
            double zb[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) zb[k] = a.cfg.zi[k] * yext[kPad - 1];
#pragma unroll
            for (int k = kPad - 1; k >= 0; --k) iir_step(zb, yext[k], b, fa);
#pragma unroll
            for (int k = 0; k < 4; ++k) st[L.zend + k * a.C + c] = zb[k];
        }
    };
    // steady state (16 <= i <= n - 17: no head/tail bookkeeping, no odd extensions):
    // Balloon, forward IIR, block summaries; the block-end store is the only branch
    // (no divergent branch around it: the block counters and the table address stay
    // wave-uniform, in SGPRs; tail lanes of a COPY launch compute on a shadow column
    // and only their stores are masked)
    auto steady = [&](double x, int r, int m) {  // r, m: (block position, block) of the sample (32-bit, SGPRs)
        const double bold = balloon(x);
        const double y = BP ? iir_step_bp(zf, bold, b, fa) : iir_step(zf, bold, b, fa);
        const tab_ptr tab = tab_row(st, L, r);  // wave-uniform row: scalar loads
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[j] += tab[j] * y;
        if (r == (int)a.cfg.dec - 1) {
            if (live) {
                st[L.yzs + (int64_t)m * L.C + c] = acc[0];
#pragma unroll
                for (int j = 0; j < 4; ++j) st[L.u + ((int64_t)m * 4 + j) * L.C + c] = acc[1 + j];
            }
#pragma unroll
            for (int j = 0; j < 5; ++j) acc[j] = 0.0;
        }
    };
    // Samples come in batches of 16, software-pipelined: batch k+1 is loaded while
    // batch k is integrated, so the load latency overlaps the fp64 chain.  With COPY
    // the next batch's loads are also issued BEFORE the previous 32-sample tile's
    // row stores: vmcnt retires in issue order, so a load issued after those stores
    // would wait for them (that ordering cost 7 ms per chunk at C3).
    auto load = [&](ET (&x)[kBat], int64_t tb) {
        if (sizeof(ET) == 4 && e_ld == 0) {
            // time-major fp32: one descriptor per batch (uniform base E + tb*C, the row
            // offset j*C*4 in an SGPR), the lane's column offset in one VGPR
            const int64_t nrow = Tc - tb < kBat ? Tc - tb : kBat;
            const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<ET*>(E) + tb * a.C, 0, (int)(nrow * a.C * 4), 0x00020000);
#pragma unroll
            for (int j = 0; j < kBat; ++j) {
                const int jj = j < nrow ? j : 0;
                const uint32_t u = __builtin_amdgcn_raw_buffer_load_b32(ers, (int)(ce * 4), (int)(jj * a.C * 4), 0);
                x[j] = (ET)__uint_as_float(u);
            }
        } else {
#pragma unroll
            for (int j = 0; j < kBat; ++j) {
                const int64_t tt = tb + j < Tc ? tb + j : tb;
                x[j] = E[e_ld ? ce * e_ld + tt : tt * a.C + ce];
            }
        }
    };
    // STEADY launches cover only 16 <= i <= n - 17 (the host splits the chunk)
    auto process = [&](const ET (&x)[kBat], int64_t tb) {
        const int k0 = (int)(tb % kCopyT);
        if constexpr (COPY) {
            if (k0 == 0 && tb > 0) flush(tb - kCopyT, kCopyT);
        }
        // STEADY: (position in block, block) of the batch's first sample, uniform 32-bit scalars
        // (64-bit inequalities of scalars have no SALU compare and went to the VALU per sample)
        const int64_t ib = t0 + tb - neq;
        const int dec = (int)a.cfg.dec;
        int mb = STEADY ? (int)(ib / dec) : 0, rb = STEADY ? (int)(ib - (int64_t)mb * dec) : 0;
        const int rem = Tc - tb < kBat ? (int)(Tc - tb) : kBat;  // samples of this batch inside the chunk
#pragma unroll
        for (int j = 0; j < kBat; ++j) {
            if constexpr (COPY) tile[lane * (kCopyT + 1) + k0 + j] = (float)x[j];
            if (STEADY) {
                if (j < rem) steady((double)x[j], rb, mb);
                if (++rb == dec) {
                    rb = 0;
                    ++mb;
                }
            } else {
                if (live && tb + j < Tc) sample((double)x[j], tb + j);
            }
        }
    };
    ET xa[kBat];
    load(xa, 0);
#if WC_BOLD_PINGPONG
    if constexpr (STEADY) {
        // two batches per iteration with static buffers: no register copy of in-flight loads (a copy
        // would wait for them, vmcnt retiring in order)
        ET xb[kBat];
        int64_t tb = 0;
        for (; tb + kBat < Tc; tb += 2 * kBat) {
            load(xb, tb + kBat);
            process(xa, tb);
            if (tb + 2 * kBat < Tc) load(xa, tb + 2 * kBat);
            process(xb, tb + kBat);
        }
        if (tb < Tc) process(xa, tb);
    } else
#endif
    for (int64_t tb = 0; tb < Tc; tb += kBat) {
        if (STEADY) {
            ET xb[kBat];
            if (tb + kBat < Tc) load(xb, tb + kBat);
            process(xa, tb);
#pragma unroll
            for (int j = 0; j < kBat; ++j) xa[j] = xb[j];
        } else {
            if (tb > 0) load(xa, tb);
            process(xa, tb);
        }
    }
    if constexpr (COPY) {
        const int64_t last = ((Tc - 1) / kCopyT) * kCopyT;
        flush(last, (int)(Tc - last));
    }
    if (!live) return;
    st[L.bal + c] = s;
    st[L.bal + a.C + c] = f;
    st[L.bal + 2 * a.C + c] = v;
    st[L.bal + 3 * a.C + c] = q;
#pragma unroll
    for (int k = 0; k < 4; ++k) st[L.zf + k * a.C + c] = zf[k];
#pragma unroll
    for (int k = 0; k < 5; ++k) st[L.acc + k * a.C + c] = acc[k];
}

__global__ void bold_init_kernel(int64_t C, double* st) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    st[c] = 0.0;          // s
    st[C + c] = 1.0;      // f
    st[2 * C + c] = 1.0;  // v
    st[3 * C + c] = 1.0;  // q
#pragma unroll
    for (int k = 0; k < 4; ++k) st[4 * C + k * C + c] = 0.0;
    const BoldLayout L(C, 0, 0);
#pragma unroll
    for (int k = 0; k < 5; ++k) st[L.acc + k * C + c] = 0.0;
}

// ---- block combination in the filter's modal basis, double-double ----
// In the DF2T state basis the companion matrix A is violently non-normal
// (|A^1000| ~ 3e7 for this band-pass), so propagating block-boundary states
// as z <- A^L z + u amplifies rounding at every block.  In the eigenbasis
// A = V diag(lam) V^-1 the propagation is a contraction (|lam|^1000 <= 0.1);
// V (cond ~2e7) is only applied through double-double arithmetic, so the
// combination adds nothing above filtfilt's own fp64 rounding noise.
#pragma clang fp contract(off)
struct dd { double hi, lo; };
struct cdd { dd re, im; };
__host__ __device__ inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd quick_two_sum(double a, double b) {
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd dd_add(dd x, dd y) {
    dd s = two_sum(x.hi, y.hi), t = two_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
__host__ __device__ inline dd dd_neg(dd x) { return {-x.hi, -x.lo}; }
__host__ __device__ inline dd dd_mul(dd x, dd y) {
    const double p = x.hi * y.hi;
    double e = fma(x.hi, y.hi, -p);
    e += x.hi * y.lo + x.lo * y.hi;
    return quick_two_sum(p, e);
}
__host__ __device__ inline dd dd_mul_d(dd x, double d) {
    const double p = x.hi * d;
    double e = fma(x.hi, d, -p);
    e += x.lo * d;
    return quick_two_sum(p, e);
}
__host__ __device__ inline cdd cdd_mul(cdd a, cdd b) {
    return {dd_add(dd_mul(a.re, b.re), dd_neg(dd_mul(a.im, b.im))), dd_add(dd_mul(a.re, b.im), dd_mul(a.im, b.re))};
}
__host__ __device__ inline cdd cdd_add(cdd a, cdd b) { return {dd_add(a.re, b.re), dd_add(a.im, b.im)}; }

// (h, G) table of the backward zero-state pass: DF2T impulse response h[k] and
// state G[k] after k zero steps following a unit impulse, in double-double (one thread)
__global__ void bold_table_kernel(const wc_bold_cfg cfg, double* tab) {
    dd z[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
    for (int64_t k = 0; k < cfg.dec; ++k) {
        const double x = k == 0 ? 1.0 : 0.0;
        const dd y = dd_add(z[0], {x * cfg.b[0], 0.0});
        z[0] = dd_add(dd_add(z[1], {x * cfg.b[1], 0.0}), dd_neg(dd_mul_d(y, cfg.a[1])));
        z[1] = dd_add(dd_add(z[2], {x * cfg.b[2], 0.0}), dd_neg(dd_mul_d(y, cfg.a[2])));
        z[2] = dd_add(dd_add(z[3], {x * cfg.b[3], 0.0}), dd_neg(dd_mul_d(y, cfg.a[3])));
        z[3] = dd_add({x * cfg.b[4], 0.0}, dd_neg(dd_mul_d(y, cfg.a[4])));
        tab[5 * k] = y.hi + y.lo;
#pragma unroll
        for (int j = 0; j < 4; ++j) tab[5 * k + 1 + j] = z[j].hi + z[j].lo;
    }
}
__host__ __device__ inline cdd cdd_mul_d(cdd a, double d) { return {dd_mul_d(a.re, d), dd_mul_d(a.im, d)}; }
#pragma clang fp contract(on)

struct FinishArgs {
    int64_t C, M, dec;
    cdd Vi[16];             // V^-1 (row-major)
    cdd lamL[4], lamL1[4];  // lam^dec, lam^(dec-1)
    cdd lamT[4], lamT1[4];  // the same for the last (possibly short) block
};

__global__ void bold_finish_kernel(const FinishArgs f, const double* __restrict__ st, double* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= f.C) return;
    const BoldLayout L(f.C, f.M, f.dec);
    // w = V^-1 z_end
    double z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = st[L.zend + k * f.C + c];
    cdd w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        cdd acc = {{0, 0}, {0, 0}};
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = cdd_add(acc, cdd_mul_d(f.Vi[i * 4 + k], z[k]));
        w[i] = acc;
    }
    for (int64_t m = f.M - 1; m >= 0; --m) {
        const bool last = m == f.M - 1;
        // output at the block start: y_zs + c V lam^(L-1) w, and c V = (1, 1, 1, 1)
        dd y = {st[L.yzs + m * f.C + c], 0.0};
#pragma unroll
        for (int i = 0; i < 4; ++i) y = dd_add(y, cdd_mul(last ? f.lamT1[i] : f.lamL1[i], w[i]).re);
        out[m * f.C + c] = y.hi + y.lo;
        // w <- lam^L w + V^-1 u_m
        double u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = st[L.u + (m * 4 + k) * f.C + c];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            cdd acc = cdd_mul(last ? f.lamT[i] : f.lamL[i], w[i]);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = cdd_add(acc, cdd_mul_d(f.Vi[i * 4 + k], u[k]));
            w[i] = acc;
        }
    }
}

// ---------------- Hilbert phases (utils.kuramoto's hilbert, axis 0) ----------------
// imag(hilbert(x))[t] = sum_tau x[tau] q[(t - tau) mod M],  q[d] = (2/M) sum_{k=1}^{K} sin(2 pi k d / M)
// (K = M/2 - 1 for even M, (M-1)/2 for odd): the analytic signal's real part is
// x itself.  Output: unit phasor (cos, sin) of angle(x + i H) per [t][c].
constexpr int kHilNodes = 8;    // columns per workgroup
constexpr int kHilT = 32;       // time slices per column
__global__ void __launch_bounds__(256) hilbert_phase_kernel(int64_t C, int M, const double* __restrict__ x,
                                                            const double* __restrict__ qk,
                                                            double* __restrict__ ph) {
    extern __shared__ double sq[];  // q[0..M)
    for (int i = threadIdx.x; i < M; i += blockDim.x) sq[i] = qk[i];
    __syncthreads();
    const int lc = threadIdx.x % kHilNodes, ts = threadIdx.x / kHilNodes;
    const int64_t c = (int64_t)blockIdx.x * kHilNodes + lc;
    if (c >= C) return;
    const int per = (M + kHilT - 1) / kHilT;
    const int tb = ts * per, te = min(M, tb + per);
    double acc[16];
    for (int t0 = tb; t0 < te; t0 += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[k] = 0.0;
        for (int tau = 0; tau < M; ++tau) {
            const double xv = x[(int64_t)tau * C + c];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                int d = t0 + k - tau;
                d += d < 0 ? M : 0;
                acc[k] += xv * sq[d < M ? d : 0];
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int t = t0 + k;
            if (t < te) {
                const double re = x[(int64_t)t * C + c];
                const double r = sqrt(re * re + acc[k] * acc[k]);
                ph[((int64_t)t * C + c) * 2] = r > 0 ? re / r : 1.0;  // numpy: angle(0) = 0
                ph[((int64_t)t * C + c) * 2 + 1] = r > 0 ? acc[k] / r : 0.0;
            }
        }
    }
}

// q[d] = (2/M) sum_{k=1}^{K} sin(2 pi k d / M), exact (k d mod M) reduction
__global__ void hilbert_kernel_q(int M, double* q) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= M) return;
    const int K = (M % 2 == 0) ? M / 2 - 1 : (M - 1) / 2;
    double s = 0;
    for (int k = 1; k <= K; ++k) s += sinpi(2.0 * (double)((int64_t)k * d % M) / M);
    q[d] = 2.0 * s / M;
}

// ---------------- per-simulation FC, goodness of fit, mean, Kuramoto ----------------
constexpr int kFcThreads = 256;
constexpr int kMaxN = 96;  // wc_fc_metrics: N <= 96

__device__ double block_sum(double v, double* red) {
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

// Kuramoto order parameter of B groups of N columns: R(t) = |mean_n phasor|,
// out[b] = (mean_t R, std_t R) (utils.py:37-39, np.std ddof 0)
__global__ void __launch_bounds__(256) kuramoto_kernel(int B, int N, int M, const double* __restrict__ ph,
                                                       double* __restrict__ out) {
    __shared__ double red[8];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int64_t C = (int64_t)B * N;
    double r1 = 0;
    for (int t = tid; t < M; t += blockDim.x) {
        double cr = 0, ci = 0;
        const double* p = ph + ((int64_t)t * C + (int64_t)b * N) * 2;
        for (int n = 0; n < N; ++n) {
            cr += p[2 * n];
            ci += p[2 * n + 1];
        }
        r1 += sqrt((cr / N) * (cr / N) + (ci / N) * (ci / N));
    }
    const double sync = block_sum(r1, red) / M;
    double r2 = 0;
    for (int t = tid; t < M; t += blockDim.x) {
        double cr = 0, ci = 0;
        const double* p = ph + ((int64_t)t * C + (int64_t)b * N) * 2;
        for (int n = 0; n < N; ++n) {
            cr += p[2 * n];
            ci += p[2 * n + 1];
        }
        const double R = sqrt((cr / N) * (cr / N) + (ci / N) * (ci / N));
        r2 += (R - sync) * (R - sync);
    }
    const double meta = sqrt(block_sum(r2, red) / M);
    if (tid == 0) {
        out[2 * b] = sync;
        out[2 * b + 1] = meta;
    }
}

struct FcArgs {
    int B, N, M, K;
    const double* bold;   // [M][B][N] band-passed, decimated BOLD (NULL: take fc_in)
    const double* fc_in;  // [B][N][N] precomputed FC (used when bold == NULL)
    const double* emp;    // [K][N][N]
    const double* ph;     // [M][B][N][2] Hilbert phasors (may be NULL)
    double* fc;           // [B][N][N] (may be NULL)
    double* metrics;      // [B][K][4]: corr, euc, ssim, new_metric
    double* extra;        // [B][3]: mean(FC), sync, meta
    double data_range;    // SSIM data range (utils.py:48 passes 1)
};

// LDS: fc[N*N] | emp[N*N] (also the time-chunk staging area before emp is loaded) | red[8]
__global__ void __launch_bounds__(kFcThreads) fc_metrics_kernel(const FcArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = a.N, M = a.M, NN = N * N, NN2 = (NN + 1) & ~1;  // NN2: 16-B aligned areas
    double* fc = lds;
    double* emp = lds + NN2;
    double* red = emp + NN2;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int64_t C = (int64_t)a.B * N;
    const double* xb = a.bold ? a.bold + (int64_t)b * N : nullptr;

    if (!a.bold) {
        for (int i = tid; i < NN; i += blockDim.x) fc[i] = a.fc_in[(int64_t)b * NN + i];
        __syncthreads();
    } else {
    // ---- np.cov: node means, centred cross products, 1/(M-1) ----
    // means: S = kFcThreads / N slices per node (t = h, h + S, ...), combined in slice order
    double* mean = red + 8;        // [N] after red
    double* msl = mean + kMaxN;    // [S][N] slice sums
    const int S = kFcThreads / N;
    if (tid < S * N) {
        const int n = tid % N, h = tid / N;
        double sm = 0;
        for (int t = h; t < M; t += S) sm += xb[(int64_t)t * C + n];
        msl[h * N + n] = sm;
    }
    __syncthreads();
    for (int n = tid; n < N; n += blockDim.x) {
        double sm = 0;
        for (int h = 0; h < S; ++h) sm += msl[h * N + n];
        mean[n] = sm / M;
    }
    __syncthreads();
    // cross products as 4 x 4 register tiles of the (padded) upper triangle: per sample
    // a tile reads 2 x 4 centred values (4 ds_read_b128) for 16 FMAs; every (i, j) still
    // sums its samples in time order.  Time is staged through LDS (emp area).
    const int Np = (N + 3) & ~3, NB = Np / 4;
    const int ntiles = NB * (NB + 1) / 2;
    constexpr int kMaxTiles = ((kMaxN / 4) * (kMaxN / 4 + 1) / 2 + kFcThreads - 1) / kFcThreads;  // 2
    double acc[kMaxTiles][4][4];
    int ti[kMaxTiles], tj[kMaxTiles];
#pragma unroll
    for (int k = 0; k < kMaxTiles; ++k) {
        const int p = min(tid + k * kFcThreads, ntiles - 1);
        // p -> (bi, bj), bi <= bj, row-major over the upper triangle of NB x NB blocks
        int bi = (int)((2 * NB + 1 - sqrt((double)(2 * NB + 1) * (2 * NB + 1) - 8.0 * p)) / 2);
        while (bi > 0 && bi * (2 * NB - bi + 1) / 2 > p) --bi;
        while ((bi + 1) * (2 * NB - bi) / 2 <= p) ++bi;
        ti[k] = 4 * bi;
        tj[k] = 4 * (bi + (p - bi * (2 * NB - bi + 1) / 2));
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[k][r][q] = 0.0;
    }
    const int TCH = NN / Np;  // time samples per staging chunk (N*N doubles of room)
    for (int t0 = 0; t0 < M; t0 += TCH) {
        const int tn = min(TCH, M - t0);
        for (int i = tid; i < tn * Np; i += blockDim.x) {
            const int tt = i / Np, n = i % Np;
            emp[i] = n < N ? xb[(int64_t)(t0 + tt) * C + n] - mean[n] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kMaxTiles; ++k) {
            if (tid + k * kFcThreads < ntiles) {
                for (int tt = 0; tt < tn; ++tt) {
                    const double2* row = reinterpret_cast<const double2*>(emp + tt * Np);
                    const double2 a0 = row[ti[k] / 2], a1 = row[ti[k] / 2 + 1];
                    const double2 b0 = row[tj[k] / 2], b1 = row[tj[k] / 2 + 1];
                    const double xi[4] = {a0.x, a0.y, a1.x, a1.y}, xj[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[k][r][q] += xi[r] * xj[q];
                }
            }
        }
        __syncthreads();
    }
    const double fact = 1.0 / (M - 1);
#pragma unroll
    for (int k = 0; k < kMaxTiles; ++k) {
        if (tid + k * kFcThreads < ntiles) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = ti[k] + r, j = tj[k] + q;
                    if (i < N && j < N && i <= j) {
                        const double cv = acc[k][r][q] * fact;
                        fc[i * N + j] = cv;
                        fc[j * N + i] = cv;
                    }
                }
        }
    }
    __syncthreads();
    // ---- corrcoef: c /= sd[:,None]; c /= sd[None,:]; clip to [-1, 1] ----
    double* sd = emp;  // reuse
    for (int n = tid; n < N; n += blockDim.x) sd[n] = sqrt(fc[n * N + n]);
    __syncthreads();
    for (int i = tid; i < NN; i += blockDim.x) {
        const int r = i / N, q = i % N;
        double v = fc[i] / sd[r];
        v = v / sd[q];
        fc[i] = fmin(1.0, fmax(-1.0, v));
    }
    __syncthreads();
    }
    if (a.fc)
        for (int i = tid; i < NN; i += blockDim.x) a.fc[(int64_t)b * NN + i] = fc[i];
    // ---- mean(sFC) over all N^2 entries ----
    double s = 0;
    for (int i = tid; i < NN; i += blockDim.x) s += fc[i];
    const double fcmean = block_sum(s, red) / NN;

    // ---- goodness of fit against each empirical FC ----
    const int nflat = N * (N - 1) / 2;
    const int P = N - 6;  // SSIM interior (crop (7-1)/2 on each side)
    for (int k = 0; k < a.K; ++k) {
        for (int i = tid; i < NN; i += blockDim.x) emp[i] = a.emp[(int64_t)k * NN + i];
        __syncthreads();
        // flat upper triangles: means, then centred sums (np.corrcoef of two vectors)
        double sx = 0, sy = 0;
        for (int p = tid; p < NN; p += blockDim.x) {
            const int r = p / N, q = p % N;
            if (q > r) { sx += fc[p]; sy += emp[p]; }
        }
        const double mx = block_sum(sx, red) / nflat;
        const double my = block_sum(sy, red) / nflat;
        double sxx = 0, syy = 0, sxy = 0, see = 0;
        for (int p = tid; p < NN; p += blockDim.x) {
            const int r = p / N, q = p % N;
            if (q > r) {
                const double dx = fc[p] - mx, dy = emp[p] - my, de = emp[p] - fc[p];
                sxx += dx * dx;
                syy += dy * dy;
                sxy += dx * dy;
                see += de * de;
            }
        }
        sxx = block_sum(sxx, red);
        syy = block_sum(syy, red);
        sxy = block_sum(sxy, red);
        see = block_sum(see, red);
        const double f1 = 1.0 / (nflat - 1);
        double corr = (sxy * f1) / sqrt(sxx * f1) / sqrt(syy * f1);
        corr = fmin(1.0, fmax(-1.0, corr));
        const double euc = sqrt(see);
        const double newm = 1.0 - corr + (mx - my) * (mx - my);
        // SSIM (skimage 0.18 defaults): 7x7 uniform filter of x, y, xx, yy, xy
        // (row sums /7 then column sums /7), sample covariance 49/48, mean of the
        // interior P x P map.  Thread = (output column, row band).
        double ssum = 0;
        const int nbands = (int)blockDim.x / P;
        const int jcol = tid % P, band = tid / P;
        if (band < nbands) {
            const int j = jcol + 3;
            const int r0 = 3 + (P * band) / nbands, r1 = 3 + (P * (band + 1)) / nbands;
            const double C1 = (0.01 * a.data_range) * (0.01 * a.data_range),
                         C2 = (0.03 * a.data_range) * (0.03 * a.data_range), cov_norm = 49.0 / 48.0;
            for (int i = r0; i < r1; ++i) {
                double vx = 0, vy = 0, vxx = 0, vyy = 0, vxy = 0;
                for (int di = -3; di <= 3; ++di) {
                    const int r = i + di;
                    double hx = 0, hy = 0, hxx = 0, hyy = 0, hxy = 0;
                    for (int dj = -3; dj <= 3; ++dj) {
                        const double xv = fc[r * N + j + dj], yv = emp[r * N + j + dj];
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
        }
        const double ssim = block_sum(ssum, red) / ((double)P * P);
        if (tid == 0) {
            double* o = a.metrics + ((int64_t)b * a.K + k) * 4;
            o[0] = corr;
            o[1] = euc;
            o[2] = ssim;
            o[3] = newm;
        }
        __syncthreads();
    }
    // ---- Kuramoto order parameter R(t) = |mean_n exp(i theta_n(t))|: mean and std ----
    double sync = 0, meta = 0;
    if (a.ph) {
        double r1 = 0, r2 = 0;
        for (int t = tid; t < M; t += blockDim.x) {
            double cr = 0, ci = 0;
            const double* p = a.ph + ((int64_t)t * C + (int64_t)b * N) * 2;
            for (int n = 0; n < N; ++n) {
                cr += p[2 * n];
                ci += p[2 * n + 1];
            }
            cr /= N;
            ci /= N;
            const double R = sqrt(cr * cr + ci * ci);
            r1 += R;
            emp[t] = R;  // emp is free now
        }
        sync = block_sum(r1, red) / M;
        for (int t = tid; t < M; t += blockDim.x) r2 += (emp[t] - sync) * (emp[t] - sync);
        meta = sqrt(block_sum(r2, red) / M);
    }
    if (tid == 0) {
        a.extra[b * 3 + 0] = fcmean;
        a.extra[b * 3 + 1] = sync;
        a.extra[b * 3 + 2] = meta;
    }
}

// ---- host: poles, eigenvectors and their inverse in long double ----
typedef std::complex<long double> cld;

cdd to_cdd(cld x) {
    const long double r = x.real(), i = x.imag();
    const double rh = (double)r, ih = (double)i;
    return {{rh, (double)(r - rh)}, {ih, (double)(i - ih)}};
}

// roots of z^4 + a1 z^3 + a2 z^2 + a3 z + a4 (Durand-Kerner, then Newton polish)
void poles(const double* a, cld lam[4]) {
    auto P = [&](cld z) { return (((z + (long double)a[1]) * z + (long double)a[2]) * z + (long double)a[3]) * z + (long double)a[4]; };
    auto dP = [&](cld z) { return ((4.0L * z + 3.0L * (long double)a[1]) * z + 2.0L * (long double)a[2]) * z + (long double)a[3]; };
    const cld seed(0.4L, 0.9L);
    cld r[4] = {1.0L, seed, seed * seed, seed * seed * seed};
    for (int it = 0; it < 2000; ++it) {
        long double delta = 0;
        for (int i = 0; i < 4; ++i) {
            cld den = 1.0L;
            for (int j = 0; j < 4; ++j)
                if (j != i) den *= (r[i] - r[j]);
            const cld d = P(r[i]) / den;
            r[i] -= d;
            delta = std::max(delta, std::abs(d));
        }
        if (delta < 1e-30L) break;
    }
    for (int i = 0; i < 4; ++i)
        for (int it = 0; it < 5; ++it) r[i] -= P(r[i]) / dP(r[i]);
    for (int i = 0; i < 4; ++i) lam[i] = r[i];
}

// V[:, i] = (1, lam+a1, lam^2+a1 lam+a2, lam^3+a1 lam^2+a2 lam+a3) is the
// eigenvector of the DF2T companion (A[k][0] = -a[k+1], A[k][k+1] = 1); invert it
bool modal_inverse(const double* a, const cld lam[4], cld Vi[16]) {
    cld M[4][8];
    for (int i = 0; i < 4; ++i) {
        const cld l = lam[i];
        const cld v1 = l + (long double)a[1], v2 = l * v1 + (long double)a[2], v3 = l * v2 + (long double)a[3];
        const cld col[4] = {1.0L, v1, v2, v3};
        for (int r = 0; r < 4; ++r) M[r][i] = col[r];
    }
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) M[r][4 + k] = (r == k) ? 1.0L : 0.0L;
    for (int col = 0; col < 4; ++col) {
        int piv = col;
        for (int r = col + 1; r < 4; ++r)
            if (std::abs(M[r][col]) > std::abs(M[piv][col])) piv = r;
        if (std::abs(M[piv][col]) == 0) return false;
        for (int k = 0; k < 8; ++k) std::swap(M[col][k], M[piv][k]);
        const cld d = M[col][col];
        for (int k = 0; k < 8; ++k) M[col][k] /= d;
        for (int r = 0; r < 4; ++r)
            if (r != col) {
                const cld fct = M[r][col];
                for (int k = 0; k < 8; ++k) M[r][k] -= fct * M[col][k];
            }
    }
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) Vi[r * 4 + k] = M[r][4 + k];
    return true;
}

cld cpow_int(cld x, int64_t p) {
    cld r = 1.0L;
    while (p > 0) {
        if (p & 1) r *= x;
        x *= x;
        p >>= 1;
    }
    return r;
}

int check_cfg(const wc_bold_cfg* cfg, int64_t C) {
    if (!cfg || C <= 0 || cfg->dec <= 0 || cfg->neq < 0 || cfg->n_total - cfg->neq < 16)
        return wc_set_err(WC_EINVAL, "wc_bold: invalid configuration (need n_total - neq >= 16)");
    if (cfg->a[0] != 1.0) return wc_set_err(WC_EINVAL, "wc_bold: a[0] must be 1");
    return WC_OK;
}

template <typename ET, bool COPY>
void launch_chunk(bool steady, bool bp, dim3 g, hipStream_t st, const BoldArgs& a, const ET* e, int64_t e_ld,
                  int64_t t0, int64_t len, double* state, float* c, int64_t copy_ld) {
    if (!steady)
        hipLaunchKernelGGL((bold_chunk_kernel<ET, COPY, false, false>), g, dim3(256), 0, st, a, e, e_ld, t0, len, state,
                           c, copy_ld);
    else if (bp)
        hipLaunchKernelGGL((bold_chunk_kernel<ET, COPY, true, true>), g, dim3(256), 0, st, a, e, e_ld, t0, len, state,
                           c, copy_ld);
    else
        hipLaunchKernelGGL((bold_chunk_kernel<ET, COPY, true, false>), g, dim3(256), 0, st, a, e, e_ld, t0, len, state,
                           c, copy_ld);
}

BoldArgs make_bold_args(const wc_bold_cfg* cfg, int64_t C) {
    BoldArgs a;
    a.cfg = *cfg;
    a.C = C;
    a.n = cfg->n_total - cfg->neq;
    a.M = (a.n + cfg->dec - 1) / cfg->dec;
    // Balloon-Windkessel constants (assumed BD.Sim; DESIGN.md "BOLD model")
    a.itaus = 1.0 / 0.65;
    a.itauf = 1.0 / 0.41;
    a.itauo = 1.0 / 0.98;
    a.ialpha = 1.0 / 0.32;
    a.alpha_3125 = a.ialpha == 3.125;
    a.iEo = 1.0 / 0.4;
    a.vo = 0.04;
    const double Eo = 0.4;
    a.k1 = 7.0 * Eo;
    a.k2 = 2.0;
    a.k3 = 2.0 * Eo - 0.2;
    a.log2_1mEo = log2(1.0 - Eo);
    a.dq_b = cfg->dt * a.itauo;
    a.dq_a = cfg->dt * a.itauo * a.iEo;
    a.bc0 = a.vo * (a.k1 + a.k2 + a.k3);
    a.bc1 = a.vo * a.k1;
    a.bc2 = a.vo * a.k2;
    a.bc3 = a.vo * a.k3;
    return a;
}

}  // namespace

extern "C" {

int64_t wc_bold_blocks(const wc_bold_cfg* cfg) {
    if (!cfg || cfg->dec <= 0 || cfg->n_total <= cfg->neq) return 0;
    return (cfg->n_total - cfg->neq + cfg->dec - 1) / cfg->dec;
}

size_t wc_bold_state_doubles(const wc_bold_cfg* cfg, int64_t C) {
    if (!cfg || cfg->dec <= 0 || C <= 0) return 0;
    return (size_t)BoldLayout(C, wc_bold_blocks(cfg), cfg->dec).total;
}

int wc_bold_init(const wc_bold_cfg* cfg, int64_t C, double* state, void* stream) {
    wc_clear_err();
    int rc = check_cfg(cfg, C);
    if (rc) return rc;
    if (!state) return wc_set_err(WC_EINVAL, "wc_bold_init: NULL state");
    hipLaunchKernelGGL(bold_init_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), C, state);
    const BoldLayout L(C, wc_bold_blocks(cfg), cfg->dec);
    hipLaunchKernelGGL(bold_table_kernel, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), *cfg,
                       state + L.tab);
    return wc_hip_check("wc_bold_init");
}

int wc_bold_chunk(const wc_bold_cfg* cfg, int64_t C, const void* E, int e_f64, int64_t e_ld, int64_t t0,
                  int64_t Tc, double* state, void* copy, int64_t copy_ld, void* stream) {
    wc_clear_err();
    int rc = check_cfg(cfg, C);
    if (rc) return rc;
    if (!E || !state || t0 < 0 || Tc < 0 || t0 + Tc > cfg->n_total || e_ld < 0 || (e_ld > 0 && e_ld < Tc))
        return wc_set_err(WC_EINVAL, "wc_bold_chunk: bad E/state/t0/Tc");
    if (Tc == 0) return WC_OK;
    const BoldArgs a = make_bold_args(cfg, C);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((C + 255) / 256));
    if (copy && (e_f64 || e_ld != 0 || copy_ld < Tc))
        return wc_set_err(WC_EINVAL, "wc_bold_chunk: copy needs fp32 time-major E and copy_ld >= Tc");
    // 32-bit buffer offsets: 16 rows of fp32 time-major E, 64 rows of the copy
    if ((!e_f64 && e_ld == 0 && C > (INT32_MAX / 64)) || (copy && copy_ld > INT32_MAX / 256))
        return wc_set_err(WC_EINVAL, "wc_bold_chunk: C or copy_ld too large for 32-bit buffer offsets");
    float* cp = static_cast<float*>(copy);
    // split [t0, t0+Tc) into the steady range (data index 16 <= i <= n-17: Balloon,
    // IIR and block sums only) and the rest (pre-equilibration samples, the head
    // with the front odd extension, the tail with the back one)
    const int64_t n = cfg->n_total - cfg->neq;
    const int64_t ts = std::max(t0, cfg->neq + 16), te = std::min(t0 + Tc, cfg->neq + n - 16);
    const bool steady_ok = a.alpha_3125 != 0;           // the STEADY balloon assumes 1/alpha == 3.125
    const bool bp = cfg->b[1] == 0.0 && cfg->b[3] == 0.0;  // band-pass zeros at +-1 (b = b0 (1,0,-2,0,1))
    auto seg = [&](int64_t s0, int64_t len, bool steady) {
        if (len <= 0) return;
        if (e_f64) {
            launch_chunk<double, false>(steady, bp, grid, st, a, static_cast<const double*>(E) + (e_ld ? s0 : s0 * C),
                                        e_ld, t0 + s0, len, state, nullptr, copy_ld);
        } else {
            const float* e = static_cast<const float*>(E) + (e_ld ? s0 : s0 * C);
            if (cp)
                launch_chunk<float, true>(steady, bp, grid, st, a, e, e_ld, t0 + s0, len, state, cp + s0, copy_ld);
            else
                launch_chunk<float, false>(steady, bp, grid, st, a, e, e_ld, t0 + s0, len, state, nullptr, copy_ld);
        }
    };
    if (steady_ok && ts < te) {
        seg(0, ts - t0, false);
        seg(ts - t0, te - ts, true);
        seg(te - t0, t0 + Tc - te, false);
    } else {
        seg(0, Tc, false);
    }
    return wc_hip_check("wc_bold_chunk");
}

int wc_bold_finish(const wc_bold_cfg* cfg, int64_t C, const double* state, double* out, void* stream) {
    wc_clear_err();
    int rc = check_cfg(cfg, C);
    if (rc) return rc;
    if (!state || !out) return wc_set_err(WC_EINVAL, "wc_bold_finish: NULL argument");
    FinishArgs f;
    f.C = C;
    f.dec = cfg->dec;
    const int64_t n = cfg->n_total - cfg->neq;
    f.M = (n + cfg->dec - 1) / cfg->dec;
    const int64_t Llast = n - (f.M - 1) * cfg->dec;
    cld lam[4], Vi[16];
    poles(cfg->a, lam);
    if (!modal_inverse(cfg->a, lam, Vi)) return wc_set_err(WC_EINVAL, "wc_bold_finish: degenerate filter");
    for (int i = 0; i < 16; ++i) f.Vi[i] = to_cdd(Vi[i]);
    if (getenv("WCSDE_DEBUG")) {
        fprintf(stderr, "wc_bold_finish: a = %.17g %.17g %.17g %.17g %.17g dec=%lld M=%lld C=%lld\n", cfg->a[0],
                cfg->a[1], cfg->a[2], cfg->a[3], cfg->a[4], (long long)cfg->dec, (long long)f.M, (long long)C);
        for (int i = 0; i < 4; ++i)
            fprintf(stderr, "  lam[%d] = %.20Lg %.20Lg   Vi[%d][0] = %Lg %Lg\n", i, lam[i].real(), lam[i].imag(), i,
                    Vi[i * 4].real(), Vi[i * 4].imag());
    }
    for (int i = 0; i < 4; ++i) {
        f.lamL[i] = to_cdd(cpow_int(lam[i], cfg->dec));
        f.lamL1[i] = to_cdd(cpow_int(lam[i], cfg->dec - 1));
        f.lamT[i] = to_cdd(cpow_int(lam[i], Llast));
        f.lamT1[i] = to_cdd(cpow_int(lam[i], Llast - 1));
    }
    hipLaunchKernelGGL(bold_finish_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), f, state, out);
    return wc_hip_check("wc_bold_finish");
}

int wc_hilbert_phase(int64_t C, int M, const double* x, double* phasor, void* workspace, size_t ws_bytes,
                     void* stream) {
    wc_clear_err();
    if (C <= 0 || M <= 1 || !x || !phasor) return wc_set_err(WC_EINVAL, "wc_hilbert_phase: bad arguments");
    if (!workspace || ws_bytes < (size_t)M * sizeof(double))
        return wc_set_err(WC_EWORKSPACE, "wc_hilbert_phase: workspace < M doubles");
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(hilbert_kernel_q, dim3((M + 255) / 256), dim3(256), 0, st, M, static_cast<double*>(workspace));
    const unsigned blocks = (unsigned)((C + kHilNodes - 1) / kHilNodes);
    hipLaunchKernelGGL(hilbert_phase_kernel, dim3(blocks), dim3(kHilNodes * kHilT), M * sizeof(double), st, C, M, x,
                       static_cast<const double*>(workspace), phasor);
    return wc_hip_check("wc_hilbert_phase");
}

int wc_kuramoto(int B, int N, int M, const double* phasor, double* out, void* stream) {
    wc_clear_err();
    if (B <= 0 || N <= 0 || M <= 0 || !phasor || !out) return wc_set_err(WC_EINVAL, "wc_kuramoto: bad arguments");
    hipLaunchKernelGGL(kuramoto_kernel, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream), B, N, M, phasor, out);
    return wc_hip_check("wc_kuramoto");
}

size_t wc_fc_metrics_workspace_size(int B, int N, int M, int K, int want_fc) {
    if (B <= 0 || N <= kMaxN || M < 2 || K < 0) return 0;  // N <= 96: everything in LDS
    return wc_large_fc_metrics_workspace_size(B, N, K, !want_fc) + 2 * (size_t)B * sizeof(double);
}

int wc_fc_metrics(int B, int N, int M, const double* bold, const double* fc_in, const double* empfc, int K,
                  double data_range, const double* phasor, double* fc_out, double* metrics, double* extra,
                  void* workspace, size_t ws_bytes, void* stream) {
    wc_clear_err();
    if (B <= 0 || N < 7 || M < 2 || K < 0 || (!bold && !fc_in) || !extra || (K > 0 && (!empfc || !metrics)))
        return wc_set_err(WC_EINVAL, "wc_fc_metrics: bad arguments (N >= 7)");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (N > kMaxN) {
        const size_t need = wc_fc_metrics_workspace_size(B, N, M, K, fc_out != nullptr);
        if (!workspace || ws_bytes < need)
            return wc_set_err(WC_EWORKSPACE, "wc_fc_metrics: workspace < wc_fc_metrics_workspace_size() for N > 96");
        double* kur = nullptr;
        if (phasor) {
            kur = reinterpret_cast<double*>(static_cast<char*>(workspace) + need) - 2 * (size_t)B;
            hipLaunchKernelGGL(kuramoto_kernel, dim3(B), dim3(256), 0, st, B, N, M, phasor, kur);
        }
        return wc_large_fc_metrics(B, N, M, bold, fc_in, empfc, K, data_range, kur, fc_out, metrics, extra, workspace,
                                   need - 2 * (size_t)B * sizeof(double), st);
    }
    FcArgs a{B, N, M, K, bold, fc_in, empfc, phasor, fc_out, metrics, extra, data_range};
    const size_t lds = (size_t)(2 * ((N * N + 1) & ~1) + 8 + kMaxN + kFcThreads) * sizeof(double);
    hipError_t e = hipFuncSetAttribute((const void*)fc_metrics_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    hipLaunchKernelGGL(fc_metrics_kernel, dim3(B), dim3(kFcThreads), lds, st, a);
    return wc_hip_check("wc_fc_metrics");
}

}  // extern "C"
