// wc_device.h -- device helpers shared by the Wilson-Cowan integrators (gfx950):
// the Philox4x32-10 noise stream of include/wcsde.h, Box-Muller normals,
// precision traits (sigmoid, MFMA), the 3-way bf16 split and the compensated
// a_ie accumulator.  Both wc_sde.hip (N <= 96, register-resident) and
// wc_sde_large.hip (N > 96, one launch per step) draw the SAME normals for a
// given (key, step, node), so the two paths integrate the same stochastic
// trajectory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/wcsde.h"

namespace wcdev {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// ---------------- noise: Philox4x32-10 (must match oracle/wc_oracle.c) ----------------
// key = (WC_PHILOX_KEY0, WC_PHILOX_KEY1) for every simulation (wave-uniform: the
// key schedule lives in SGPRs); counter = (step lo32, (step hi16 << 16) | quad,
// simkey lo32, simkey hi32).  Outputs feed two Box-Muller pairs -> the standard
// normals of nodes 4*quad + 0..3.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// one v_mad_u64_u32 for hi:lo.  Written in C, not inline asm: the compiler picks the carry-out
// SGPR pair itself, whereas an asm block writing vcc got an s_nop after every multiply (18 per
// wave-step in the C3 integrator)
__device__ __forceinline__ void mul_wide(uint32_t a, uint32_t m, uint32_t& hi, uint32_t& lo) {
    const uint64_t r = (uint64_t)a * (uint64_t)m;
    hi = (uint32_t)(r >> 32);
    lo = (uint32_t)r;
}

__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
    uint32_t k0 = WC_PHILOX_KEY0, k1 = WC_PHILOX_KEY1;
    // round 1: c0 (the step) is wave-uniform -> scalar multiply
    {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = xor3(hi1, c1, k0);
        c1 = lo1;
        c2 = xor3(hi0, c3, k1);
        c3 = lo0;
    }
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
        uint32_t hi0, lo0, hi1, lo1;
        mul_wide(c0, 0xD2511F53u, hi0, lo0);
        mul_wide(c2, 0xCD9E8D57u, hi1, lo1);
        c0 = xor3(hi1, c1, k0);
        c1 = lo1;
        c2 = xor3(hi0, c3, k1);
        c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ void philox_ctr(uint64_t step, uint32_t quad, uint64_t simkey, uint32_t out[4]) {
    philox((uint32_t)step, ((uint32_t)(step >> 32) << 16) | quad, (uint32_t)simkey, (uint32_t)(simkey >> 32),
           out);
}

// u = (2*(x>>9)+1) * 2^-24, exact in fp32 and fp64, in (0,1)
__device__ __forceinline__ float u01f(uint32_t x) { return (float)(2u * (x >> 9) + 1u) * 5.9604644775390625e-8f; }
__device__ __forceinline__ double u01d(uint32_t x) { return (double)(2u * (x >> 9) + 1u) * 5.9604644775390625e-8; }

// the same u as u01f in two VALU ops: (1 + m 2^-23) - (1 - 2^-24) = (2m + 1) 2^-24
// exactly (Sterbenz; the result is an odd multiple of 2^-24 below 1: 24 bits).  The
// bits of 1 + m 2^-23 are one funnel shift: ({0x7F, x} >> 9) = 0x3F800000 | (x >> 9)
__device__ __forceinline__ float u01f_fast(uint32_t x) {
    return __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, x, 9u)) - 0.99999994039535522461f;
}

// fp32, unscaled: z / sqrt(2 ln 2) = sqrt(-log2 u0) (cos, sin)(2 pi u1) -- the caller
// folds sqrt(2 ln 2) into its noise scale.  Hardware transcendentals; v_sin/v_cos
// take revolutions; inputs are never denormal (u >= 2^-24).
constexpr float kSqrt2Ln2 = 1.1774100225154747f;
__device__ __forceinline__ void quad_normals_raw(uint64_t step, uint32_t q, uint64_t key, float z[4]) {
    uint32_t x[4];
    philox_ctr(step, q, key, x);
    const float r0 = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u01f_fast(x[0])));
    const float r1 = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u01f_fast(x[2])));
    const float a0 = u01f_fast(x[1]), a1 = u01f_fast(x[3]);
    z[0] = r0 * __builtin_amdgcn_cosf(a0);
    z[1] = r0 * __builtin_amdgcn_sinf(a0);
    z[2] = r1 * __builtin_amdgcn_cosf(a1);
    z[3] = r1 * __builtin_amdgcn_sinf(a1);
}

// packed fp32 pair (v_pk_fma/mul/add_f32: two cells per instruction, each rounded like its scalar form)
typedef float f2v __attribute__((ext_vector_type(2)));

// quad_normals_raw with the radius products packed: (z0, z1), (z2, z3) -- the same bits
__device__ __forceinline__ void quad_normals_pk(uint64_t step, uint32_t q, uint64_t key, f2v z[2]) {
    uint32_t x[4];
    philox_ctr(step, q, key, x);
    const float r0 = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u01f_fast(x[0])));
    const float r1 = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u01f_fast(x[2])));
    const float a0 = u01f_fast(x[1]), a1 = u01f_fast(x[3]);
    z[0] = f2v{__builtin_amdgcn_cosf(a0), __builtin_amdgcn_sinf(a0)} * r0;
    z[1] = f2v{__builtin_amdgcn_cosf(a1), __builtin_amdgcn_sinf(a1)} * r1;
}

// fp32 standard normals (test hook, N > 96 path)
__device__ __forceinline__ void quad_normals(uint64_t step, uint32_t q, uint64_t key, float z[4]) {
    quad_normals_raw(step, q, key, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] *= kSqrt2Ln2;
}
template <typename Coef>
__device__ __forceinline__ void quad_normals(uint64_t step, uint32_t q, uint64_t key, float z[4], Coef) {
    quad_normals(step, q, key, z);
}

// ---------------- fp64 elementary functions for the parity path ----------------
// Straight-line forms for the inputs this build produces (no special cases, no tables), each
// within 2 ulp of an 80-bit reference over its whole input domain (tests/test_f64m_gpu.py, through
// the diagnostic build's wc_diag_f64m);
// ocml's general exp / log / sincospi and the IEEE division sequence took about half of the fp64
// integrator's VALU.  Coefficients: Taylor series, their truncation below 5e-18 relative.
namespace f64m {
// The coefficients, indexed: exp2 [0, 13), log [13, 25) (the last two ln 2 hi and lo), sqrt 2 [25],
// sin [26, 35), cos [35, 44).  Two ways to read them (the Coef parameter of each function):
// LitCoef folds them into the code as literals; TabCoef reads them from kCoefDev through a pointer
// the fp64 integrator launders once per step, so they are scalar loads next to their uses: as
// literals all ~44 fp64 coefficients are hoisted out of its step loop into ~88 SGPRs and push the
// kernel's own scalars into VGPR-lane spills re-read by v_readlane every step.
// One list, two arrays (the literal and the table forms cannot drift apart); kCoefDev has internal
// linkage, one copy per translation unit that uses it.
#define WC_F64M_COEFS \
    1.3691488853904128e-12, 2.5678435993488206e-11, 4.4455382718708116e-10, 7.054911620801123e-09, \
    1.01780860092397e-07, 1.321548679014431e-06, 1.5252733804059841e-05, 0.0001540353039338161, \
    0.0013333558146428443, 0.009618129107628477, 0.05550410866482158, 0.24022650695910072, 0.6931471805599453, \
    0.09523809523809523, 0.10526315789473684, 0.11764705882352941, 0.13333333333333333, 0.15384615384615385, \
    0.18181818181818182, 0.2222222222222222, 0.2857142857142857, 0.4, 0.6666666666666666, \
    6.93147180369123816490e-01, 1.90821492927058770002e-10, \
    1.4142135623730951, \
    7.952054001475513e-07, -2.1915353447830217e-05, 0.00046630280576761255, -0.0073704309457143504, \
    0.08214588661112823, -0.5992645293207921, 2.5501640398773455, -5.16771278004997, 3.141592653589793, \
    -1.3878952462213771e-07, 4.303069587032947e-06, -0.0001046381049248457, 0.0019295743094039231, \
    -0.02580689139001406, 0.2353306303588932, -1.3352627688545895, 4.0587121264167685, -4.934802200544679
constexpr double kCoef[44] = {WC_F64M_COEFS};
static __constant__ double kCoefDev[44] = {WC_F64M_COEFS};
#undef WC_F64M_COEFS
enum : int { kExp = 0, kLog = 13, kLn2Hi = 23, kLn2Lo = 24, kSqrt2 = 25, kSin = 26, kCos = 35 };
struct LitCoef {
    __device__ constexpr double operator[](int i) const { return kCoef[i]; }
    __device__ constexpr LitCoef fresh() const { return *this; }
};
typedef __attribute__((address_space(4))) const double* coef_ptr;  // constant address space: scalar loads
struct TabCoef {
    coef_ptr p;
    __device__ double operator[](int i) const { return p[i]; }
    // a fresh copy of the pointer per function call: its loads cannot be merged with another call's
    // (each call's coefficients live only in that call)
    __device__ TabCoef fresh() const {
        coef_ptr q = p;
        asm volatile("" : "+s"(q));
        return TabCoef{q};
    }
};
// TabCoef over kCoefDev with the pointer laundered here (call once per loop iteration)
__device__ __forceinline__ TabCoef tab_coef() {
    coef_ptr p = (coef_ptr)kCoefDev;
    asm volatile("" : "+s"(p));
    return TabCoef{p};
}

// 2^t, |t| <= 1000: t = n + r, |r| <= 1/2, e^(r ln 2) to degree 13, scaled by 2^n
template <typename Coef = LitCoef>
__device__ __forceinline__ double exp2(double t, Coef c0 = Coef{}) {
    const Coef c = c0;
    t = __builtin_fmin(__builtin_fmax(t, -1000.0), 1000.0);
    const double n = __builtin_rint(t);
    const double r = t - n;  // exact
    double p = c[kExp];
#pragma unroll
    for (int i = 1; i < 13; ++i) p = __builtin_fma(p, r, c[kExp + i]);
    p = __builtin_fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)n);
}
// 1 / d for a normal positive d: the hardware seed and two Newton steps
__device__ __forceinline__ double rcp(double d) {
    double x = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, x, 1.0);
    x = __builtin_fma(x, e, x);
    e = __builtin_fma(-d, x, 1.0);
    return __builtin_fma(x, e, x);
}
// sqrt(x) for a normal positive x (the Box-Muller radius: -2 ln u in [2^-23, 34]): the hardware
// reciprocal square root and Newton-Raphson on (sqrt, 1/(2 sqrt)) -- the device library's sequence
// without its denormal scaling and special-value class checks
__device__ __forceinline__ double sqrt_pos(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double s = x * y, h = 0.5 * y;
    const double r = __builtin_fma(-s, h, 0.5);
    s = __builtin_fma(s, r, s);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-s, s, x);
    s = __builtin_fma(d, h, s);
    d = __builtin_fma(-s, s, x);
    return __builtin_fma(d, h, s);
}
// ln(v 2^-24) for an odd v < 2^24 (the uniforms u01d): v = f 2^k with f in [1/sqrt2, sqrt2),
// ln f = 2 atanh(s) = 2 s + s^3 P(s^2), s = (f - 1) / (f + 1), |s| <= 0.172, series to s^21.
// e ln 2 + 2 s is summed exactly (ln 2 split Cody-Waite style, hi with 32 trailing zero bits so
// e ln2_hi is exact; Fast2Sum since |e ln 2| >= |2 s| whenever e != 0) and every small term --
// the quotient's residual, s^3 P, e ln2_lo -- rounds once into the tail: about 0.55 ulp (the
// single-sum form reached 2.06 ulp where e ln 2 and ln f nearly cancel)
template <typename Coef = LitCoef>
__device__ __forceinline__ double log_u24(uint32_t v, Coef c0 = Coef{}) {
    const Coef c = c0;
    const int k = 31 - __builtin_clz(v);
    double f = __builtin_ldexp((double)v, -k);  // [1, 2), exact
    const bool hi = f > c[kSqrt2];
    f = hi ? 0.5 * f : f;
    const double e = (double)(k - 24 + (hi ? 1 : 0));
    const double num = f - 1.0, den = f + 1.0, rd = rcp(den);  // num, den exact
    const double s = num * rd;
    const double s_lo = __builtin_fma(-s, den, num) * rd;  // s + s_lo = num / den to ~2^-106
    const double s2 = s * s;
    double p = c[kLog];
#pragma unroll
    for (int i = 1; i < 10; ++i) p = __builtin_fma(p, s2, c[kLog + i]);
    const double tail = __builtin_fma(s * s2, p, __builtin_fma(e, c[kLn2Lo], 2.0 * s_lo));
    const double a = e * c[kLn2Hi], b = 2.0 * s;  // both exact
    const double sum = a + b, err = (a - sum) + b;  // Fast2Sum (a = 0 gives err = 0)
    return sum + (err + tail);
}
// (sin, cos)(pi x) for x = v 2^-23 (v odd, < 2^24: x = 2 u01d): x = n/2 + r, |r| <= 1/4 exactly,
// sin(pi r) and cos(pi r) to r^17 and r^18, rotated by n quarter turns
template <typename Coef = LitCoef>
__device__ __forceinline__ void sincospi_v23(uint32_t v, double& sn, double& cs, Coef c0 = Coef{}) {
    const Coef c = c0;
    const uint32_t n = (v + (1u << 21)) >> 22;
    const double r = __builtin_ldexp((double)((int)v - (int)(n << 22)), -23);
    const double r2 = r * r;
    double ps = c[kSin];
#pragma unroll
    for (int i = 1; i < 9; ++i) ps = __builtin_fma(ps, r2, c[kSin + i]);
    ps *= r;
    double pc = c[kCos];
#pragma unroll
    for (int i = 1; i < 9; ++i) pc = __builtin_fma(pc, r2, c[kCos + i]);
    pc = __builtin_fma(pc, r2, 1.0);
    const uint32_t m = n & 3u;
    const double a = (m & 1u) ? pc : ps, b = (m & 1u) ? ps : pc;  // quarter turns: swap
    sn = (m == 2u || m == 3u) ? -a : a;
    cs = (m == 1u || m == 2u) ? -b : b;
}
}  // namespace f64m

// fp64 Box-Muller: sqrt(-2 ln u0) (cos, sin)(2 pi u1) with the straight-line forms above
template <typename Coef = f64m::LitCoef>
__device__ __forceinline__ void quad_normals(uint64_t step, uint32_t q, uint64_t key, double z[4], Coef cf = Coef{}) {
    uint32_t x[4];
    philox_ctr(step, q, key, x);
    const double r0 = f64m::sqrt_pos(-2.0 * f64m::log_u24(2u * (x[0] >> 9) + 1u, cf));
    const double r1 = f64m::sqrt_pos(-2.0 * f64m::log_u24(2u * (x[2] >> 9) + 1u, cf));
    double s0, c0, s1, c1;
    f64m::sincospi_v23(2u * (x[1] >> 9) + 1u, s0, c0, cf);
    f64m::sincospi_v23(2u * (x[3] >> 9) + 1u, s1, c1, cf);
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
    template <typename Coef>
    __device__ static __forceinline__ float sig(float x, float mu, float sl, Coef) { return sig(x, mu, sl); }
    __device__ static __forceinline__ float slope(double s) { return (float)(s * 1.4426950408889634); }
    // C/D row of a 16x16x4 f32 tile is (lane>>4)*4 + reg: identity row->node map
    __host__ __device__ static __forceinline__ int row_node(int rho) { return rho; }
};
template <> struct Tr<double> {
    typedef f64x4 acc_t;
    __device__ static __forceinline__ acc_t mfma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // 1 / (1 + e^(-(x - mu) s)) as 1 / (1 + 2^t), t = (mu - x) s log2(e): exp2 and rcp are within
    // 2 and 1 ulp, but t is rounded first, so the relative error grows as ~2.1 |t| 2^-53 (tens of
    // ulp at |t| ~ 40; tests/test_f64m_gpu.py states the measured bound)
    template <typename Coef = f64m::LitCoef>
    __device__ static __forceinline__ double sig(double x, double mu, double s, Coef c = Coef{}) {
        return f64m::rcp(1.0 + f64m::exp2((mu - x) * s * 1.4426950408889634, c));
    }
    __device__ static __forceinline__ double slope(double s) { return s; }
    // f64 16x16x4 C/D row is (lane>>4) + 4*reg; permute so that lane group g,
    // register r still means node 4g + r of the tile
    __host__ __device__ static __forceinline__ int row_node(int rho) { return 4 * (rho & 3) + (rho >> 2); }
};

// v = hi + mid + lo, each a bf16: |v - hi - mid - lo| <= 2^-27 |v|
__device__ __forceinline__ void split3(const float v[4], bf16x4& hi, bf16x4& mid, bf16x4& lo) {
    // pairwise: one v_cvt_pk_bf16_f32 (RNE) per two values and part, residuals by packed subtracts
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const f2 x = {v[2 * p], v[2 * p + 1]};
        const b2 h = __builtin_convertvector(x, b2);
        const f2 r = x - __builtin_convertvector(h, f2);
        const b2 m = __builtin_convertvector(r, b2);
        const b2 l = __builtin_convertvector(r - __builtin_convertvector(m, f2), b2);
        hi[2 * p] = h[0];
        hi[2 * p + 1] = h[1];
        mid[2 * p] = m[0];
        mid[2 * p + 1] = m[1];
        lo[2 * p] = l[0];
        lo[2 * p + 1] = l[1];
    }
}

// fp16 two-part split of v * 2^10 (v in [0, 1]): hi = fp16(RNE), lo = fp16(v 2^10 - hi);
// v 2^10 - hi is exact in fp32, so hi + lo carries 22 significant bits and, scaled,
// both parts stay normal fp16 down to v ~ 1e-4
// lo = fp16(x - hi) in one v_fma_mix{lo,hi}_f16 per value: x (fp32) * 1 - hi (read as
// fp16), rounded once to fp16; x - hi is exact in fp32, so the result is the same as
// converting hi back, subtracting and converting (two ops fewer per pair)
// PRE: v is already E 2^10 (the N <= 96 product kernels keep E in those units, so the
// split needs no scaling multiply)
template <bool PRE = false>
__device__ __forceinline__ void split2h(const float v[4], f16x4& hi, f16x4& lo) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const f2 x = PRE ? (f2){v[2 * p], v[2 * p + 1]} : (f2){v[2 * p], v[2 * p + 1]} * 1024.0f;
        const h2 h = __builtin_convertvector(x, h2);
        uint32_t lb;
        asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lb) : "v"(x[0]), "v"(h));
        asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lb) : "v"(x[1]), "v"(h));
        const h2 l = __builtin_bit_cast(h2, lb);
        hi[2 * p] = h[0];
        hi[2 * p + 1] = h[1];
        lo[2 * p] = l[0];
        lo[2 * p + 1] = l[1];
    }
}

// split2h of ONE pair (rows v[0], v[1]): the same operations as one iteration of split2h's loop,
// the two fp16 halves packed in a dword each (hi, lo)
template <bool PRE = false>
__device__ __forceinline__ void split2h_pair(const float v[2], uint32_t& hi, uint32_t& lo) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const f2 x = PRE ? (f2){v[0], v[1]} : (f2){v[0], v[1]} * 1024.0f;
    const h2 h = __builtin_convertvector(x, h2);
    uint32_t lb;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lb) : "v"(x[0]), "v"(h));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lb) : "v"(x[1]), "v"(h));
    hi = __builtin_bit_cast(uint32_t, h);
    lo = lb;
}

// fp16 three-part split of v * 2^10 (the V_F16X6 A/B): hi = fp16(x), r = x - hi exact in fp32 (one
// v_fma_mix_f32 per value), mid = fp16(r), lo = fp16(r - mid) (v_fma_mix{lo,hi}_f16, rounded once)
template <bool PRE = false>
__device__ __forceinline__ void split3h(const float v[4], f16x4& hi, f16x4& mid, f16x4& lo) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const f2 x = PRE ? (f2){v[2 * p], v[2 * p + 1]} : (f2){v[2 * p], v[2 * p + 1]} * 1024.0f;
        const h2 h = __builtin_convertvector(x, h2);
        float r0, r1;
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(x[0]), "v"(h));
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(x[1]), "v"(h));
        const f2 r = {r0, r1};
        const h2 m = __builtin_convertvector(r, h2);
        uint32_t lb;
        asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lb) : "v"(r[0]), "v"(m));
        asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lb) : "v"(r[1]), "v"(m));
        const h2 l = __builtin_bit_cast(h2, lb);
        hi[2 * p] = h[0];
        hi[2 * p + 1] = h[1];
        mid[2 * p] = m[0];
        mid[2 * p + 1] = m[1];
        lo[2 * p] = l[0];
        lo[2 * p + 1] = l[1];
    }
}

// Plasticity variable a_ie: fp64, or a compensated fp32 pair (increments of
// ~1e-6 on a ~2.5 are below fp32 half-ulp: plain fp32 would drop them).
template <bool kPair> struct AccA;
template <> struct AccA<false> {
    double v;
    __device__ void set(double x) { v = x; }
    __device__ double get() const { return v; }
    template <typename Real> __device__ Real val() const { return (Real)v; }
    __device__ void add(float inc) { v += (double)inc; }
    __device__ void add(double inc) { v += inc; }
};
template <> struct AccA<true> {
    float hi, lo;
    __device__ void set(double x) { hi = (float)x; lo = (float)(x - (double)hi); }
    __device__ double get() const { return (double)hi + (double)lo; }
    template <typename Real> __device__ Real val() const { return (Real)(hi + lo); }
    // fp32 value: |lo| <= ulp(hi)/2 after every add, so round(hi + lo) == hi (up to ties)
    __device__ float fast() const { return hi; }
    __device__ void add(float inc) {  // Kahan-Babuska: |hi| >> |inc|
        const float t = inc + lo;
        const float s = hi + t;
        lo = t - (s - hi);
        hi = s;
    }
};


}  // namespace wcdev

namespace {
// fp16 x3 coupling: CM scaled by sA = 2^(13 - e), max|CM| in [2^(e-1), 2^e), so every
// |CM sA| < 2^14 (fp16 max 65504 with the 2^10-scaled E: products < 2^24).
// scl[0] = sA, scl[1] = 1 / (2^10 sA) (folded into G by the kernel)
// One workgroup of 1024 threads; 8 independent loads per thread in flight (a one-load-per-iteration
// loop was latency-bound: 1.6 ms for N = 1000).
__global__ void __launch_bounds__(1024) coupling_scale_kernel(const double* __restrict__ sc, int N,
                                                              float* __restrict__ scl) {
    __shared__ double red[1024];
    constexpr int kU = 8;
    const size_t n = (size_t)N * N;
    double m[kU] = {0, 0, 0, 0, 0, 0, 0, 0};
    size_t i = threadIdx.x;
    for (; i + (kU - 1) * 1024 < n; i += kU * 1024) {
#pragma unroll
        for (int k = 0; k < kU; ++k) m[k] = fmax(m[k], fabs(sc[i + k * 1024]));
    }
    for (; i < n; i += 1024) m[0] = fmax(m[0], fabs(sc[i]));
#pragma unroll
    for (int k = 1; k < kU; ++k) m[0] = fmax(m[0], m[k]);
    red[threadIdx.x] = m[0];
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int e = 0;
        if (red[0] > 0.0) frexp(red[0], &e);
        e = max(-100, min(100, e));
        scl[0] = ldexpf(1.0f, 13 - e);
        scl[1] = ldexpf(1.0f, e - 23);
    }
}

}  // namespace
