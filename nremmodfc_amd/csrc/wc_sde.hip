// wc_sde.hip -- batched Wilson-Cowan Euler-Maruyama integrator for gfx950.
//
// Replaces the numba hot loop of netwWilsonCowanPlastic.py (wilsonCowan
// wc:77-83, run wc:86-137) for a whole batch of (G, sigmaE, seed) simulations.
//
// Layout (DESIGN.md "Kernel 1").  A workgroup of NW waves integrates 16
// simulations.  Lane l = 16*g + j of every wave serves simulation j; wave w
// owns the OT = NT/NW node tiles T0 = w*OT .. T0+OT-1, and within tile t lane
// group g owns nodes 16t + 4g + r (r = 0..3): E, I, a_ie, G, sigmaE of those
// nodes live in registers for the whole launch.  That layout is at once
//   * the C/D layout of the coupling MFMA  D[node][sim] = CM . E^T, and
//   * the B-operand layout of the next step's MFMA,
// so SC@E needs no lane shuffles: each wave publishes its new E tiles to a
// double-buffered LDS image (lane-to-lane copy), one s_barrier, and every wave
// streams the whole E vector back from LDS as MFMA B operands.
//
// Coupling arithmetic:
//   fp32 product path (V_F16X3): E 2^10 and CM sA (sA a power of two putting
//     max|CM| just under 2^14) are split into two fp16 parts (hi + lo, 22
//     significant bits, both normal over the range that matters) and the three
//     cross terms hi.hi, hi.lo, lo.hi run on v_mfma_f32_16x16x32_f16 with fp32
//     accumulation; 1/(2^10 sA) is folded into G.  Same trajectories vs the oracle
//     as the six-term bf16 split (V_BF16X6, kept as an ablation) at half the MFMAs.
//   fp64 parity path: v_mfma_f64_16x16x4_f64 (rows permuted, Tr<double>).
// The elementwise update (two logistic sigmoids, homeostatic plasticity,
// Philox4x32-10 noise + Box-Muller) runs on the VALU beside the MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <type_traits>
#include "wc_common.h"
#include "wc_device.h"

// N > 96: wc_sde_large.hip (fp32: one persistent cooperative launch, the state in registers;
// fallback and fp64: one GEMM-shaped launch per Euler step)
size_t wc_large_workspace_size(int B, int N, int precision);
int wc_large_status(const void* workspace, int B, int N, int precision, hipStream_t st);
int wc_large_integrate(const wc_params* p, int precision, int B, int N, const double* sc, const double* G,
                       const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                       int64_t nsteps, double tau_ip, int64_t rec_every, int64_t rec_ld, void* recE, void* recI,
                       void* recA, void* workspace, hipStream_t st);
#ifdef WCSDE_DIAG
int wc_large_diag(int variant, const wc_params* p, int B, int N, const double* sc, const double* G,
                  const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                  int64_t nsteps, double tau_ip, void* workspace, hipStream_t st);
#endif

namespace {
using namespace wcdev;


constexpr int kSims = 16;     // simulations per workgroup (MFMA N dimension)
constexpr int kMaxTiles = 6;  // N <= 96 on the register-resident path

struct KArgs {
    double a_ee, a_ei, a_ii, tauE, tauI, P, rhoE, rE, rI, mu, sigmaI, sqdtD, dtSim;
    double tau_ip;
    const double* G;
    const double* sigmaE;
    const uint64_t* keys;
    double* E;
    double* I;
    double* A;
    const void* frag;  // A-operand image (build_frag / build_frag_bf16)
    void* recE;
    void* recI;
    void* recA;
    int64_t step0;
    int64_t rec_every;
    int64_t rec_ld;  // 0: records [n_rec][B][N]; >0: node-major, (k, c) at c*rec_ld + k
    int nsteps;
    int B, N;
    const float4* zbuf;  // V_ZMEM: this launch's raw normals, [step][tile][Bp][lane group] (zblock_kernel)
    int zBp;             // simulations per step in zbuf (B rounded up to 16)
    // V_ZMEM: workgroups blockIdx >= zgen_b0 run on the CUs the integrator leaves idle and draw the
    // NEXT launch's normals (zgen_K steps from global step zgen_step0) into zbuf_next
    float4* zbuf_next;
    int zgen_b0, zgen_K;
    int64_t zgen_step0;
    int b0;  // first simulation of this launch (a launch may cover a range of the groups of 16)
};

// ---------------- A-operand (connectome) images ----------------
// native MFMA: frag[(T*NT + t)*64 + lane][r] = CM[16T + row_node(lane&15)][16t + 4(lane>>4) + r]
template <typename Real, int NT>
__global__ void build_frag(const double* __restrict__ sc, int N, Real* __restrict__ frag) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= NT * NT * 64 * 4) return;
    const int r = idx & 3;
    const int lane = (idx >> 2) & 63;
    const int tt = idx >> 8;
    const int T = tt / NT, t = tt % NT;
    const int row = 16 * T + Tr<Real>::row_node(lane & 15);
    const int col = 16 * t + 4 * (lane >> 4) + r;
    frag[idx] = (row < N && col < N) ? (Real)sc[(size_t)row * N + col] : (Real)0;
}

// bf16x6: frag[((T*NC + c)*3 + p)*64 + lane][jj] = part p of
//   CM[16T + (lane&15)][16(2c + jj/4) + 4(lane>>4) + jj%4]    (k-chunk c = tiles 2c, 2c+1)
// (the B operand of chunk c, lane l, element jj is E of that same node)
template <int NT>
__global__ void build_frag_bf16(const double* __restrict__ sc, int N, bf16x8* __restrict__ frag) {
    constexpr int NC = NT / 2;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= NT * NC * 64) return;
    const int lane = idx & 63;
    const int tc = idx >> 6;
    const int T = tc / NC, c = tc % NC;
    const int row = 16 * T + (lane & 15);
    bf16x8 part[3];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int col = 16 * (2 * c + (jj >> 2)) + 4 * (lane >> 4) + (jj & 3);
        const double x = (row < N && col < N) ? sc[(size_t)row * N + col] : 0.0;
        const __bf16 h = (__bf16)(float)x;
        const double r1 = x - (double)(float)h;
        const __bf16 m = (__bf16)(float)r1;
        part[0][jj] = h;
        part[1][jj] = m;
        part[2][jj] = (__bf16)(float)(r1 - (double)(float)m);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) frag[(size_t)(tc * 3 + p) * 64 + lane] = part[p];
}

// the two scale floats follow the fp16 image (inside the fp32 workspace, which is
// sized for the 3-part bf16 image)
// (P = 3: the three-part image of V_F16X6; frag_bytes leaves room for the scales behind it)
__host__ __device__ constexpr size_t hf_scale_offset(int NT, int P = 2) { return (size_t)NT * (NT / 2) * P * 64 * 16 / 4; }

// fp16 x3: frag[((T*NC + c)*2 + p)*64 + lane][jj] = part p of CM[..] sA, hi = fp16(x),
// lo = fp16(x - hi) (same element order as build_frag_bf16)
template <int NT, int P = 2>
__global__ void build_frag_f16(const double* __restrict__ sc, int N, const float* __restrict__ scl,
                               f16x8* __restrict__ frag) {
    constexpr int NC = NT / 2;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= NT * NC * 64) return;
    const int lane = idx & 63, tc = idx >> 6;
    const int T = tc / NC, c = tc % NC;
    const double sA = scl[0];
    const int row = 16 * T + (lane & 15);
    f16x8 part[P];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int col = 16 * (2 * c + (jj >> 2)) + 4 * (lane >> 4) + (jj & 3);
        const double x = (row < N && col < N) ? sc[(size_t)row * N + col] * sA : 0.0;
        const _Float16 h = (_Float16)(float)x;
        const double r = x - (double)(float)h;
        part[0][jj] = h;
        part[1][jj] = (_Float16)(float)r;
        if constexpr (P == 3) part[2][jj] = (_Float16)(float)(r - (double)(float)part[1][jj]);
    }
#pragma unroll
    for (int p = 0; p < P; ++p) frag[(size_t)(tc * P + p) * 64 + lane] = part[p];
}

// ---------------- packed fp32 cell pair (the fp32 product update) ----------------
struct PkConsts {
    f2v a_ee, Pm, knoise, cIe, cIi, cI0, rE, rI, dtE, dtI, dtA, rhoE, cA;
};

// Two cells of the folded-constant fp32 update (wc:77-83; the scalar form is in wc_sde_kernel's
// kFast branch) as packed fp32 math: v_pk_fma/mul/add_f32 carry two cells per instruction and
// round exactly like their scalar forms, the transcendentals stay scalar.  Same operations in
// the same order as the scalar form, so the same bits.
//
// ES: e is E 2^10 (the units of the MFMA operand split, which then needs no scaling multiply).
// The host scales a_ee, rE, cIe and dtA by 2^-10 and rhoE by 2^10 (exact), and the sigmoid
// returns SE 2^10 as rcp(2^-10 (1 + 2^te)), the denominator by one fma with 2^-10 (exact), so
// every rounding is the unscaled form's times 2^10: the same trajectory bit for bit (the
// hardware reciprocal is exponent-transparent; tools/cmp_libs.py checks the bits).
// WC_INC2 (default): the a_ie increment as in (E dtA - rhoE dtA), two operations instead of
// three (WC_INC2=0: the round-2 form in (E tA - rhoE tA), tA = in dtA; -2.5% per C3 launch).
#ifndef WC_F64_PREGS
#define WC_F64_PREGS 1
#endif
#ifndef WC_F64_TAB
#define WC_F64_TAB 0  // 1: the fp64 polynomial coefficients as scalar loads from a laundered table pointer
#endif
#ifndef WC_INC2
#define WC_INC2 1
#endif
// LEAN (V_LEAN): a_ie as a two-part running sum without per-step compensation -- lo collects
// the increments (one add), the value used is hi + lo (one add), and the caller folds lo into
// hi every 16 steps (renorm_a) -- two operations per cell pair fewer than Kahan-Babuska, the
// same value to within an fp32 rounding of a_ie.  AII0 (V_AII0): a_ii == 0 (the reference's
// value, wc:25), so the inhibitory sigmoid's in * cIi term, exactly cI0 + 0, is dropped.
#pragma clang fp contract(off)
template <bool ES = false, bool LEAN = false, bool AII0 = false>
__device__ __forceinline__ void cell_pair_f32(const PkConsts& k, f2v& e, f2v& in, f2v& ahi, f2v& alo, f2v cpl,
                                              f2v G, f2v sl, f2v z) {
    const f2v e0 = e, in0 = in;
    f2v x = __builtin_elementwise_fma(k.a_ee, e0, k.Pm);
    x = __builtin_elementwise_fma(LEAN ? -(ahi + alo) : -ahi, in0, x);
    x = __builtin_elementwise_fma(G, cpl, x);
    x = __builtin_elementwise_fma(k.knoise, z, x);
    const f2v te = x * sl;
    const f2v ex = {__builtin_amdgcn_exp2f(te.x), __builtin_amdgcn_exp2f(te.y)};
    const f2v one = {1.0f, 1.0f};
    constexpr float kS = ES ? 0x1p-10f : 1.0f;
    const f2v de = ES ? __builtin_elementwise_fma(ex, f2v{kS, kS}, f2v{kS, kS}) : one + ex;
    const f2v SE = {__builtin_amdgcn_rcpf(de.x), __builtin_amdgcn_rcpf(de.y)};
    const f2v ti = AII0 ? __builtin_elementwise_fma(e0, k.cIe, k.cI0)
                        : __builtin_elementwise_fma(e0, k.cIe, __builtin_elementwise_fma(in0, k.cIi, k.cI0));
    const f2v di = 1.0f + f2v{__builtin_amdgcn_exp2f(ti.x), __builtin_amdgcn_exp2f(ti.y)};
    const f2v SI = {__builtin_amdgcn_rcpf(di.x), __builtin_amdgcn_rcpf(di.y)};
    // (a_ie first: e0 and in0 are last read by their own updates, which can then write in place)
#if WC_INC2
    const f2v inc = in0 * __builtin_elementwise_fma(e0, k.dtA, k.cA);
#else
    const f2v tA = in0 * k.dtA;
    const f2v inc = __builtin_elementwise_fma(e0, tA, -k.rhoE * tA);
#endif
    if constexpr (LEAN) {
        alo = alo + inc;
    } else {
        const f2v t = inc + alo;  // Kahan-Babuska, as AccA<true>::add
        const f2v s = ahi + t;
        alo = t - (s - ahi);
        ahi = s;
    }
    // (ES: SE and e0 both carry 2^10, rE 2^-10: the same roundings times 2^10)
    e = __builtin_elementwise_fma(k.dtE, __builtin_elementwise_fma(__builtin_elementwise_fma(-k.rE, e0, one), SE, -e0), e0);
    in = __builtin_elementwise_fma(k.dtI, __builtin_elementwise_fma(__builtin_elementwise_fma(-k.rI, in0, one), SI, -in0), in0);
}

#pragma clang fp contract(on)

// ---------------- variants ----------------
enum : int {
    V_FRAG_REGS = 1,  // A-operand fragments held in registers (else streamed from LDS each step)
    V_NO_RNG = 2,     // ablation: noise term zero
    V_NO_MFMA = 4,    // ablation: coupling skipped
    V_KAHAN_A = 8,    // fp32: a_ie as a compensated fp32 pair instead of fp64
    V_BF16X6 = 32,    // fp32 coupling as the six bf16 cross terms (product)
    V_BF16X3 = 64,    // ablation: only the three leading terms (~2^-17 relative)
    V_REC2 = 128,     // node-major E records buffered 2 deep: one 8-B store per node per 2 records
    V_REC4 = 256,     // ... 4 deep: one 16-B store per node per 4 records (host checks eligibility)
    V_F16X3 = 512,    // fp32 coupling as three fp16 cross terms of two-part (22-bit) operands
    V_ZFIRST = 1024,  // fp32 fast path: the step's normals drawn before the coupling MFMAs
    V_ILV = 2048,     // ... interleaved with them (sched_group_barrier: 1 MFMA, 6 VALU)
    V_ILV2 = 4096,    // ... interleaved with them (1 MFMA, 2 VALU: the free half of a 16x16x32 gap)
    V_SCALAR = 8192,  // ablation: the fp32 fast update one cell per instruction (round-2 form)
    V_MIX = 16384,    // NT = 6 over NW = 4 waves per group, two waves with 2 tiles and two with 1,
                      // the pattern rotated per group so the SIMDs of a 3-group workgroup carry
                      // 5/4/5/4 tiles instead of 6/4/4/4 (3 waves of 2 tiles)
    V_LEAN = 32768,   // packed fp32 update: a_ie as hi + lo running sum, renormalised every 16 steps
    V_AII0 = 65536,   // a_ii == 0 (host-checked): the inhibitory sigmoid without its in * cIi term
    V_ZMEM = 131072,  // the raw normals come precomputed from zbuf (zblock_kernel on otherwise idle CUs)
    V_HALF2 = 262144, // NW = 2 NT: two waves per node tile, each updating two of a lane's four rows
                      // (both run the tile's coupling MFMAs; with V_ZMEM, so no Philox is repeated)
    V_F16X6 = 1048576, // A/B: three-part fp16 operands (E and CM each hi + mid + lo), six cross terms
                       // down to 2^-22 (>= 24 significant bits of both operands)
    V_ZPAIR = 524288, // SG = 2, V_ZMEM, one workgroup per CU: workgroups < zgen_b0 integrate two groups,
                      // the others one group while their second group's waves draw the next block's
                      // normals, one step's share per step between the workgroup's barriers
};

constexpr bool kFragRegs_(int var) { return (var & V_FRAG_REGS) != 0; }

// SG > 1: one workgroup holds SG groups of 16 simulations (SG x NW waves) that
// share ONE LDS copy of the connectome image; each group has its own E exchange.
template <typename Real, int NT, int NW, int VAR, int MINW, int SG = 1>
__global__ void __launch_bounds__(NW * 64 * SG, MINW) wc_sde_kernel(const KArgs a) {
    typedef typename Tr<Real>::acc_t acc_t;
    typedef __attribute__((ext_vector_type(4))) Real real4;
    constexpr bool kMix = (VAR & V_MIX) != 0;
    constexpr bool kHalf = (VAR & V_HALF2) != 0;
    static_assert(kMix ? (NT == 6 && NW == 4) : kHalf ? (NW == 2 * NT && SG == 1) : NT % NW == 0, "NW must divide NT");
    constexpr int OT = kMix ? 2 : kHalf ? 1 : NT / NW;  // tile slots per wave
    constexpr int RW = kHalf ? 2 : 4;                    // rows of a lane's 4 (one MFMA column quad) owned
    constexpr bool kHf3 = (VAR & V_F16X6) != 0;
    constexpr bool kHf = (VAR & (V_F16X3 | V_F16X6)) != 0;
    constexpr int kTerms = (VAR & V_BF16X6) ? 6 : (VAR & V_BF16X3) ? 3 : kHf3 ? 6 : kHf ? 3 : 0;
    constexpr bool kBf = kTerms > 0;  // 16-bit split coupling (bf16 or fp16 parts)
    static_assert(!kBf || (sizeof(Real) == 4 && NT % 2 == 0), "split coupling: fp32, even tile count");
    constexpr int NC = NT / 2;  // 16-bit k-chunks (2 tiles = 32 nodes)
    constexpr int NP = kTerms == 6 ? 3 : 2;
    constexpr int PS = (kHf && !kHf3) ? 2 : 3;  // parts per chunk in the images
    constexpr bool kFragRegs = (VAR & V_FRAG_REGS) != 0;
    constexpr bool kRng = (VAR & V_NO_RNG) == 0;
    constexpr bool kMfma = (VAR & V_NO_MFMA) == 0;
    constexpr bool kPairA = sizeof(Real) == 4 && (VAR & V_KAHAN_A) != 0;
    // G and the slope per cell in registers (fp64: WC_F64_PREGS; else re-read from memory every step)
    constexpr bool kParamRegs = sizeof(Real) == 4 || WC_F64_PREGS;
    // fp32 with the compensated a_ie: the folded-constant update (Sl holds -sigmaE log2 e)
    constexpr bool kFast = sizeof(Real) == 4 && kPairA;
    constexpr bool kZFirst = kFast && kRng && (VAR & V_ZFIRST) != 0;
    constexpr bool kPk = (VAR & V_SCALAR) == 0;  // packed fp32 cell pairs (cell_pair_f32)
    // the fp16x3 packed product path keeps E in units of 2^-10 (E[][] holds E 2^10): the
    // MFMA operand split needs no scaling multiply (cell_pair_f32<true>)
    constexpr bool kEs = kFast && kPk && kHf;
    constexpr bool kLean = kFast && kPk && (VAR & V_LEAN) != 0;
    constexpr bool kAii0 = kFast && kPk && (VAR & V_AII0) != 0;
    constexpr bool kZMem = kFast && kPk && kRng && (VAR & V_ZMEM) != 0;
    static_assert(!kHalf || (kZMem && kHf && !kHf3), "V_HALF2: the fp16x3 packed path with precomputed normals");
    constexpr bool kZPair = (VAR & V_ZPAIR) != 0;
    static_assert(!kZPair || (kZMem && SG == 2 && NW > 1 && !kHalf), "V_ZPAIR: two groups, normals from zbuf");
    constexpr float kEsc = kEs ? 1024.0f : 1.0f, kEinv = kEs ? 0x1p-10f : 1.0f;
    // VALU slots after each MFMA in the interleaved schedule (0: compiler's own order)
    constexpr int kIlv = !(kZFirst && kBf && kMfma) ? 0 : (VAR & V_ILV) ? 6 : (VAR & V_ILV2) ? 2 : 0;
    constexpr int kFragUnits = kBf ? NT * NC * PS : NT * NT;  // 16-B (bf16x8 / real4 f32) or 32-B units

    extern __shared__ __attribute__((aligned(16))) char smem[];
    if constexpr ((VAR & V_ZMEM) != 0 && !kZPair) {
        if ((int)blockIdx.x >= a.zgen_b0) {  // generator workgroup: the next block's normals, grid-stride
            const uint32_t total = (uint32_t)a.zgen_K * NT * (uint32_t)a.zBp * 4u;
            const uint32_t stride = (gridDim.x - a.zgen_b0) * blockDim.x;
            for (uint32_t i = (blockIdx.x - a.zgen_b0) * blockDim.x + threadIdx.x; i < total; i += stride) {
                const uint32_t gq = i & 3u, bq = (i >> 2) % (uint32_t)a.zBp, row = (i >> 2) / (uint32_t)a.zBp;
                const uint32_t tq = row % NT, sq = row / NT;
                f2v zp[2];
                quad_normals_pk((uint64_t)(a.zgen_step0 + sq), 4u * tq + gq, a.keys[bq < (uint32_t)a.B ? bq : a.B - 1], zp);
                a.zbuf_next[i] = make_float4(zp[0].x, zp[0].y, zp[1].x, zp[1].y);
            }
            return;
        }
    }
    // LDS: [A-operand image, unless kFragRegs] [E exchange, 2 buffers, if NW > 1]
    const size_t frag_bytes = kFragRegs ? 0 : (size_t)kFragUnits * 64 * (kBf ? 16 : sizeof(real4));
    const int grp = SG == 1 ? 0 : (threadIdx.x >> 6) / NW;
    char* xraw = smem + frag_bytes;
    bf16x8* xb16 = reinterpret_cast<bf16x8*>(xraw) + grp * (2 * NC * PS * 64);  // [2][NC][PS][64] per group
    real4* xbn = reinterpret_cast<real4*>(xraw) + grp * (2 * NT * 64);         // [2][NT][64] per group

    const int lane = threadIdx.x & 63;
    const int w = SG == 1 ? threadIdx.x >> 6 : (threadIdx.x >> 6) % NW;
    const int j = lane & 15, g = lane >> 4;
    // V_ZPAIR: workgroup i < zgen_b0 holds groups 2i, 2i + 1; a later one group zgen_b0 + i and,
    // in its second group's waves, a normals generator (no simulation: b past the batch)
    const bool zgen = kZPair && (int)blockIdx.x >= a.zgen_b0 && grp == 1;
    const int gidx = !kZPair ? (int)blockIdx.x * SG + grp
                   : (int)blockIdx.x < a.zgen_b0 ? 2 * (int)blockIdx.x + grp : a.zgen_b0 + (int)blockIdx.x;
    const int b = zgen ? a.B + j : a.b0 + gidx * kSims + j;
    const bool live = b < a.B;
    const int bb = live ? b : a.B - 1;  // tail lanes mirror the last sim, never store
    const int N = a.N;
    // this wave's tiles T0 .. T0 + nt - 1 (nt = OT except in V_MIX); a slot u >= nt maps to the
    // dead tile NT, whose nodes (>= 96 >= N) every n < N test skips
    int T0 = NW == 1 ? 0 : kHalf ? (w >> 1) : w * OT, nt = OT;
    const int R0 = kHalf ? 2 * (w & 1) : 0;  // first owned row of the lane's four
    if constexpr (kMix) {
        static_assert(!kFragRegs_(VAR) && (VAR & V_ZFIRST) == 0, "V_MIX: LDS fragments, plain schedule");
        const int rot = grp & 3;
        auto cnt = [&](int v) { return ((v + 4 - rot) & 3) < 2 ? 2 : 1; };  // (2, 2, 1, 1) rotated
        nt = cnt(w);
        T0 = 0;
        for (int v = 0; v < w; ++v) T0 += cnt(v);
    }
    auto TL = [&](int u) { return !kMix || u < nt ? T0 + u : NT; };
    auto owned = [&](int u) { return !kMix || u < nt; };  // (wave-uniform)

    // ---- A operand: this wave's rows, in registers or the whole image in LDS ----
    constexpr bool kRegBf = kFragRegs && kBf, kRegN = kFragRegs && !kBf;
    bf16x8 F16[kRegBf ? OT : 1][kRegBf ? NC : 1][kRegBf ? NP : 1];
    real4 FN[kRegN ? OT : 1][kRegN ? NT : 1];
    {
        const bf16x8* g16 = reinterpret_cast<const bf16x8*>(a.frag);
        const real4* gn = reinterpret_cast<const real4*>(a.frag);
        if constexpr (kRegBf) {
#pragma unroll
            for (int u = 0; u < OT; ++u)
#pragma unroll
                for (int c = 0; c < NC; ++c)
#pragma unroll
                    for (int p = 0; p < NP; ++p) F16[u][c][p] = g16[((TL(u) * NC + c) * PS + p) * 64 + lane];
        } else if constexpr (kRegN) {
#pragma unroll
            for (int u = 0; u < OT; ++u)
#pragma unroll
                for (int t = 0; t < NT; ++t) FN[u][t] = gn[(TL(u) * NT + t) * 64 + lane];
        } else if constexpr (kBf) {
            bf16x8* l16 = reinterpret_cast<bf16x8*>(smem);
            for (int i = threadIdx.x; i < kFragUnits * 64; i += blockDim.x) l16[i] = g16[i];
        } else {
            real4* ln = reinterpret_cast<real4*>(smem);
            for (int i = threadIdx.x; i < kFragUnits * 64; i += blockDim.x) ln[i] = gn[i];
        }
    }

    const uint64_t key = a.keys[bb];
    // fp16 coupling: the MFMA sums CM sA x E 2^10; 1 / (2^10 sA) is folded into G (exact)
    Real gscale = 1;
    if constexpr (kHf) gscale = reinterpret_cast<const float*>(a.frag)[hf_scale_offset(NT, PS) + 1];

    // ---- own state and per-node parameters ----
    constexpr int PT = kParamRegs ? OT : 1;
    Real E[OT][RW], I[OT][RW], Gc[PT][RW], Sl[PT][RW];
    AccA<kPairA> A[OT][RW];
#pragma unroll
    for (int u = 0; u < OT; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int n = 16 * TL(u) + 4 * g + R0 + r;
            const bool ok = n < N;
            const size_t o = (size_t)bb * N + (ok ? n : 0);
            E[u][r] = ok ? (Real)a.E[o] * (Real)kEsc : (Real)0;
            I[u][r] = ok ? (Real)a.I[o] : (Real)0;
            A[u][r].set(ok ? a.A[o] : 0.0);
            if constexpr (kParamRegs) {
                Gc[u][r] = ok ? (Real)a.G[o] * gscale : (Real)0;
                Sl[u][r] = ok ? (kFast ? -1 : 1) * Tr<Real>::slope(a.sigmaE[o]) : (Real)0;
            }
        }

    // ---- B operand (E of every node) ----
    // NW == 1: registers.  NW > 1: each wave publishes its own tiles to the LDS
    // image of the step, then every wave reads chunks back at the point of use
    // (register arrays are only ever indexed by compile-time constants).
    bf16x8 XB[(kBf && NW == 1) ? NC : 1][NP];
    Real X[(!kBf && NW == 1) ? NT : 1][4];
    auto publish = [&](int buf) {
        if constexpr (NW == 1) {
            if constexpr (kBf) {
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    bf16x4 h0, m0, l0, h1, m1, l1;
                    if constexpr (kHf3) {
                        split3h<kEs>(E[2 * c], reinterpret_cast<f16x4&>(h0), reinterpret_cast<f16x4&>(m0),
                                     reinterpret_cast<f16x4&>(l0));
                        split3h<kEs>(E[2 * c + 1], reinterpret_cast<f16x4&>(h1), reinterpret_cast<f16x4&>(m1),
                                     reinterpret_cast<f16x4&>(l1));
                    } else if constexpr (kHf) {
                        split2h<kEs>(E[2 * c], reinterpret_cast<f16x4&>(h0), reinterpret_cast<f16x4&>(m0));
                        split2h<kEs>(E[2 * c + 1], reinterpret_cast<f16x4&>(h1), reinterpret_cast<f16x4&>(m1));
                    } else {
                        split3(E[2 * c], h0, m0, l0);
                        split3(E[2 * c + 1], h1, m1, l1);
                    }
                    XB[c][0] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                    XB[c][1] = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
                    if constexpr (NP == 3) XB[c][2] = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
                }
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) X[t][r] = E[t][r];
            }
        } else {
            if constexpr (kHalf) {
                // the owned two rows: one dword (two fp16) of the tile's 8-B slot per part
                uint32_t* x2 = reinterpret_cast<uint32_t*>(xb16 + buf * NC * PS * 64);
                const int t = TL(0);
                uint32_t hl[2];
                split2h_pair<kEs>(E[0], hl[0], hl[1]);
#pragma unroll
                for (int p = 0; p < 2; ++p) x2[((((t >> 1) * PS + p) * 64 + lane) * 2 + (t & 1)) * 2 + (R0 >> 1)] = hl[p];
            } else if constexpr (kBf) {
                bf16x4* x4 = reinterpret_cast<bf16x4*>(xb16 + buf * NC * PS * 64);
#pragma unroll
                for (int u = 0; u < OT; ++u) {
                    if (!owned(u)) continue;
                    const int t = TL(u);  // chunk t/2, half t&1 (runtime: address arithmetic only)
                    bf16x4 hmo[3];
                    if constexpr (kHf3)
                        split3h<kEs>(E[u], reinterpret_cast<f16x4&>(hmo[0]), reinterpret_cast<f16x4&>(hmo[1]),
                                     reinterpret_cast<f16x4&>(hmo[2]));
                    else if constexpr (kHf) split2h<kEs>(E[u], reinterpret_cast<f16x4&>(hmo[0]), reinterpret_cast<f16x4&>(hmo[1]));
                    else split3(E[u], hmo[0], hmo[1], hmo[2]);
#pragma unroll
                    for (int p = 0; p < NP; ++p) x4[(((t >> 1) * PS + p) * 64 + lane) * 2 + (t & 1)] = hmo[p];
                }
            } else {
                real4* xb = xbn + buf * NT * 64;
#pragma unroll
                for (int u = 0; u < OT; ++u) xb[TL(u) * 64 + lane] = real4{E[u][0], E[u][1], E[u][2], E[u][3]};
            }
            __syncthreads();  // no LDS-DMA in flight: lgkmcnt(0) + s_barrier
        }
    };
    if constexpr (!kFragRegs) __syncthreads();  // A-operand image staged
    if constexpr (kZPair) {
        if (zgen) {
            // the integrating group's barriers, one for publish(0) and one per step, are matched one
            // for one (raw s_barrier: nothing of this wave's needs ordering against them, and its
            // normals stores must not be waited for at every step); between two of them this wave
            // draws its share of one step of the next block: the same quads every step (key and
            // quad index loaded once), quad_normals_pk and the zbuf layout of zblock_kernel
            constexpr int kGI = 2;  // quads per thread and step at most (host: zpair_shape)
            const uint32_t Bq = (uint32_t)a.zBp;
            const uint32_t per_step = (uint32_t)NT * Bq * 4u, step_stride = per_step;
            const uint32_t nthr = (gridDim.x - (uint32_t)a.zgen_b0) * (NW * 64u);
            const uint32_t me = (blockIdx.x - (uint32_t)a.zgen_b0) * (NW * 64u) + (threadIdx.x - NW * 64u);
            uint64_t gkey[kGI];
            uint32_t gquad[kGI], goff[kGI];
            bool gon[kGI];
#pragma unroll
            for (int k = 0; k < kGI; ++k) {
                const uint32_t i0 = me + (uint32_t)k * nthr;
                gon[k] = i0 < per_step;
                const uint32_t i = gon[k] ? i0 : 0u;  // (a thread with one quad draws quad 0 twice, stores once)
                const uint32_t bq = (i >> 2) % Bq, tq = (i >> 2) / Bq;
                gquad[k] = 4u * tq + (i & 3u);
                goff[k] = (tq * (uint32_t)a.zBp + bq) * 4u + (i & 3u);
                gkey[k] = a.keys[bq < (uint32_t)a.B ? bq : a.B - 1];
            }
            __builtin_amdgcn_s_barrier();
            float4* zo = a.zbuf_next;
            for (int s = 0; s < a.nsteps; ++s) {
                if (s < a.zgen_K) {
                    // every quad drawn unconditionally (independent Philox chains side by side), stored if owned
                    f2v zp[kGI][2];
#pragma unroll
                    for (int k = 0; k < kGI; ++k) quad_normals_pk((uint64_t)(a.zgen_step0 + s), gquad[k], gkey[k], zp[k]);
#pragma unroll
                    for (int k = 0; k < kGI; ++k)
                        if (gon[k]) zo[goff[k]] = make_float4(zp[k][0].x, zp[k][0].y, zp[k][1].x, zp[k][1].y);
                    zo += step_stride;
                }
                __builtin_amdgcn_s_barrier();
            }
            return;
        }
    }
    publish(0);

    Real a_ee = (Real)a.a_ee, a_ei = (Real)a.a_ei, a_ii = (Real)a.a_ii;
    Real P = (Real)a.P, rhoE = (Real)a.rhoE, rE = (Real)a.rE, rI = (Real)a.rI;
    Real mu = (Real)a.mu, slI = Tr<Real>::slope(a.sigmaI), sqdtD = (Real)a.sqdtD;
    // fp32 product path: folded constants (see the kFast update)
    const float Pm = (float)(a.P - a.mu), knoise = (float)(a.sqdtD * (double)kSqrt2Ln2);
    const float cIe = (float)(-a.a_ei * a.sigmaI * 1.4426950408889634);
    const float cIi = (float)(a.a_ii * a.sigmaI * 1.4426950408889634);
    const float cI0 = (float)(a.mu * a.sigmaI * 1.4426950408889634);
    const Real dtE = (Real)(a.dtSim / a.tauE), dtI = (Real)(a.dtSim / a.tauI);
    Real dt = (Real)a.dtSim;
    const Real dtA = (Real)(a.dtSim / a.tau_ip);
    Real tauE = (Real)a.tauE, tauI = (Real)a.tauI, tau_ip = (Real)a.tau_ip;  // fp64 exact forms
    Real itauE = (Real)(1.0 / a.tauE), itauI = (Real)(1.0 / a.tauI), itau_ip = (Real)(1.0 / a.tau_ip);
    if constexpr (sizeof(Real) == 8) {
        asm volatile("" : "+v"(itauE), "+v"(itauI), "+v"(itau_ip));
        // fp64: the model constants pinned in VGPR pairs.  As wave-uniform doubles they sit in
        // SGPRs beside the Philox round keys and the ocml polynomial constants, overflow the SGPR
        // file and come back through v_readlane (262 per step loop, plus their s_nop hazards).
        asm volatile("" : "+v"(a_ee), "+v"(a_ei), "+v"(a_ii), "+v"(P), "+v"(rhoE), "+v"(rE));
        asm volatile("" : "+v"(rI), "+v"(mu), "+v"(slI), "+v"(sqdtD), "+v"(dt));
        asm volatile("" : "+v"(tauE), "+v"(tauI), "+v"(tau_ip));
    }
    PkConsts pk{};
    if constexpr (kFast && kPk) {
        auto bc = [](float v) { return f2v{v, v}; };
        // (kEs: E-side constants carry 2^-10, rhoE 2^10, all exact)
        pk = PkConsts{bc((float)a_ee * kEinv), bc(Pm), bc(knoise), bc(cIe * kEinv), bc(cIi), bc(cI0),
                      bc((float)rE * kEinv), bc((float)rI), bc((float)dtE), bc((float)dtI),
                      bc((float)dtA * kEinv), bc((float)rhoE * kEsc), bc((float)(-a.rhoE * a.dtSim / a.tau_ip))};
    }
    const size_t BN = (size_t)a.B * N;
    const int rec_every = (int)a.rec_every;
    int rec_cnt = 0, rec_row = 0;
    // record buffer (RB > 1): the RB-1 previous E records of this lane's nodes, oldest first
    constexpr int RB = (VAR & V_REC4) ? 4 : (VAR & V_REC2) ? 2 : 1;
    Real rbuf[RB > 1 ? OT : 1][RW][RB > 1 ? RB - 1 : 1];

    // V_ZMEM: normals of the next kZD steps in flight
    constexpr int kZD = kZMem ? 4 : 1;
    typedef std::conditional_t<kHalf, float2, float4> zt;  // V_HALF2: the owned rows' two normals
    auto zload = [&](int st_, int u) -> zt {
        const size_t q = (((size_t)st_ * NT + TL(u)) * a.zBp + (size_t)b) * 4 + g;
        if constexpr (kHalf) return reinterpret_cast<const float2*>(a.zbuf)[q * 2 + (R0 >> 1)];
        else return a.zbuf[q];
    };
    zt zq[kZD][kZMem ? OT : 1];
    if constexpr (kZMem) {
#pragma unroll
        for (int d = 0; d < kZD; ++d)
#pragma unroll
            for (int u = 0; u < OT; ++u) zq[d][u] = zload(min(d, a.nsteps - 1), u);
    }
    // one Euler step; ZS = the V_ZMEM prefetch slot of step s (s % kZD: a compile-time index, so the
    // in-flight normals are never moved between registers -- a move would wait for every older load)
    auto step_body = [&](const int s, auto zslot) {
        constexpr int ZS = decltype(zslot)::value;
        const int buf = s & 1;
        // ---- record the state before the update (wc:124-125) ----
        if (rec_every > 0) {
            if (rec_cnt == 0) {
                if constexpr (RB > 1) {
                    // node-major ring, E only: flush RB records as one vector store per node
                    if (rec_row % RB == RB - 1) {
                        if (live) {
#pragma unroll
                            for (int u = 0; u < OT; ++u)
#pragma unroll
                                for (int r = 0; r < RW; ++r) {
                                    const int n = 16 * TL(u) + 4 * g + R0 + r;
                                    if (n < N) {
                                        Real* dst = static_cast<Real*>(a.recE) + ((size_t)bb * N + n) * a.rec_ld +
                                                    (rec_row - (RB - 1));
                                        if constexpr (RB == 4) {
                                            *reinterpret_cast<real4*>(dst) =
                                                real4{rbuf[u][r][0], rbuf[u][r][1], rbuf[u][r][2], E[u][r] * (Real)kEinv};
                                        } else {
                                            typedef __attribute__((ext_vector_type(2))) Real real2;
                                            *reinterpret_cast<real2*>(dst) = real2{rbuf[u][r][0], E[u][r] * (Real)kEinv};
                                        }
                                    }
                                }
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < OT; ++u)
#pragma unroll
                            for (int r = 0; r < RW; ++r) {
#pragma unroll
                                for (int k = 0; k + 1 < RB - 1; ++k) rbuf[u][r][k] = rbuf[u][r][k + 1];
                                rbuf[u][r][RB - 2] = E[u][r] * (Real)kEinv;
                            }
                    }
                } else if (live) {
                    // (N and the record stride laundered here: addresses computed from them cannot be
                    // hoisted out of the step loop, where they would pin 64-bit VGPR pairs)
                    int Nn = N;
                    int64_t ld = a.rec_ld;
                    asm volatile("" : "+s"(Nn), "+s"(ld));
                    if (ld == 0 && BN < ((size_t)1 << 29)) {
                        // time-major (the pipeline's fp32 form): the record row's base is uniform (an SGPR
                        // pair) and a lane's cells sit at 32-bit element offsets cb + 16 TL(u) + r from it,
                        // so the stores take the saddr form with immediate offsets and no 64-bit cell
                        // address is held across the step loop (eight of them had spilled to scratch)
                        Real* recE_row = static_cast<Real*>(a.recE) + (size_t)rec_row * BN;
                        Real* recI_row = a.recI ? static_cast<Real*>(a.recI) + (size_t)rec_row * BN : nullptr;
                        Real* recA_row = a.recA ? static_cast<Real*>(a.recA) + (size_t)rec_row * BN : nullptr;
                        const uint32_t cb = (uint32_t)bb * (uint32_t)Nn + (uint32_t)(4 * g + R0);
#pragma unroll
                        for (int u = 0; u < OT; ++u)
#pragma unroll
                            for (int r = 0; r < RW; ++r) {
                                const int n = 16 * TL(u) + 4 * g + R0 + r;
                                if (n < N) {
                                    const uint32_t cc = cb + (uint32_t)(16 * TL(u) + r);
                                    recE_row[cc] = E[u][r] * (Real)kEinv;
                                    if (recI_row) recI_row[cc] = I[u][r];
                                    if (recA_row) recA_row[cc] = (Real)A[u][r].get();
                                }
                            }
                    } else {
#pragma unroll
                        for (int u = 0; u < OT; ++u)
#pragma unroll
                            for (int r = 0; r < RW; ++r) {
                                const int n = 16 * TL(u) + 4 * g + R0 + r;
                                if (n < N) {
                                    const size_t cc = (size_t)bb * Nn + n;
                                    const size_t o = ld ? cc * ld + rec_row : (size_t)rec_row * BN + cc;
                                    static_cast<Real*>(a.recE)[o] = E[u][r] * (Real)kEinv;
                                    if (a.recI) static_cast<Real*>(a.recI)[o] = I[u][r];
                                    if (a.recA) static_cast<Real*>(a.recA)[o] = (Real)A[u][r].get();
                                }
                            }
                    }
                }
                ++rec_row;
                rec_cnt = rec_every;
            }
            --rec_cnt;
        }

        // ---- coupling: acc[u][r] = sum_k CM[node(T0+u, g, r)][k] E[k]  (np.dot, wc:81) ----
        acc_t acc[OT];
#pragma unroll
        for (int u = 0; u < OT; ++u) acc[u] = acc_t{0, 0, 0, 0};
        int fl = lane;
        if constexpr (!kFragRegs || NW > 1) asm volatile("" : "+v"(fl));  // opaque: LDS reads stay in the loop
        const uint64_t gstep = (uint64_t)(a.step0 + s);
        // V_ZMEM: this step's normals were loaded kZD steps ago (a step is shorter than a memory
        // round trip); issue the load of step s + kZD now (clamped to the block's last step)
        zt zm[kZMem ? OT : 1];
        if constexpr (kZMem) {
            const int sl = min(s + kZD, a.nsteps - 1);
#pragma unroll
            for (int u = 0; u < OT; ++u) {
                zm[u] = zq[ZS][u];
                zq[ZS][u] = zload(sl, u);
            }
        }
        // V_ZFIRST: the normals do not depend on the coupling, so they can fill the MFMA chain's gaps
        float zz[kZFirst ? OT : 1][4];
        if constexpr (kZFirst) {
#pragma unroll
            for (int u = 0; u < OT; ++u) quad_normals_raw(gstep, (uint32_t)(4 * TL(u) + g), key, zz[u]);
        }
        if constexpr (kMfma && kBf) {
            const bf16x8* l16 = reinterpret_cast<const bf16x8*>(smem);
            const bf16x8* xb = xb16 + buf * NC * PS * 64;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                bf16x8 xe[NP];
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    if constexpr (NW == 1) xe[p] = XB[c][p];
                    else xe[p] = xb[(c * PS + p) * 64 + fl];
                }
#pragma unroll
                for (int u = 0; u < OT; ++u) {
                    if (!owned(u)) continue;
                    bf16x8 f[NP];
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        if constexpr (kFragRegs) f[p] = F16[u][c][p];
                        else f[p] = l16[((TL(u) * NC + c) * PS + p) * 64 + fl];
                    }
                    if constexpr (kHf) {  // small terms first: [2^-22 (lo.hi, mid.mid, hi.lo)], 2^-11 (lo.hi, hi.lo), 1 (hi.hi)
                        typedef f16x8 h8;
                        if constexpr (kHf3) {
                            acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[2], (h8)xe[0], acc[u], 0, 0, 0);
                            acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[1], (h8)xe[1], acc[u], 0, 0, 0);
                            acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[0], (h8)xe[2], acc[u], 0, 0, 0);
                        }
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[1], (h8)xe[0], acc[u], 0, 0, 0);
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[0], (h8)xe[1], acc[u], 0, 0, 0);
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)f[0], (h8)xe[0], acc[u], 0, 0, 0);
                        continue;
                    }
                    // small terms first: 2^-18 (lo.hi, mid.mid, hi.lo), 2^-9 (mid.hi, hi.mid), 1 (hi.hi)
                    if constexpr (NP == 3) {
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[2], xe[0], acc[u], 0, 0, 0);
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], xe[1], acc[u], 0, 0, 0);
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], xe[2], acc[u], 0, 0, 0);
                    }
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], xe[0], acc[u], 0, 0, 0);
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], xe[1], acc[u], 0, 0, 0);
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], xe[0], acc[u], 0, 0, 0);
                }
            }
        } else if constexpr (kMfma) {
            const real4* ln = reinterpret_cast<const real4*>(smem);
            const real4* xb = xbn + buf * NT * 64;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                Real xe[4];
                if constexpr (NW == 1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) xe[r] = X[t][r];
                } else {
                    const real4 v = xb[t * 64 + fl];
#pragma unroll
                    for (int r = 0; r < 4; ++r) xe[r] = v[r];
                }
#pragma unroll
                for (int u = 0; u < OT; ++u) {
                    if constexpr (!kFragRegs && sizeof(Real) == 8)
                        if ((u & 1) == 0) __builtin_amdgcn_sched_barrier(0);  // bound fp64 read look-ahead
                    const real4 f = kFragRegs ? FN[u][t] : ln[(TL(u) * NT + t) * 64 + fl];
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[u] = Tr<Real>::mfma(f[r], xe[r], acc[u]);
                }
            }
        }

        if constexpr (kIlv > 0) {
            // LDS reads first, then each MFMA followed by a slice of the (independent) normal generation
#pragma unroll
            for (int i = 0; i < NC * NP * (OT + 1); ++i) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int i = 0; i < NC * OT * kTerms; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, kIlv, 0);
            }
        }
        // ---- elementwise update (wc:77-83), noise drawn inside the E sigmoid ----
#pragma unroll
        for (int u = 0; u < OT; ++u) {
            if (!owned(u)) continue;
            if constexpr (sizeof(Real) == 8) __builtin_amdgcn_sched_barrier(0);  // fp64: bound live ranges
            Real z[4] = {0, 0, 0, 0};
            if constexpr (kHalf) {
                // the owned pair (rows R0, R0 + 1): pair R0 / 2 of the full-tile form, same operations
                f2v e = {E[u][0], E[u][1]}, in = {I[u][0], I[u][1]};
                f2v ahi = {A[u][0].hi, A[u][1].hi}, alo = {A[u][0].lo, A[u][1].lo};
                const f2v cpl = R0 ? f2v{acc[u][2], acc[u][3]} : f2v{acc[u][0], acc[u][1]};
                cell_pair_f32<kEs, kLean, kAii0>(pk, e, in, ahi, alo, cpl, f2v{Gc[u][0], Gc[u][1]},
                                                  f2v{Sl[u][0], Sl[u][1]}, f2v{zm[u].x, zm[u].y});
                E[u][0] = e.x;
                E[u][1] = e.y;
                I[u][0] = in.x;
                I[u][1] = in.y;
                A[u][0].hi = ahi.x;
                A[u][1].hi = ahi.y;
                A[u][0].lo = alo.x;
                A[u][1].lo = alo.y;
                continue;
            } else if constexpr (kFast && kPk) {
                f2v zp[2] = {f2v{0, 0}, f2v{0, 0}};
                if constexpr (kZMem) {
                    zp[0] = f2v{zm[u].x, zm[u].y};
                    zp[1] = f2v{zm[u].z, zm[u].w};
                } else if constexpr (kZFirst) {
                    zp[0] = f2v{zz[u][0], zz[u][1]};
                    zp[1] = f2v{zz[u][2], zz[u][3]};
                } else if constexpr (kRng) {
                    quad_normals_pk(gstep, (uint32_t)(4 * TL(u) + g), key, zp);
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int r = 2 * h;
                    f2v e = {E[u][r], E[u][r + 1]}, in = {I[u][r], I[u][r + 1]};
                    f2v ahi = {A[u][r].hi, A[u][r + 1].hi}, alo = {A[u][r].lo, A[u][r + 1].lo};
                    const f2v cpl = kMfma ? f2v{acc[u][r], acc[u][r + 1]} : e * kEinv;
                    cell_pair_f32<kEs, kLean, kAii0>(pk, e, in, ahi, alo, cpl, f2v{Gc[u][r], Gc[u][r + 1]},
                                                      f2v{Sl[u][r], Sl[u][r + 1]}, zp[h]);
                    E[u][r] = e.x;
                    E[u][r + 1] = e.y;
                    I[u][r] = in.x;
                    I[u][r + 1] = in.y;
                    A[u][r].hi = ahi.x;
                    A[u][r + 1].hi = ahi.y;
                    A[u][r].lo = alo.x;
                    A[u][r + 1].lo = alo.y;
                }
                continue;
            }
            if constexpr (kFast && !kHalf) {
                if constexpr (kZFirst) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) z[r] = zz[u][r];
                } else if constexpr (kRng) {
                    quad_normals_raw(gstep, (uint32_t)(4 * TL(u) + g), key, z);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // wc:80-83 in fp32 with the constants folded:
                    //   x' = xE - mu; SE = 1/(1 + 2^(x' * (-sigmaE log2 e)));
                    //   SI = 1/(1 + 2^(e cIe + in cIi + cI0)); noise = knoise * raw normal
                    const float e = E[u][r], in = I[u][r];
                    const float ai = A[u][r].fast();
                    const float cpl = kMfma ? acc[u][r] : e;
                    float x = __builtin_fmaf(a_ee, e, Pm);
                    x = __builtin_fmaf(-ai, in, x);
                    x = __builtin_fmaf(Gc[u][r], cpl, x);
                    x = __builtin_fmaf(knoise, z[r], x);
                    const float SE = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * Sl[u][r]));
                    const float SI = __builtin_amdgcn_rcpf(
                        1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(e, cIe, __builtin_fmaf(in, cIi, cI0))));
                    E[u][r] = __builtin_fmaf(dtE, __builtin_fmaf(__builtin_fmaf(-rE, e, 1.0f), SE, -e), e);
                    I[u][r] = __builtin_fmaf(dtI, __builtin_fmaf(__builtin_fmaf(-rI, in, 1.0f), SI, -in), in);
#if WC_INC2
                    A[u][r].add(in * __builtin_fmaf(e, dtA, (float)(-a.rhoE * a.dtSim / a.tau_ip)));
#else
                    const float tA = in * dtA;
                    A[u][r].add(__builtin_fmaf(e, tA, -rhoE * tA));
#endif
                }
                continue;
            }
            if constexpr (!kHalf) {
            // fp64: the polynomial coefficients as scalar loads from a table, the pointer laundered
            // here so they are not hoisted out of the step loop into SGPRs (f64m, wc_device.h)
            const auto cf = [] {
                if constexpr (sizeof(Real) == 8 && WC_F64_TAB) return f64m::tab_coef();
                else return f64m::LitCoef{};
            }();
            if constexpr (kRng) quad_normals(gstep, (uint32_t)(4 * TL(u) + g), key, z, cf);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const Real e = E[u][r], in = I[u][r];
                const Real ai = A[u][r].template val<Real>();
                Real gc, sl;
                if constexpr (kParamRegs) {
                    gc = Gc[u][r];
                    sl = Sl[u][r];
                } else {
                    const int n = 16 * TL(u) + 4 * g + r;
                    const size_t o = (size_t)bb * N + (n < N ? n : 0);
                    gc = n < N ? (Real)a.G[o] : (Real)0;
                    sl = n < N ? Tr<Real>::slope(a.sigmaE[o]) : (Real)0;
                }
                const Real cpl = kMfma ? acc[u][r] : e;
                const Real xE = a_ee * e - ai * in + gc * cpl + P + sqdtD * z[r];
                const Real SE = Tr<Real>::sig(xE, mu, sl, cf);
                const Real xI = a_ei * e - a_ii * in;
                const Real SI = Tr<Real>::sig(xI, mu, slI, cf);
                if constexpr (sizeof(Real) == 8) {
                    // (the divisions by the time constants as a product with the reciprocal plus one
                    // correction step: the quotient to within an ulp, without the IEEE sequence)
                    auto qdiv = [](double x, double y, double iy) {
                        const double q = x * iy;
                        return __builtin_fma(__builtin_fma(-y, q, x), iy, q);
                    };
                    const Real dE = qdiv(-e + (1 - rE * e) * SE, tauE, itauE);
                    const Real dI = qdiv(-in + (1 - rI * in) * SI, tauI, itauI);
                    const Real dA = qdiv(in * (e - rhoE), tau_ip, itau_ip);
                    E[u][r] = e + dt * dE;
                    I[u][r] = in + dt * dI;
                    A[u][r].add(dt * dA);
                } else {
                    E[u][r] = e + dtE * (-e + (1 - rE * e) * SE);
                    I[u][r] = in + dtI * (-in + (1 - rI * in) * SI);
                    A[u][r].add(dtA * (in * (e - rhoE)));
                }
            }
            }  // !kHalf
        }
        if constexpr (kLean) {
            if ((s & 15) == 15) {  // fold the running increments into hi (wave-uniform branch)
#pragma unroll
                for (int u = 0; u < OT; ++u)
#pragma unroll
                    for (int r = 0; r < RW; ++r) {
                        const float hs = A[u][r].hi + A[u][r].lo;
                        A[u][r].lo = A[u][r].lo - (hs - A[u][r].hi);
                        A[u][r].hi = hs;
                    }
            }
        }
        publish(buf ^ 1);
    };
    if constexpr (kZMem) {
        int s = 0;
        for (; s + kZD <= a.nsteps; s += kZD) {
            step_body(s, std::integral_constant<int, 0>{});
            step_body(s + 1, std::integral_constant<int, 1 % kZD>{});
            step_body(s + 2, std::integral_constant<int, 2 % kZD>{});
            step_body(s + 3, std::integral_constant<int, 3 % kZD>{});
        }
        static_assert(kZD == 4, "the unrolled loop above assumes four slots");
        if (s < a.nsteps) step_body(s++, std::integral_constant<int, 0>{});
        if (s < a.nsteps) step_body(s++, std::integral_constant<int, 1 % kZD>{});
        if (s < a.nsteps) step_body(s++, std::integral_constant<int, 2 % kZD>{});
    } else {
        for (int s = 0; s < a.nsteps; ++s) step_body(s, std::integral_constant<int, 0>{});
    }

    // ---- records still buffered (rec_row % RB of them): the newest are the last rbuf slots ----
    if constexpr (RB > 1) {
        const int m = rec_row % RB;
        if (rec_every > 0 && m > 0 && live) {
#pragma unroll
            for (int u = 0; u < OT; ++u)
#pragma unroll
                for (int r = 0; r < RW; ++r) {
                    const int n = 16 * TL(u) + 4 * g + R0 + r;
                    if (n < N) {
                        Real* dst = static_cast<Real*>(a.recE) + ((size_t)bb * N + n) * a.rec_ld + (rec_row - m);
#pragma unroll
                        for (int k = 0; k < RB - 1; ++k)
                            if (k < m) dst[k] = rbuf[u][r][RB - 1 - m + k];
                    }
                }
        }
    }
    // ---- write back the state (own tiles) ----
    if (live) {
#pragma unroll
        for (int u = 0; u < OT; ++u)
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                const int n = 16 * TL(u) + 4 * g + R0 + r;
                if (n < N) {
                    const size_t o = (size_t)b * N + n;
                    a.E[o] = (double)(E[u][r] * (Real)kEinv);
                    a.I[o] = (double)I[u][r];
                    a.A[o] = A[u][r].get();
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
    Real z[4];
    quad_normals((uint64_t)step, (uint32_t)q, keys[b], z);
    for (int r = 0; r < 4; ++r)
        if (4 * q + r < N) out[(size_t)b * N + 4 * q + r] = z[r];
}

// The raw normals (quad_normals_pk, the integrator's own arithmetic: the same bits) of K steps for
// V_ZMEM, laid out for the integrator's loads: z[step][tile t][simulation b][lane group g] is the
// float4 of quad 4t + g of simulation b -- a wave's load for one tile is 1 KB contiguous.
__global__ void __launch_bounds__(256) zblock_kernel(const uint64_t* __restrict__ keys, int B, int Bp, int NT,
                                                     int64_t step0, float4* __restrict__ z) {
    // grid: x over (simulation, lane group) pairs of a step, y = s * NT + t (32-bit index math only)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Bp * 4) return;
    const int g = i & 3, b = i >> 2;
    const int t = (int)(blockIdx.y % (unsigned)NT), s = (int)(blockIdx.y / (unsigned)NT);
    f2v zp[2];
    quad_normals_pk((uint64_t)(step0 + s), (uint32_t)(4 * t + g), keys[b < B ? b : B - 1], zp);
    z[((size_t)blockIdx.y * Bp + b) * 4 + g] = make_float4(zp[0].x, zp[0].y, zp[1].x, zp[1].y);
}

int tiles_for(int N) { return (N + 15) / 16; }

template <typename Real, int NT, int NW, int VAR, int MINW = 1, int SG = 1>
int launch_v(const KArgs& ka, const double* sc, void* ws, hipStream_t st, bool prep = true, int extra_blocks = 0,
             size_t lds_floor = 0, int g0 = 0, int ng = -1) {
    constexpr bool hf = (VAR & (V_F16X3 | V_F16X6)) != 0;
    constexpr int HP = (VAR & V_F16X6) ? 3 : 2;  // fp16 parts per operand
    constexpr bool bf = (VAR & (V_BF16X6 | V_BF16X3)) != 0;
    constexpr bool frag_regs = (VAR & V_FRAG_REGS) != 0;
    size_t lds;
    if constexpr (hf) {
        const int total = NT * (NT / 2) * 64;
        float* scl = static_cast<float*>(ws) + hf_scale_offset(NT, HP);
        if (prep) {  // (prep = false: a later launch of the same call reuses the image)
            hipLaunchKernelGGL(coupling_scale_kernel, dim3(1), dim3(1024), 0, st, sc, ka.N, scl);
            hipLaunchKernelGGL((build_frag_f16<NT, HP>), dim3((total + 255) / 256), dim3(256), 0, st, sc, ka.N,
                               static_cast<const float*>(scl), static_cast<f16x8*>(ws));
        }
        lds = (frag_regs ? 0 : (size_t)NT * (NT / 2) * HP * 64 * 16) +
              (NW > 1 ? (size_t)SG * 2 * (NT / 2) * HP * 64 * 16 : 0);
    } else if constexpr (bf) {
        const int total = NT * (NT / 2) * 64;
        hipLaunchKernelGGL((build_frag_bf16<NT>), dim3((total + 255) / 256), dim3(256), 0, st, sc, ka.N,
                           static_cast<bf16x8*>(ws));
        lds = (frag_regs ? 0 : (size_t)NT * (NT / 2) * 3 * 64 * 16) +
              (NW > 1 ? (size_t)SG * 2 * (NT / 2) * 3 * 64 * 16 : 0);
    } else {
        const int total = NT * NT * 64 * 4;
        if (prep)
            hipLaunchKernelGGL((build_frag<Real, NT>), dim3((total + 255) / 256), dim3(256), 0, st, sc, ka.N,
                               static_cast<Real*>(ws));
        lds = (frag_regs ? 0 : (size_t)NT * NT * 64 * 4 * sizeof(Real)) +
              (NW > 1 ? (size_t)SG * 2 * NT * 64 * 4 * sizeof(Real) : 0);
    }
    // groups of 16 simulations g0 .. g0 + ng - 1 (ng < 0: to the last)
    KArgs kl = ka;
    kl.b0 = g0 * kSims;
    if (ng < 0) ng = (ka.B + kSims - 1) / kSims - g0;
    const int blocks = (ng + SG - 1) / SG + extra_blocks;
    lds = std::max(lds, lds_floor);  // (a floor above half the CU's LDS: one workgroup per CU)
    auto kern = wc_sde_kernel<Real, NT, NW, VAR, MINW, SG>;
    if (lds > 65536) {
        hipError_t ea = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(ea));
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(NW * 64 * SG), lds, st, kl);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    return WC_OK;
}

// ---------------- product configurations ----------------
constexpr int kVarF32 = V_F16X3 | V_FRAG_REGS | V_KAHAN_A;
#ifndef WC_F64_VAR_EXTRA
#define WC_F64_VAR_EXTRA 0  // ablation builds only (e.g. V_NO_MFMA, V_NO_RNG)
#endif
constexpr int kVarF64 = WC_F64_VAR_EXTRA;

size_t frag_bytes(int N, int precision) {
    if (precision == WC_F64) {
        const int nt = tiles_for(N);
        return (size_t)nt * nt * 64 * 4 * 8;
    }
    const int nt = (tiles_for(N) + 1) & ~1;  // bf16 k-chunks pair tiles
    return (size_t)nt * (nt / 2) * 3 * 64 * 16 + 256;  // (+ the fp16 scales behind a three-part image)
}

// the two normals blocks of the small-batch path follow the fp32 connectome image (256-B aligned)
size_t zmem_offset(int N) { return (frag_bytes(N, WC_F32) + 255) / 256 * 256; }

// ---- small batches: normals precomputed on the CUs the integrator leaves idle (V_ZMEM) ----
// A strong-scaled shard (e.g. 2,500 simulations = 157 groups of 16 on 256 CUs) keeps only part of
// the chip busy, and each busy CU's step is latency-bound; Philox + Box-Muller are about a third
// of a tile's step.  Each launch covers kZK steps with one workgroup per CU: the integrating
// workgroups read this block's normals from a buffer, the others draw the next block's
// (double-buffered, ordered by the launches on one stream; launch_zmem).
#ifndef WC_ZMEM_HALF
#define WC_ZMEM_HALF 1  // the normals-block path runs 12 waves per group, half a node tile each (V_HALF2;
                        // 0: six waves of one tile, 2,500 sims 0.747 vs 0.708 us per step, profiles/r03_half_ab.log)
#endif
constexpr int kZK = 1000;                // steps per launch (a multiple of the drivers' rec_every 20)
constexpr int kZMinIdle = 32;            // CUs the generator needs at least
constexpr int kZMaxGroups = 160;         // measured regime: up to 2,560 simulations (the 8-way C3 shard)

int cu_count();

size_t zmem_block_bytes(int B) {
    const int Bp = (B + kSims - 1) / kSims * kSims;
    return (size_t)kZK * kMaxTiles * Bp * 4 * sizeof(float4);
}

// B and N for which the small-batch path precomputes its normals (fp32, 81 <= N <= 96)
// V_ZPAIR regime: CUs < groups <= kZPairMax x CUs (the generators, one per one-group workgroup,
// draw at most ~2.5 quads per thread and step)
// (1.25: <= 1.67 quads per generator thread and step, i.e. <= kGI = 2.  Measured: 4,100 simulations 0.973 us per step
// against 1.138 for the plain two-group kernel, 5,000 1.051 vs 1.144, but 5,700 (357 groups, 2.3
// quads per thread) 1.181 vs 1.144: the generators set the step; profiles/r06/zpair.log)
constexpr double kZPairMax = 1.25;
bool zpair_shape(int groups, int cus) {
    const char* env = getenv("WCSDE_ZPAIR");
    if (env && env[0] == '0') return false;
    return groups > cus && groups <= (int)(kZPairMax * cus);
}

bool zmem_eligible_shape(int B, int N) {
    const char* env = getenv("WCSDE_ZMEM");
    if (env && env[0] == '0') return false;
    const int groups = (B + kSims - 1) / kSims;
    const int cus = cu_count();
    return tiles_for(N) == kMaxTiles && (groups <= std::min(kZMaxGroups, cus - kZMinIdle) || zpair_shape(groups, cus));
}

int cu_count() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
        return 256;
    return n;
}

// 81 <= N <= 96 (NT = 6).  Few groups of 16 sims (B <= 8192: the per-GPU shards of a
// strong-scaled sweep): the register-resident kernel with SIX waves per group, one node
// tile each (connectome fragments in VGPRs) -- the step is latency-bound there, and one
// tile per wave halves each wave's dependent chain (2,500 sims: 1.06 -> 0.83 us per step,
// tools/time_small.py); the per-tile arithmetic is the 3-wave kernel's, bit for bit.
// Many groups: ONE workgroup per CU holding SG = ceil(groups / CUs) groups that
// share the LDS connectome image (<= 155 / 128 registers): every simulation is
// resident at once (a single round of workgroups, no tail) at 3-4 waves/SIMD.
template <int X, bool PAIR = false>
int launch_zmem(const KArgs& ka, const double* sc, void* ws, hipStream_t st, int groups, int cus) {
    // one launch per block of kZK steps on the caller's stream, ONE workgroup per CU (an LDS floor
    // above half the CU's LDS): the first `groups` workgroups integrate this block from the buffered
    // normals, the other cus - groups draw the next block's normals into the other buffer.  The
    // first block's normals come from one zblock_kernel launch over the whole chip.
    const int Bp = groups * kSims;
    const size_t R = (size_t)ka.rec_every;
    float4* zb[2] = {const_cast<float4*>(ka.zbuf), const_cast<float4*>(ka.zbuf) + zmem_block_bytes(ka.B) / sizeof(float4)};
    const int K0 = std::min(kZK, ka.nsteps);
    hipLaunchKernelGGL(zblock_kernel, dim3((unsigned)((Bp * 4 + 255) / 256), (unsigned)(K0 * kMaxTiles)), dim3(256), 0, st,
                       ka.keys, ka.B, Bp, kMaxTiles, ka.step0, zb[0]);
    const int nb = (ka.nsteps + kZK - 1) / kZK;
    for (int k = 0; k < nb; ++k) {
        KArgs kb = ka;
        kb.step0 = ka.step0 + (int64_t)k * kZK;
        kb.nsteps = std::min(kZK, ka.nsteps - k * kZK);
        kb.zbuf = zb[k & 1];
        kb.zBp = Bp;
        kb.zbuf_next = zb[(k + 1) & 1];
        kb.zgen_b0 = PAIR ? groups - cus : groups;  // PAIR: the two-group workgroups come first
        kb.zgen_step0 = kb.step0 + kZK;
        kb.zgen_K = k + 1 < nb ? std::min(kZK, ka.nsteps - (k + 1) * kZK) : 0;
#ifdef WCSDE_DIAG
        if (getenv("WCSDE_ZGEN_OFF")) kb.zgen_K = 0;  // timing ablation only: later blocks read stale normals
#endif
        if (R) {  // this block's first record row (kZK is a multiple of rec_every)
            const size_t row = (size_t)k * kZK / R;
            const size_t off = ka.rec_ld ? row : row * (size_t)ka.B * ka.N;
            kb.recE = static_cast<float*>(ka.recE) + off;
            if (ka.recI) kb.recI = static_cast<float*>(ka.recI) + off;
            if (ka.recA) kb.recA = static_cast<float*>(ka.recA) + off;
        }
        int rc;
        if constexpr (PAIR) {
            // one workgroup per CU: groups - cus of them with two groups, the rest one group + generator
            constexpr int V = V_F16X3 | V_KAHAN_A | X | V_ZMEM | V_ZPAIR;
            const bool rec2 = ka.rec_every > 0 && ka.rec_ld > 0 && ka.rec_ld % 2 == 0 && !ka.recI && !ka.recA &&
                              ((uintptr_t)ka.recE & 7) == 0;
            const int extra = cus - (groups + 1) / 2;
            rc = rec2 ? launch_v<float, 6, 6, V | V_REC2, 1, 2>(kb, sc, ws, st, k == 0, extra, 96 * 1024)
                      : launch_v<float, 6, 6, V, 1, 2>(kb, sc, ws, st, k == 0, extra, 96 * 1024);
        } else {
#if WC_ZMEM_HALF
        rc = launch_v<float, 6, 12, kVarF32 | X | V_ZMEM | V_HALF2>(kb, sc, ws, st, k == 0, cus - groups, 96 * 1024);
#else
        rc = launch_v<float, 6, 6, kVarF32 | X | V_ZMEM>(kb, sc, ws, st, k == 0, cus - groups, 96 * 1024);
#endif
        }
        if (rc != WC_OK) return rc;
    }
    return wc_hip_check("wc_integrate (normals-block path)");
}

// X: extra variant bits of every product kernel (V_AII0 when a_ii == 0, the reference's value:
// -2.2% per C3 launch, bit-identical, tools/diag_variants.py 38 vs 41)
#ifndef WC_SG2
#define WC_SG2 1  // CUs < groups <= 2 CUs: two six-wave groups per workgroup (0: one group per workgroup)
#endif
template <int X>
int launch_f32_nt6(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    constexpr int V = V_F16X3 | V_KAHAN_A | X;
    const int groups = (ka.B + kSims - 1) / kSims;
    const int cus = cu_count();
    if (groups <= 2 * cus) {
        if (groups <= std::min(kZMaxGroups, cus - kZMinIdle) && ka.nsteps >= 2 * kZK && ka.zbuf &&
            (ka.rec_every == 0 || kZK % ka.rec_every == 0))
            return launch_zmem<X>(ka, sc, ws, st, groups, cus);
    }
    // node-major E-only recording (the sweep pipeline's ring): pairs of records per 8-B store
    const bool rec2 = ka.rec_every > 0 && ka.rec_ld > 0 && ka.rec_ld % 2 == 0 && !ka.recI && !ka.recA &&
                      ((uintptr_t)ka.recE & 7) == 0;
    constexpr int V2 = V | V_REC2;
    if (groups <= 2 * cus) {
        if (zpair_shape(groups, cus) && ka.nsteps >= 2 * kZK && ka.zbuf && (ka.rec_every == 0 || kZK % ka.rec_every == 0))
            return launch_zmem<X, true>(ka, sc, ws, st, groups, cus);
#if WC_SG2
        // CUs < groups <= 2 CUs (the 4-GPU C3 shard: 313 groups): two groups of six one-tile waves per
        // workgroup sharing one LDS image, 12 waves per CU.  One group per workgroup put two
        // six-wave workgroups on groups - CUs of the CUs (1.33 us per step at 5,000 simulations);
        // this runs 1.15 (tools/time_small.py variant 51, profiles/r06/small_sg2.log)
        if (groups > cus)
            return rec2 ? launch_v<float, 6, 6, V2, 1, 2>(ka, sc, ws, st) : launch_v<float, 6, 6, V, 1, 2>(ka, sc, ws, st);
#endif
        return launch_v<float, 6, 6, kVarF32 | X>(ka, sc, ws, st);
    }
    switch (std::min(5, (groups + cus - 1) / cus)) {
#ifndef WC_NO_MIX
        // three groups per CU: four waves per group with (2, 2, 1, 1) tiles rotated per group (V_MIX)
        case 3: return rec2 ? launch_v<float, 6, 4, V2 | V_MIX, 1, 3>(ka, sc, ws, st)
                            : launch_v<float, 6, 4, V | V_MIX, 1, 3>(ka, sc, ws, st);
#else
        case 3: return rec2 ? launch_v<float, 6, 3, V2, 1, 3>(ka, sc, ws, st) : launch_v<float, 6, 3, V, 1, 3>(ka, sc, ws, st);
#endif
        case 4: return rec2 ? launch_v<float, 6, 3, V2, 1, 4>(ka, sc, ws, st) : launch_v<float, 6, 3, V, 1, 4>(ka, sc, ws, st);
        default: return rec2 ? launch_v<float, 6, 3, V2, 1, 5>(ka, sc, ws, st) : launch_v<float, 6, 3, V, 1, 5>(ka, sc, ws, st);
    }
}

template <int X>
int launch_f32_x(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    switch ((tiles_for(ka.N) + 1) & ~1) {
        case 2: return launch_v<float, 2, 1, kVarF32 | X>(ka, sc, ws, st);
        case 4: return launch_v<float, 4, 2, kVarF32 | X>(ka, sc, ws, st);
        case 6: return launch_f32_nt6<X>(ka, sc, ws, st);
        default: return wc_set_err(WC_EUNSUPPORTED, "N > 96 not supported by the register-resident kernel");
    }
}

int launch_f32(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    return ka.a_ii == 0.0 ? launch_f32_x<V_AII0>(ka, sc, ws, st) : launch_f32_x<0>(ka, sc, ws, st);
}

// fp64 parity path: one wave per node tile (NW = NT; E exchanged through LDS), so the
// latency-bound step of a small batch is spread over NT waves; the per-tile MFMA order is
// the one-wave kernel's, so the results are the same bits for any NW
#ifndef WC_F64_SG
#define WC_F64_SG 2
#endif
#ifndef WC_F64_TAIL
#define WC_F64_TAIL 1
#endif
// N 81..96: WC_F64_SG groups of 16 simulations per workgroup share one LDS copy of the fp64
// connectome image (73.7 KB), one workgroup per CU.  The groups left over after the full rounds of
// WC_F64_SG x CUs, when they fit one group per CU, run as a second launch of one-group workgroups
// (WC_F64_TAIL): a CU's step with six waves takes ~0.7 of the two-group step, so the last round
// costs that instead of a whole round (1,250 groups on 256 CUs: two full rounds + 226 groups)
int launch_f64_nt6(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    constexpr int SG = WC_F64_SG;
    const int groups = (ka.B + kSims - 1) / kSims, cus = cu_count();
    const int rem = groups % (SG * cus), full = groups - rem;
    if (SG == 1 || !WC_F64_TAIL || rem == 0 || rem > cus)
        return launch_v<double, 6, 6, kVarF64, 1, SG>(ka, sc, ws, st);
    if (full > 0) {
        const int rc = launch_v<double, 6, 6, kVarF64, 1, SG>(ka, sc, ws, st, true, 0, 0, 0, full);
        if (rc != WC_OK) return rc;
    }
    return launch_v<double, 6, 6, kVarF64, 1, 1>(ka, sc, ws, st, full == 0, 0, 0, full, rem);
}
int launch_f64(const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    switch (tiles_for(ka.N)) {
        case 1: return launch_v<double, 1, 1, kVarF64>(ka, sc, ws, st);
        case 2: return launch_v<double, 2, 2, kVarF64>(ka, sc, ws, st);
        case 3: return launch_v<double, 3, 3, kVarF64>(ka, sc, ws, st);
        case 4: return launch_v<double, 4, 4, kVarF64>(ka, sc, ws, st);
        case 5: return launch_v<double, 5, 5, kVarF64>(ka, sc, ws, st);
        case 6: return launch_f64_nt6(ka, sc, ws, st);
        default: return wc_set_err(WC_EUNSUPPORTED, "N > 96 not supported by the register-resident kernel");
    }
}

#ifdef WCSDE_DIAG
// diagnostic variants (81 <= N <= 96, fp32) for on-GPU ablation; compiled only into
// libwcsde_diag.so (python -m nremmodfc_amd._build --diag), never into the product library
int launch_diag(int variant, const KArgs& ka, const double* sc, void* ws, hipStream_t st) {
    constexpr int K = V_KAHAN_A;
    switch (variant) {
        case 0: return launch_v<float, 6, 1, V_FRAG_REGS | K>(ka, sc, ws, st);          // f32 MFMA, 1 wave
        case 1: return launch_v<float, 6, 3, V_FRAG_REGS | K>(ka, sc, ws, st);          // f32 MFMA, 3 waves
        case 2: return launch_v<float, 6, 3, K>(ka, sc, ws, st);                        // f32 MFMA, LDS frags
        case 3: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS | K>(ka, sc, ws, st);  // product
        case 4: return launch_v<float, 6, 3, V_BF16X6 | K>(ka, sc, ws, st);
        case 5: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS | K, 3>(ka, sc, ws, st);
        case 6: return launch_v<float, 6, 3, V_BF16X6 | K, 4>(ka, sc, ws, st);
        case 7: return launch_v<float, 6, 2, V_BF16X6 | V_FRAG_REGS | K>(ka, sc, ws, st);
        case 8: return launch_v<float, 6, 2, V_BF16X6 | K, 3>(ka, sc, ws, st);
        case 9: return launch_v<float, 6, 6, V_BF16X6 | K>(ka, sc, ws, st);
        case 10: return launch_v<float, 6, 1, V_BF16X6 | V_FRAG_REGS | K>(ka, sc, ws, st);
        case 11: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS | K | V_NO_RNG>(ka, sc, ws, st);
        case 12: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS | K | V_NO_MFMA>(ka, sc, ws, st);
        case 13: return launch_v<float, 6, 3, V_BF16X3 | V_FRAG_REGS | K>(ka, sc, ws, st);
        case 14: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS>(ka, sc, ws, st);  // fp64 a_ie
        // one workgroup per CU: SG groups of 16 sims share the LDS connectome image
        case 15: return launch_v<float, 6, 3, V_BF16X6 | K, 1, 5>(ka, sc, ws, st);
        case 16: return launch_v<float, 6, 3, V_BF16X6 | K, 1, 4>(ka, sc, ws, st);
        case 17: return launch_v<float, 6, 3, V_BF16X6 | K, 1, 3>(ka, sc, ws, st);
        case 18: return launch_v<float, 6, 2, V_BF16X6 | K, 1, 5>(ka, sc, ws, st);
        case 19: return launch_v<float, 6, 6, V_BF16X6 | K, 1, 2>(ka, sc, ws, st);
        // node-major record buffering (needs rec_ld % 4 == 0, E records only)
        case 20: return launch_v<float, 6, 3, V_BF16X6 | K | V_REC4, 1, 5>(ka, sc, ws, st);
        case 21: return launch_v<float, 6, 3, V_BF16X6 | K | V_REC2, 1, 5>(ka, sc, ws, st);
        case 22: return launch_v<float, 6, 3, V_BF16X6 | V_FRAG_REGS | K | V_REC4>(ka, sc, ws, st);
        case 23: return launch_v<float, 6, 3, V_BF16X6 | K, 1, 5>(ka, sc, ws, st);  // = 15, node-major records
        // ablations of the grouped product kernel (15): noise off, coupling off
        case 24: return launch_v<float, 6, 3, V_BF16X6 | K | V_NO_RNG, 1, 5>(ka, sc, ws, st);
        case 25: return launch_v<float, 6, 3, V_BF16X6 | K | V_NO_MFMA, 1, 5>(ka, sc, ws, st);
        // fp16 x3 coupling: grouped (as 15), register-resident (as 3)
        case 26: return launch_v<float, 6, 3, V_F16X3 | K, 1, 5>(ka, sc, ws, st);
        case 27: return launch_v<float, 6, 3, V_F16X3 | V_FRAG_REGS | K>(ka, sc, ws, st);
        // the grouped fp16 product (26) with the normals drawn before / interleaved with the MFMAs
        case 28: return launch_v<float, 6, 3, V_F16X3 | K | V_ZFIRST, 1, 5>(ka, sc, ws, st);
        case 29: return launch_v<float, 6, 3, V_F16X3 | K | V_ZFIRST | V_ILV, 1, 5>(ka, sc, ws, st);
        case 30: return launch_v<float, 6, 3, V_F16X3 | K | V_ZFIRST | V_ILV2, 1, 5>(ka, sc, ws, st);
        // small batches (strong-scaling shards): more waves per group of 16 simulations
        case 31: return launch_v<float, 6, 6, V_F16X3 | V_FRAG_REGS | K>(ka, sc, ws, st);
        case 32: return launch_v<float, 6, 6, V_F16X3 | V_FRAG_REGS | K | V_ZFIRST>(ka, sc, ws, st);
        case 33: return launch_v<float, 6, 3, V_F16X3 | V_FRAG_REGS | K | V_ZFIRST>(ka, sc, ws, st);
        case 34: return launch_v<float, 6, 6, V_F16X3 | K>(ka, sc, ws, st);
        case 35: return launch_v<float, 6, 6, V_F16X3 | V_FRAG_REGS | K | V_ZFIRST | V_ILV2>(ka, sc, ws, st);
        case 36: return launch_v<float, 6, 2, V_F16X3 | V_FRAG_REGS | K | V_ZFIRST>(ka, sc, ws, st);
        // 37: the C3 product configuration (SG = 5, paired records) with the round-2 one-cell-per-instruction update
        case 37: return launch_v<float, 6, 3, V_F16X3 | K | V_REC2 | V_SCALAR, 1, 5>(ka, sc, ws, st);
        // the C3 product kernel (launch_f32_nt6's SG = 5 case, time-major records) and its ablations:
        // noise off, coupling MFMAs off
        case 38: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A, 1, 5>(ka, sc, ws, st);
        case 39: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_NO_RNG, 1, 5>(ka, sc, ws, st);
        case 40: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_NO_MFMA, 1, 5>(ka, sc, ws, st);
        // round 3: the C3 product kernel (38) with the a_ii = 0 sigmoid (bit-identical), the lean a_ie sum, both
        case 41: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_AII0, 1, 5>(ka, sc, ws, st);
        case 42: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_LEAN, 1, 5>(ka, sc, ws, st);
        case 43: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_LEAN | V_AII0, 1, 5>(ka, sc, ws, st);
        // the small-batch product kernel (6 waves, one tile each) and its ablations: coupling MFMAs off,
        // noise off, both off (where the latency-bound step of a strong-scaling shard goes)
        case 44: return launch_v<float, 6, 6, kVarF32 | V_AII0>(ka, sc, ws, st);
        case 45: return launch_v<float, 6, 6, kVarF32 | V_AII0 | V_NO_MFMA>(ka, sc, ws, st);
        case 46: return launch_v<float, 6, 6, kVarF32 | V_AII0 | V_NO_RNG>(ka, sc, ws, st);
        case 47: return launch_v<float, 6, 6, kVarF32 | V_AII0 | V_NO_MFMA | V_NO_RNG>(ka, sc, ws, st);
        // 256 < groups <= 512 (the 4-GPU C3 shard): two groups per workgroup sharing the LDS image
        case 50: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_AII0, 1, 2>(ka, sc, ws, st);
        case 51: return launch_v<float, 6, 6, V_F16X3 | V_KAHAN_A | V_AII0, 1, 2>(ka, sc, ws, st);
        case 52: return launch_v<float, 6, 4, V_F16X3 | V_KAHAN_A | V_AII0 | V_MIX, 1, 2>(ka, sc, ws, st);
        case 53: return launch_v<float, 6, 2, V_F16X3 | V_KAHAN_A | V_AII0, 1, 2>(ka, sc, ws, st);
        // 2 CUs < groups <= 3 CUs (the 2-GPU shard: 625 groups): three groups per workgroup
        case 54: return launch_v<float, 6, 6, V_F16X3 | V_KAHAN_A | V_AII0, 1, 3>(ka, sc, ws, st);
        case 55: return launch_v<float, 6, 3, V_F16X3 | V_KAHAN_A | V_AII0, 1, 3>(ka, sc, ws, st);
        case 56: return launch_v<float, 6, 4, V_F16X3 | V_KAHAN_A | V_AII0 | V_MIX, 1, 3>(ka, sc, ws, st);
        // the C3 product configuration (= 41, time-major records as the bench) with the >= 24-bit coupling
        case 58: return launch_v<float, 6, 3, V_F16X6 | V_KAHAN_A | V_AII0, 1, 5>(ka, sc, ws, st);
        default: return wc_set_err(WC_EINVAL, "unknown diagnostic variant");
    }
}
#endif  // WCSDE_DIAG

int make_args(KArgs& ka, const wc_params* p, int precision, int B, int N, const double* sc, const double* G,
              const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
              int64_t nsteps, double tau_ip, int64_t rec_every, int64_t rec_ld, void* recE, void* recI,
              void* recA, void* workspace, size_t ws_bytes) {
    wc_clear_err();
    if (!p || B <= 0 || N <= 0 || nsteps < 0 || nsteps > INT32_MAX || step0 < 0 || rec_every < 0 ||
        rec_every > INT32_MAX || step0 + nsteps > (int64_t(1) << 48) || rec_ld < 0 ||
        (rec_every > 0 && rec_ld > 0 && rec_ld < (nsteps + rec_every - 1) / rec_every))
        return wc_set_err(WC_EINVAL, "wc_integrate: invalid B/N/nsteps/step0/rec_every");
    if (!sc || !G || !sigmaE || !keys || !E || !I || !A)
        return wc_set_err(WC_EINVAL, "wc_integrate: NULL array argument");
    if (precision != WC_F32 && precision != WC_F64) return wc_set_err(WC_EINVAL, "wc_integrate: bad precision");
    if (rec_every > 0 && !recE) return wc_set_err(WC_EINVAL, "wc_integrate: rec_every > 0 needs recE");
    if (N > 4 * 65535) return wc_set_err(WC_EUNSUPPORTED, "wc_integrate: N > 262140 (Philox quad is 16 bits)");
    const size_t need = tiles_for(N) > kMaxTiles ? wc_large_workspace_size(B, N, precision) : frag_bytes(N, precision);
    if (!workspace || ws_bytes < need) return wc_set_err(WC_EWORKSPACE, "wc_integrate: workspace too small");
    ka.a_ee = p->a_ee; ka.a_ei = p->a_ei; ka.a_ii = p->a_ii;
    ka.tauE = p->tauE; ka.tauI = p->tauI; ka.P = p->P; ka.rhoE = p->rhoE;
    ka.rE = p->rE; ka.rI = p->rI; ka.mu = p->mu; ka.sigmaI = p->sigmaI;
    ka.sqdtD = p->sqdtD; ka.dtSim = p->dtSim; ka.tau_ip = tau_ip;
    ka.G = G; ka.sigmaE = sigmaE; ka.keys = keys; ka.E = E; ka.I = I; ka.A = A;
    ka.frag = workspace; ka.recE = recE; ka.recI = recI; ka.recA = recA;
    ka.step0 = step0; ka.rec_every = rec_every; ka.rec_ld = rec_ld; ka.nsteps = (int)nsteps; ka.B = B; ka.N = N;
    ka.zbuf = nullptr;
    ka.zBp = 0;
    ka.b0 = 0;
    if (precision == WC_F32 && zmem_eligible_shape(B, N) && ws_bytes >= zmem_offset(N) + 2 * zmem_block_bytes(B))
        ka.zbuf = reinterpret_cast<const float4*>(static_cast<char*>(workspace) + zmem_offset(N));
    return WC_OK;
}

#ifdef WCSDE_DIAG
// the fp64 parity path's straight-line elementary functions (wc_device.h, f64m), evaluated alone
// for tests/test_f64m_gpu.py: 0 exp2(t), 1 rcp(d), 2 log_u24(v), 3 sincospi_v23(v) -> (sin, cos),
// 4 the fp64 sigmoid Tr<double>::sig(x, mu = 1, s) of (x, s) pairs, 5 sqrt_pos(x); 16 + fn for 0, 2, 3:
// the same function with its coefficients read from the kCoefDev table (TabCoef, WC_F64_TAB = 1)
__global__ void f64m_kernel(int fn, int64_t n, const void* __restrict__ in, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* d = static_cast<const double*>(in);
    const uint32_t* u = static_cast<const uint32_t*>(in);
    switch (fn) {
        case 0: out[i] = f64m::exp2(d[i]); break;
        case 1: out[i] = f64m::rcp(d[i]); break;
        case 2: out[i] = f64m::log_u24(u[i]); break;
        case 3: f64m::sincospi_v23(u[i], out[2 * i], out[2 * i + 1]); break;
        case 5: out[i] = f64m::sqrt_pos(d[i]); break;
        case 16: out[i] = f64m::exp2(d[i], f64m::tab_coef()); break;
        case 18: out[i] = f64m::log_u24(u[i], f64m::tab_coef()); break;
        case 19: f64m::sincospi_v23(u[i], out[2 * i], out[2 * i + 1], f64m::tab_coef()); break;
        default: out[i] = Tr<double>::sig(d[2 * i], 1.0, d[2 * i + 1]); break;
    }
}
#endif

}  // namespace

extern "C" {

int wcsde_abi_version(void) { return WCSDE_ABI_VERSION; }

const char* wc_last_error(void) { return wc_errbuf(); }

size_t wc_workspace_size(int B, int N, int precision) {
    if (N <= 0 || B <= 0) return 0;
    if (tiles_for(N) > kMaxTiles) return wc_large_workspace_size(B, N, precision);
    // the diagnostic f32-MFMA variants need the native image; size for the larger
    const int nt = tiles_for(N);
    const size_t native = (size_t)nt * nt * 64 * 4 * (precision == WC_F64 ? 8 : 4);
    size_t need = frag_bytes(N, precision);
    if (precision == WC_F32 && zmem_eligible_shape(B, N)) need = zmem_offset(N) + 2 * zmem_block_bytes(B);
    return need > native ? need : native;
}

int wc_integrate(const wc_params* p, int precision, int B, int N, const double* sc, const double* G,
                 const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                 int64_t nsteps, double tau_ip, int64_t rec_every, int64_t rec_ld, void* recE, void* recI,
                 void* recA, void* workspace, size_t ws_bytes, void* stream) {
    KArgs ka;
    int rc = make_args(ka, p, precision, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every, rec_ld,
                       recE, recI, recA, workspace, ws_bytes);
    if (rc != WC_OK || nsteps == 0) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (tiles_for(N) > kMaxTiles)
        return wc_large_integrate(p, precision, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every,
                                  rec_ld, recE, recI, recA, workspace, st);
    return precision == WC_F64 ? launch_f64(ka, sc, workspace, st) : launch_f32(ka, sc, workspace, st);
}

int wc_integrate_status(const void* workspace, int B, int N, int precision, void* stream) {
    wc_clear_err();
    if (B <= 0 || N <= 0 || (precision != WC_F32 && precision != WC_F64))
        return wc_set_err(WC_EINVAL, "wc_integrate_status: invalid B/N/precision");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (tiles_for(N) > kMaxTiles) {
        if (!workspace) return wc_set_err(WC_EWORKSPACE, "wc_integrate_status: NULL workspace");
        return wc_large_status(workspace, B, N, precision, st);
    }
    hipError_t e = hipStreamSynchronize(st);  // N <= 96: nothing can time out; the work is finished
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}

#ifdef WCSDE_DIAG
// declared in csrc/wcsde_diag.h (tools only)
int wc_diag_integrate(int variant, const wc_params* p, int B, int N, const double* sc, const double* G,
                      const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                      int64_t nsteps, double tau_ip, int64_t rec_every, void* recE, void* workspace,
                      size_t ws_bytes, void* stream) {
    KArgs ka;
    // variants 20..37 record node-major into a dense [B*N][ld] buffer, ld = n_rec rounded up to 4
    // (38..40, the product's ablations, record time-major as the C3 pipeline does)
    const int64_t n_rec = rec_every > 0 ? (nsteps + rec_every - 1) / rec_every : 0;
    const bool nm = variant >= 20 && variant < 38;
    const int64_t ld = (nm && rec_every > 0) ? (n_rec + 3) & ~int64_t(3) : 0;
    int rc = make_args(ka, p, WC_F32, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every, ld,
                       recE, nullptr, nullptr, workspace, ws_bytes);
    if (rc != WC_OK || nsteps == 0) return rc;
    if (variant >= 100) {
        if (tiles_for(N) <= kMaxTiles) return wc_set_err(WC_EUNSUPPORTED, "wc_diag_integrate: variants >= 100 need N > 96");
        return wc_large_diag(variant, p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, workspace,
                             static_cast<hipStream_t>(stream));
    }
    if (tiles_for(N) != 6) return wc_set_err(WC_EUNSUPPORTED, "wc_diag_integrate: needs 81 <= N <= 96");
    if (ws_bytes < wc_workspace_size(B, N, WC_F32)) return wc_set_err(WC_EWORKSPACE, "wc_diag_integrate: workspace");
    return launch_diag(variant, ka, sc, workspace, static_cast<hipStream_t>(stream));
}

int wc_diag_f64m(int fn, int64_t n, const void* in, double* out, void* stream) {
    wc_clear_err();
    if (!((fn >= 0 && fn <= 5) || fn == 16 || fn == 18 || fn == 19) || n <= 0 || n > (int64_t(1) << 30) || !in || !out)
        return wc_set_err(WC_EINVAL, "wc_diag_f64m: bad arguments");
    hipLaunchKernelGGL(f64m_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       fn, n, in, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}
#endif  // WCSDE_DIAG

int wc_noise(int precision, int B, int N, const uint64_t* keys, int64_t step, void* out, void* stream) {
    wc_clear_err();
    if (B <= 0 || N <= 0 || !keys || !out || step < 0 || step >= (int64_t(1) << 48) || N > 4 * 65536)
        return wc_set_err(WC_EINVAL, "wc_noise: bad arguments");
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
    if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    return WC_OK;
}

}  // extern "C"
