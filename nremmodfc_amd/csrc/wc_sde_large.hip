// wc_sde_large.hip -- Wilson-Cowan Euler-Maruyama integrator for N > 96 (gfx950).
//
// Same model and noise stream as wc_sde.hip (wilsonCowan wc:77-83, run
// wc:86-137) for connectomes too large to keep in registers (BASELINE config 5:
// N = 1000).  The dense coupling of one Euler step over the whole batch is a
// GEMM, D[node][sim] = CM . E (M = N, N = B, K = N), so each Euler step is one
// launch of a GEMM-shaped kernel whose epilogue is the elementwise update:
//
//   * workgroup tile = 64 nodes x 64 simulations, 4 waves of 32 x 32
//     (2 x 2 MFMA 16x16 tiles); K loop over 32-node chunks fed by LDS-DMA
//     (global_load_lds_dwordx4) into 2 LDS stages (48 KB, 3 workgroups per CU;
//     3 stages at 2 workgroups per CU measured slower, as did prefetching the
//     epilogue state into registers: tools/diag_large.py variants 104, 105);
//   * fp32 product path: CM sA and E 2^10 as two fp16 parts each (22-bit
//     operands), three cross terms on v_mfma_f32_16x16x32_f16 with 1/(2^10 sA)
//     folded into G -- the coupling of wc_sde.hip.  CM's parts are pre-split in
//     the A-operand image; the epilogue writes E (fp32, tile-major) and its
//     split in the lane-linear order the DMA needs (xs_index), so the K loop is
//     DMA + ds_read_b128 + MFMA with no VALU;
//   * fp64 parity path: v_mfma_f64_16x16x4_f64 on fp64 E;
//   * the MFMA D fragment of a lane is 4 consecutive nodes of one simulation
//     = exactly one Philox4x32-10 call (quad = node/4): the epilogue draws the
//     noise, integrates E, I, a_ie (Kahan pair in fp32) and records;
//   * I, a_ie, G and sigmaE stay in a tile-major workspace image laid out like
//     the D fragment (one 16-B load per lane per array); the launch boundary
//     is the grid-wide barrier between steps (~1.5 us, cheaper than any
//     software grid barrier on this part: MI355X guide, "boundary").
// wc_integrate converts the caller's fp64 [B][N] state into this image at
// entry and back at exit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>
#include "wc_common.h"
#include "wc_device.h"

namespace {
using namespace wcdev;
typedef __attribute__((address_space(3))) void* lds_vptr;

constexpr int kTile = 64;  // node and simulation padding unit (workgroup tile edge)
constexpr int kParts = 2;  // fp16 parts per operand (hi, lo)

struct Geo {
    int B, N, Bp, Np, MT, NC, KC4;  // MT = Np/16 node tiles; NC = Np/32 fp16 chunks; KC4 = Np/4 f64 chunks
    size_t o_frag, o_scl, o_E, o_I, o_Ahi, o_Alo, o_G, o_S, o_X0, o_X1, o_GS1, o_uni, total;
};

size_t al(size_t x) { return (x + 255) & ~size_t(255); }
size_t status_offset(int B, int N, int precision);

Geo geometry(int B, int N, int precision) {
    Geo g{};
    g.B = B;
    g.N = N;
    g.Bp = (B + kTile - 1) / kTile * kTile;
    g.Np = (N + kTile - 1) / kTile * kTile;
    g.MT = g.Np / 16;
    g.NC = g.Np / 32;
    g.KC4 = g.Np / 4;
    const size_t cells = (size_t)g.Bp * g.Np;
    size_t o = 0;
    g.o_frag = o;
    if (precision == WC_F32) {
        o += al((size_t)g.MT * g.NC * kParts * 64 * 16);
        g.o_scl = o; o += al(2 * sizeof(float));  // sA, 1 / (2^10 sA)
        g.o_E = o; o += al(cells * 4);
        g.o_I = o; o += al(cells * 4);
        g.o_Ahi = o; o += al(cells * 4);
        g.o_Alo = o; o += al(cells * 4);
        g.o_G = o; o += al(cells * 4);
        g.o_S = o; o += al(cells * 4);
        g.o_X0 = o; o += al(cells * 2 * kParts);  // E 2^10 as two fp16 parts in LDS-DMA order (xs_index)
        g.o_X1 = o; o += al(cells * 2 * kParts);
        g.o_GS1 = o; o += al((size_t)g.Bp * 8);  // per-simulation (G scaled, slope) when they do not vary by node
        g.o_uni = o; o += al(sizeof(uint32_t));   // 1: every simulation's G and sigmaE are node-independent
    } else {
        o += al((size_t)g.MT * g.KC4 * 64 * 8);
        g.o_E = 0;
        g.o_I = o; o += al(cells * 8);
        g.o_Ahi = o; o += al(cells * 8);
        g.o_Alo = 0;
        g.o_G = o; o += al(cells * 8);
        g.o_S = o; o += al(cells * 8);
        g.o_X0 = o; o += al(cells * 8);
        g.o_X1 = o; o += al(cells * 8);
    }
    g.total = o;
    return g;
}

struct LArgs {
    double a_ee, a_ei, a_ii, tauE, tauI, P, rhoE, rE, rI, mu, sigmaI, sqdtD, dtSim, tau_ip;
    const uint64_t* keys;
    void* recE;
    void* recI;
    void* recA;
    int64_t rec_ld;
    int64_t step0;
    char* ws;
    Geo g;
};

// tile-major index of (sim b, node n): [b/16][n/16][lane = 16*((n%16)/4) + b%16][n%4]
__host__ __device__ __forceinline__ size_t tm_index(const Geo& g, int b, int n) {
    const int lane = 16 * ((n & 15) >> 2) + (b & 15);
    return ((((size_t)(b >> 4) * g.MT + (n >> 4)) * 64 + lane) << 2) + (n & 3);
}

// fp16 B-operand image of E 2^10 (two parts, hi + lo: 22 significant bits):
// 16-B unit ((p*NC + c)*SB + b/64)*256 + g*64 + b%64 holds, for part p, k-chunk
// c = n/32, node group g = (n%16)/4 and simulation b, the 8 values jj = 4h + r of
// nodes 16(2c + h) + 4g + r -- lane (g, b%16)'s operand.  A workgroup's (p, c)
// slab of 64 simulations is 4 KB contiguous and lands lane-linear in LDS by
// global_load_lds (position g*64 + b%64), where the wave reads it back.
__host__ __device__ __forceinline__ size_t xs_index(const Geo& g, int p, int b, int n) {
    const int c = n >> 5, h = (n >> 4) & 1, gg = (n & 15) >> 2, r = n & 3;
    const size_t unit = (((size_t)p * g.NC + c) * (g.Bp / kTile) + (b >> 6)) * 256 + gg * 64 + (b & 63);
    return unit * 8 + 4 * h + r;
}

// f64 B operand: E of node n = 4c + k, sim b at [c][b][k]
__host__ __device__ __forceinline__ size_t x64_index(const Geo& g, int b, int n) {
    return ((size_t)(n >> 2) * g.Bp + b) * 4 + (n & 3);
}

// ---- A-operand images of CM ----
// CM sA as two fp16 parts (hi = fp16(x), lo = fp16(x - hi)), sA from coupling_scale_kernel
__global__ void frag_f16_kernel(const double* __restrict__ sc, Geo g, const float* __restrict__ scl,
                                f16x8* __restrict__ frag) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // ((m*NC + c)*64 + lane)
    if (idx >= g.MT * g.NC * 64) return;
    const int lane = idx & 63;
    const int mc = idx >> 6;
    const int m = mc / g.NC, c = mc % g.NC;
    const int row = 16 * m + (lane & 15);
    const double sA = scl[0];
    f16x8 part[kParts];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int col = 16 * (2 * c + (jj >> 2)) + 4 * (lane >> 4) + (jj & 3);
        const double x = (row < g.N && col < g.N) ? sc[(size_t)row * g.N + col] * sA : 0.0;
        const _Float16 h = (_Float16)(float)x;
        part[0][jj] = h;
        part[1][jj] = (_Float16)(float)(x - (double)(float)h);
    }
#pragma unroll
    for (int p = 0; p < kParts; ++p) frag[((size_t)mc * kParts + p) * 64 + lane] = part[p];
}

__global__ void frag_f64_kernel(const double* __restrict__ sc, Geo g, double* __restrict__ frag) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // ((m*KC4 + c)*64 + lane)
    if (idx >= g.MT * g.KC4 * 64) return;
    const int lane = idx & 63;
    const int mc = idx >> 6;
    const int m = mc / g.KC4, c = mc % g.KC4;
    const int row = 16 * m + Tr<double>::row_node(lane & 15);
    const int col = 4 * c + (lane >> 4);
    frag[idx] = (row < g.N && col < g.N) ? sc[(size_t)row * g.N + col] : 0.0;
}

// ---- state in/out ----
template <typename Real>
__global__ void prep_kernel(LArgs a, const double* __restrict__ G, const double* __restrict__ sigmaE,
                            const double* __restrict__ E, const double* __restrict__ I, const double* __restrict__ A) {
    const Geo& g = a.g;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)g.Bp * g.Np) return;
    const int b = (int)(idx / g.Np), n = (int)(idx % g.Np);
    const bool ok = b < g.B && n < g.N;
    const size_t o = ok ? (size_t)b * g.N + n : 0;
    const double e = ok ? E[o] : 0.0, in = ok ? I[o] : 0.0, ai = ok ? A[o] : 0.0;
    const double gc = ok ? G[o] : 0.0, s = ok ? sigmaE[o] : 0.0;
    const size_t t = tm_index(g, b, n);
    if constexpr (sizeof(Real) == 4) {
        {
            float v[4] = {(float)e, 0.f, 0.f, 0.f};
            f16x4 h, l;
            split2h(v, h, l);
            _Float16* X = reinterpret_cast<_Float16*>(a.ws + g.o_X0);
            X[xs_index(g, 0, b, n)] = h[0];
            X[xs_index(g, 1, b, n)] = l[0];
        }
        reinterpret_cast<float*>(a.ws + g.o_E)[t] = (float)e;
        reinterpret_cast<float*>(a.ws + g.o_I)[t] = (float)in;
        AccA<true> acc;
        acc.set(ai);
        reinterpret_cast<float*>(a.ws + g.o_Ahi)[t] = acc.hi;
        reinterpret_cast<float*>(a.ws + g.o_Alo)[t] = acc.lo;
        // the MFMA sums (CM sA)(E 2^10): 1 / (2^10 sA) is folded into G (a power of two: exact)
        reinterpret_cast<float*>(a.ws + g.o_G)[t] = (float)gc * reinterpret_cast<const float*>(a.ws + g.o_scl)[1];
        reinterpret_cast<float*>(a.ws + g.o_S)[t] = Tr<float>::slope(s);
    } else {
        reinterpret_cast<double*>(a.ws + g.o_I)[t] = in;
        reinterpret_cast<double*>(a.ws + g.o_Ahi)[t] = ai;
        reinterpret_cast<double*>(a.ws + g.o_G)[t] = gc;
        reinterpret_cast<double*>(a.ws + g.o_S)[t] = s;
        reinterpret_cast<double*>(a.ws + g.o_X0)[x64_index(g, b, n)] = e;
    }
}

// homogeneous sweeps (whole_sweep_both.py) give every node of a simulation the same G and
// sigmaE: then the epilogue reads one (G, slope) pair per simulation instead of two
// per-cell images (8 of its 44 B of state per node-step).  uni starts at 1 (set by the
// host-side memset) and any node that differs from node 0 of its simulation clears it.
__global__ void uniform_params_kernel(LArgs a, const double* __restrict__ G, const double* __restrict__ sigmaE) {
    const Geo& g = a.g;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)g.B * g.N) return;
    const int b = (int)(idx / g.N);
    const size_t o0 = (size_t)b * g.N;
    if (G[idx] != G[o0] || sigmaE[idx] != sigmaE[o0]) atomicAnd(reinterpret_cast<uint32_t*>(a.ws + g.o_uni), 0u);
    if (idx == o0)
        reinterpret_cast<float2*>(a.ws + g.o_GS1)[b] =
            make_float2((float)G[o0] * reinterpret_cast<const float*>(a.ws + g.o_scl)[1], Tr<float>::slope(sigmaE[o0]));
}

template <typename Real>
__global__ void finish_kernel(LArgs a, int buf, double* __restrict__ E, double* __restrict__ I,
                              double* __restrict__ A) {
    const Geo& g = a.g;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)g.B * g.N) return;
    const int b = (int)(idx / g.N), n = (int)(idx % g.N);
    const size_t t = tm_index(g, b, n);
    if constexpr (sizeof(Real) == 4) {
        (void)buf;
        E[idx] = reinterpret_cast<const float*>(a.ws + g.o_E)[t];
        I[idx] = reinterpret_cast<const float*>(a.ws + g.o_I)[t];
        A[idx] = (double)reinterpret_cast<const float*>(a.ws + g.o_Ahi)[t] +
                 (double)reinterpret_cast<const float*>(a.ws + g.o_Alo)[t];
    } else {
        E[idx] = reinterpret_cast<const double*>(a.ws + (buf ? g.o_X1 : g.o_X0))[x64_index(g, b, n)];
        I[idx] = reinterpret_cast<const double*>(a.ws + g.o_I)[t];
        A[idx] = reinterpret_cast<const double*>(a.ws + g.o_Ahi)[t];
    }
}

// blockIdx -> (sim block, node block).  Consecutive workgroups land on
// different XCDs (round robin); each XCD gets a contiguous range of SIM blocks
// with all their node blocks.  Every XCD then streams the whole connectome image
// once per step (6.3 MB at N = 1000, shared by its concurrently running
// workgroups through its L2) and only its own columns of E -- less fabric
// traffic than splitting nodes, which would make every XCD read all of E.
__device__ __forceinline__ void tile_of(const Geo& g, int& sb, int& mb) {
    const int MB = g.Np / kTile, SB = g.Bp / kTile;
    const int W = SB * MB;
    int wid = blockIdx.x;
    if ((W & 7) == 0) wid = (blockIdx.x & 7) * (W >> 3) + (blockIdx.x >> 3);
    sb = wid / MB;
    mb = wid % MB;
}

// state arrays read and written once per step: DIAG 4 streams them past L2 (nontemporal), so that
// the connectome image the next workgroups read stays resident
template <bool NT, typename T>
__device__ __forceinline__ T ld_state(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st_state(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// wc:80-83 for one (node, simulation) cell on the fp32 product path: the folded-constant form of
// wc_sde.hip's fast path (x' = xE - mu, log2-based sigmoids, the noise scale with sqrt(2 ln 2)
// folded in for the raw Box-Muller normal, a_ie read as its high word, the a_ie increment as
// in (E dtA - rhoE dtA)), with every fusion explicit (contraction off inside).  step_kernel calls
// the scalar form, persist_kernel the packed pair form (v_pk_fma/mul/add_f32 round each
// component exactly like the scalar instruction), so the two N > 96 paths give the same bits
// whatever the surrounding code lets the compiler fuse.
struct CellConsts {
    float a_ee, Pm, rhoE, rE, rI, cIe, cIi, cI0, knoise, dtE, dtI, dtA, cA;
};
#pragma clang fp contract(off)
__device__ __forceinline__ void cell_update_f32(const CellConsts& k, float& e, float& in, AccA<true>& A, float cpl,
                                                float G, float sl, float zraw, bool pad) {
    const float e0 = e, in0 = in;
    const float ai = A.fast();
    float x = __builtin_fmaf(k.a_ee, e0, k.Pm);
    x = __builtin_fmaf(-ai, in0, x);
    x = __builtin_fmaf(G, cpl, x);
    x = __builtin_fmaf(k.knoise, zraw, x);
    const float SE = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-(x * sl)));
    const float SI = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(e0, k.cIe, __builtin_fmaf(in0, k.cIi, k.cI0))));
    e = pad ? 0.f : __builtin_fmaf(k.dtE, __builtin_fmaf(__builtin_fmaf(-k.rE, e0, 1.0f), SE, -e0), e0);
    in = __builtin_fmaf(k.dtI, __builtin_fmaf(__builtin_fmaf(-k.rI, in0, 1.0f), SI, -in0), in0);
    A.add(in0 * __builtin_fmaf(e0, k.dtA, k.cA));
}

// the same update for two cells of one simulation (nodes r, r + 1: one G and slope), packed
struct CellConsts2 {
    f2v a_ee, Pm, cIe, cIi, cI0, knoise, dtE, dtI, dtA, cA, nrE, nrI;
};
__device__ __forceinline__ CellConsts2 cell_consts2(const CellConsts& k) {
    auto b = [](float v) { return f2v{v, v}; };
    return CellConsts2{b(k.a_ee), b(k.Pm), b(k.cIe), b(k.cIi), b(k.cI0), b(k.knoise), b(k.dtE), b(k.dtI), b(k.dtA),
                       b(k.cA), b(-k.rE), b(-k.rI)};
}
__device__ __forceinline__ void cell_pair_f32(const CellConsts2& k, f2v& e, f2v& in, f2v& ahi, f2v& alo, f2v cpl,
                                              f2v G, f2v sl, f2v z, bool pad0, bool pad1) {
    const f2v e0 = e, in0 = in, one = {1.0f, 1.0f};
    f2v x = __builtin_elementwise_fma(k.a_ee, e0, k.Pm);
    x = __builtin_elementwise_fma(-ahi, in0, x);
    x = __builtin_elementwise_fma(G, cpl, x);
    x = __builtin_elementwise_fma(k.knoise, z, x);
    const f2v te = x * sl;
    const f2v de = one + f2v{__builtin_amdgcn_exp2f(-te.x), __builtin_amdgcn_exp2f(-te.y)};
    const f2v SE = {__builtin_amdgcn_rcpf(de.x), __builtin_amdgcn_rcpf(de.y)};
    const f2v ti = __builtin_elementwise_fma(e0, k.cIe, __builtin_elementwise_fma(in0, k.cIi, k.cI0));
    const f2v di = one + f2v{__builtin_amdgcn_exp2f(ti.x), __builtin_amdgcn_exp2f(ti.y)};
    const f2v SI = {__builtin_amdgcn_rcpf(di.x), __builtin_amdgcn_rcpf(di.y)};
    const f2v inc = in0 * __builtin_elementwise_fma(e0, k.dtA, k.cA);
    const f2v t = inc + alo;  // Kahan-Babuska, as AccA<true>::add
    const f2v s = ahi + t;
    alo = t - (s - ahi);
    ahi = s;
    e = __builtin_elementwise_fma(k.dtE, __builtin_elementwise_fma(__builtin_elementwise_fma(k.nrE, e0, one), SE, -e0), e0);
    if (pad0) e.x = 0.f;
    if (pad1) e.y = 0.f;
    in = __builtin_elementwise_fma(k.dtI, __builtin_elementwise_fma(__builtin_elementwise_fma(k.nrI, in0, one), SI, -in0), in0);
}
#pragma clang fp contract(on)

__host__ __device__ inline CellConsts cell_consts(double a_ee, double a_ei, double a_ii, double P, double rhoE,
                                                  double rE, double rI, double mu, double sigmaI, double sqdtD,
                                                  double dtSim, double tauE, double tauI, double tau_ip) {
    const double l2e = 1.4426950408889634;
    return CellConsts{(float)a_ee, (float)(P - mu), (float)rhoE, (float)rE, (float)rI, (float)(-a_ei * sigmaI * l2e),
                      (float)(a_ii * sigmaI * l2e), (float)(mu * sigmaI * l2e), (float)(sqdtD * (double)kSqrt2Ln2),
                      (float)(dtSim / tauE), (float)(dtSim / tauI), (float)(dtSim / tau_ip),
                      (float)(-rhoE * dtSim / tau_ip)};
}

// one Euler step of every simulation; rec_row >= 0: record the state before the update
// DIAG (ablation, tools/diag_large.py): 1 = no chunk fetch (LDS reused),
// 2 = no MFMA, 3 = no epilogue state traffic (noise + math only), 4 = nontemporal state
// loads/stores, 0 = product
template <typename Real, int DIAG = 0, int STAGES = 2, bool PF = false>
__global__ void __launch_bounds__(256) step_kernel(const LArgs a, int s, int rec_row, int buf) {
    typedef typename Tr<Real>::acc_t acc_t;
    typedef __attribute__((ext_vector_type(4))) Real real4;
    const Geo& g = a.g;
    int sb, mb;
    tile_of(g, sb, mb);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane & 15, gq = lane >> 4;
    // wave w computes node tiles m0, m0+1 x sim tiles s0, s0+1 of the 64 x 64 workgroup tile
    constexpr int NU = 2, NV = 2;
    const int m0 = mb * 4 + (w & 1) * 2;
    const int s0 = sb * 4 + (w >> 1) * 2;

    acc_t acc[NU][NV];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[u][v] = acc_t{0, 0, 0, 0};

    // PF (fp32): the epilogue's I and a_ie pair are loaded before the K loop, so their
    // latency hides behind it (48 VGPRs); G and sigmaE are read at the epilogue
    constexpr bool kPF = PF && sizeof(Real) == 4;
    real4 pfI[kPF ? NV : 1][kPF ? NU : 1], pfH[kPF ? NV : 1][kPF ? NU : 1], pfL[kPF ? NV : 1][kPF ? NU : 1];
    if constexpr (kPF) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const size_t t4 = ((size_t)(s0 + v) * g.MT + m0 + u) * 64 + lane;
                pfI[v][u] = reinterpret_cast<const real4*>(a.ws + g.o_I)[t4];
                pfH[v][u] = reinterpret_cast<const real4*>(a.ws + g.o_Ahi)[t4];
                pfL[v][u] = reinterpret_cast<const real4*>(a.ws + g.o_Alo)[t4];
            }
    }

    if constexpr (sizeof(Real) == 4) {
        // K loop fed by LDS-DMA: each 32-node k-chunk of the workgroup's A rows
        // (4 tiles x 2 fp16 parts, pre-split image) and E columns (2 parts x 64
        // sims, split by the previous step's epilogue) is 16 x 1 KB lane-linear
        // global_load_lds_dwordx4 into a ring of STAGES LDS stages (4 per wave),
        // STAGES-1 chunks in flight; a counted vmcnt + raw s_barrier retire a stage.
        // The loop body is then only ds_read_b128 + MFMA (no VALU staging).
        constexpr int kU = 2;  // A units and B units per wave per chunk
        __shared__ f16x8 lds[STAGES][2][4 * kParts * 64];  // [stage][A | B][unit][lane]
        const f16x8* F = reinterpret_cast<const f16x8*>(a.ws + g.o_frag);
        const f16x8* X = reinterpret_cast<const f16x8*>(a.ws + (buf ? g.o_X1 : g.o_X0));
        const int SB = g.Bp / kTile;
        // this wave's A units (tile ta, part pa) and B units (part pb, group gb)
        const f16x8* asrc[kU];
        const f16x8* bsrc[kU];
        int aoff[kU], boff[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i) {
            const int ua = kU * w + i, ta = ua / kParts, pa = ua % kParts;
            asrc[i] = F + ((size_t)(mb * 4 + ta) * g.NC * kParts + pa) * 64 + lane;  // + c * kParts * 64
            aoff[i] = (ta * kParts + pa) * 64;
            const int ub = kU * w + i, pb = ub / 4, gb = ub % 4;
            bsrc[i] = X + (((size_t)pb * g.NC * SB + sb) * 256 + gb * 64) + lane;  // + c * SB * 256
            boff[i] = (pb * 4 + gb) * 64;
        }
        const size_t bstep = (size_t)SB * 256;
        // K chunks in cyclic order from chunk 4 (mb / 2): the persistent kernel's order for these rows
        // (its 128-node block's own four chunks first), so both paths accumulate identically
        const int kc0 = 4 * (mb >> 1);
        auto issue = [&](int c, int st) {
            const int cc = c + kc0 < g.NC ? c + kc0 : c + kc0 - g.NC;
#pragma unroll
            for (int i = 0; i < kU; ++i) {
                __builtin_amdgcn_global_load_lds(asrc[i] + (size_t)cc * kParts * 64, (lds_vptr)(&lds[st][0][aoff[i]]), 16,
                                                 0, 0);
                __builtin_amdgcn_global_load_lds(bsrc[i] + (size_t)cc * bstep, (lds_vptr)(&lds[st][1][boff[i]]), 16, 0, 0);
            }
        };
        const int ua = (w & 1) * 2, ub = (w >> 1) * 2;  // this wave's tiles within the workgroup slab
#pragma unroll
        for (int c = 0; c < STAGES - 1; ++c)
            if (DIAG != 1 || c == 0)
                if (c < g.NC) issue(c, c);
        for (int c = 0; c < g.NC; ++c) {
            const int st = c % STAGES;
            // chunk c landed (the STAGES-2 younger chunks may stay in flight), all waves done with chunk c-1
            if (DIAG == 1 || c + STAGES - 2 >= g.NC) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else if constexpr (STAGES == 3) {
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // the younger chunk's 2 kU loads
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (DIAG != 1 && c + STAGES - 1 < g.NC) issue(c + STAGES - 1, (c + STAGES - 1) % STAGES);
            f16x8 fa[2][kParts], fb[2][kParts];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int p = 0; p < kParts; ++p) {
                    fa[u][p] = lds[DIAG == 1 ? 0 : st][0][((ua + u) * kParts + p) * 64 + lane];
                    fb[u][p] = lds[DIAG == 1 ? 0 : st][1][(p * 4 + gq) * 64 + 16 * (ub + u) + j];
                }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    if (DIAG == 2) {
                        acc[u][v][0] += (float)fa[u][0][0] * (float)fb[v][0][0];
                        continue;
                    }
                    // small terms first (2^-11: lo.hi, hi.lo; 1: hi.hi), as in wc_sde.hip
                    acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[u][1], fb[v][0], acc[u][v], 0, 0, 0);
                    acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[u][0], fb[v][1], acc[u][v], 0, 0, 0);
                    acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[u][0], fb[v][0], acc[u][v], 0, 0, 0);
                }
        }
    } else {
        const double* F = reinterpret_cast<const double*>(a.ws + g.o_frag);
        const double* X = reinterpret_cast<const double*>(a.ws + (buf ? g.o_X1 : g.o_X0));
        for (int c = 0; c < g.KC4; ++c) {  // (fp64 parity path: a requested unroll here does not apply)
            double fa[NU], fb[NV];
#pragma unroll
            for (int u = 0; u < NU; ++u) fa[u] = F[((size_t)(m0 + u) * g.KC4 + c) * 64 + lane];
#pragma unroll
            for (int v = 0; v < NV; ++v) fb[v] = X[((size_t)c * g.Bp + 16 * (s0 + v) + j) * 4 + gq];
#pragma unroll
            for (int u = 0; u < NU; ++u)
#pragma unroll
                for (int v = 0; v < NV; ++v) acc[u][v] = Tr<double>::mfma(fa[u], fb[v], acc[u][v]);
        }
    }

    // ---- epilogue: the elementwise update of wc:77-83 on the D fragments ----
    const Real a_ee = (Real)a.a_ee, a_ei = (Real)a.a_ei, a_ii = (Real)a.a_ii;
    const Real P = (Real)a.P, rhoE = (Real)a.rhoE, rE = (Real)a.rE, rI = (Real)a.rI;
    const Real mu = (Real)a.mu, slI = Tr<Real>::slope(a.sigmaI), sqdtD = (Real)a.sqdtD;
    const Real dtE = (Real)(a.dtSim / a.tauE), dtI = (Real)(a.dtSim / a.tauI), dtA = (Real)(a.dtSim / a.tau_ip);
    const Real dt = (Real)a.dtSim, tauE = (Real)a.tauE, tauI = (Real)a.tauI, tau_ip = (Real)a.tau_ip;
    const uint64_t gstep = (uint64_t)(a.step0 + s);
    const size_t BN = (size_t)g.B * g.N;
    const CellConsts kc = cell_consts(a.a_ee, a.a_ei, a.a_ii, a.P, a.rhoE, a.rE, a.rI, a.mu, a.sigmaI, a.sqdtD, a.dtSim,
                                      a.tauE, a.tauI, a.tau_ip);
    const bool uni = sizeof(Real) == 4 && __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(a.ws + g.o_uni));
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int b = 16 * (s0 + v) + j;
        const bool live = b < g.B;
        const uint64_t key = a.keys[live ? b : g.B - 1];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int mt = m0 + u;
            const int n0 = 16 * mt + 4 * gq;
            const size_t t4 = ((size_t)(s0 + v) * g.MT + mt) * 64 + lane;  // real4 index of the tile-major image
            real4* Iw = reinterpret_cast<real4*>(a.ws + g.o_I);
            real4* Ahw = reinterpret_cast<real4*>(a.ws + g.o_Ahi);
            constexpr bool kState = DIAG != 3;
            constexpr bool kNT = DIAG == 4 && sizeof(Real) == 4;
            real4 Gv, Sv;
            if (sizeof(Real) == 4 && uni) {  // one (G, slope) per simulation (uniform_params_kernel)
                const float2 gs = kState ? reinterpret_cast<const float2*>(a.ws + g.o_GS1)[live ? b : g.B - 1]
                                         : make_float2(0.16f, 11.f);
                Gv = real4{gs.x, gs.x, gs.x, gs.x};
                Sv = real4{gs.y, gs.y, gs.y, gs.y};
            } else {
                Gv = kState ? reinterpret_cast<const real4*>(a.ws + g.o_G)[t4] : real4{0.16, 0.16, 0.16, 0.16};
                Sv = kState ? reinterpret_cast<const real4*>(a.ws + g.o_S)[t4] : real4{11, 11, 11, 11};
            }
            real4 Ev, Iv;
            if constexpr (kPF) Iv = pfI[v][u];
            else Iv = kState ? ld_state<kNT>(Iw + t4) : real4{0.1, 0.1, 0.1, 0.1};
            AccA<sizeof(Real) == 4> Av[4];
            real4* Xn;  // next step's E image (f64) / tile-major E (f32)
            if constexpr (sizeof(Real) == 4) {
                // E of this lane's 4 nodes (fp32 state, tile-major like I)
                Ev = kState ? ld_state<kNT>(reinterpret_cast<const real4*>(a.ws + g.o_E) + t4)
                            : real4{0.1, 0.1, 0.1, 0.1};
                Xn = nullptr;
                real4 hi, lo;
                if constexpr (kPF) {
                    hi = pfH[v][u];
                    lo = pfL[v][u];
                } else {
                    hi = kState ? ld_state<kNT>(Ahw + t4) : real4{2.5, 2.5, 2.5, 2.5};
                    lo = kState ? ld_state<kNT>(reinterpret_cast<const real4*>(a.ws + g.o_Alo) + t4)
                                : real4{0, 0, 0, 0};
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    Av[r].hi = hi[r];
                    Av[r].lo = lo[r];
                }
            } else {
                const real4* Xc = reinterpret_cast<const real4*>(a.ws + (buf ? g.o_X1 : g.o_X0));
                const size_t x4 = (size_t)(4 * mt + gq) * g.Bp + b;  // [c][b][4] as real4
                Ev = Xc[x4];
                Xn = reinterpret_cast<real4*>(a.ws + (buf ? g.o_X0 : g.o_X1));
                const real4 av = Ahw[t4];
#pragma unroll
                for (int r = 0; r < 4; ++r) Av[r].set(av[r]);
            }
            if (rec_row >= 0 && live) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = n0 + r;
                    if (n < g.N) {
                        const size_t cc = (size_t)b * g.N + n;
                        const size_t o = a.rec_ld ? cc * a.rec_ld + rec_row : (size_t)rec_row * BN + cc;
                        static_cast<Real*>(a.recE)[o] = Ev[r];
                        if (a.recI) static_cast<Real*>(a.recI)[o] = Iv[r];
                        if (a.recA) static_cast<Real*>(a.recA)[o] = (Real)Av[r].get();
                    }
                }
            }
            Real z[4];
            if constexpr (sizeof(Real) == 4) quad_normals_raw(gstep, (uint32_t)(4 * mt + gq), key, z);
            else quad_normals(gstep, (uint32_t)(4 * mt + gq), key, z);
            real4 En, In;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool pad = n0 + r >= g.N;  // padding nodes stay exactly 0 (zero B-operand rows)
                if constexpr (sizeof(Real) == 8) {
                    const Real e = Ev[r], in = Iv[r];
                    const Real ai = Av[r].template val<Real>();
                    const Real xE = a_ee * e - ai * in + Gv[r] * acc[u][v][r] + P + sqdtD * z[r];
                    const Real SE = Tr<Real>::sig(xE, mu, Sv[r]);
                    const Real SI = Tr<Real>::sig(a_ei * e - a_ii * in, mu, slI);
                    En[r] = pad ? 0.0 : e + dt * ((-e + (1 - rE * e) * SE) / tauE);
                    In[r] = in + dt * ((-in + (1 - rI * in) * SI) / tauI);
                    Av[r].add(dt * ((in * (e - rhoE)) / tau_ip));
                } else {
                    float e = Ev[r], in = Iv[r];
                    cell_update_f32(kc, e, in, Av[r], acc[u][v][r], Gv[r], Sv[r], z[r], pad);
                    En[r] = e;
                    In[r] = in;
                }
            }
            if (kState) st_state<kNT>(Iw + t4, In);
            if constexpr (sizeof(Real) == 4) {
                // next step's B operand: the fp16 split of the new E 2^10
                float ev[4] = {En[0], En[1], En[2], En[3]};
                f16x4 ph[kParts];
                split2h(ev, ph[0], ph[1]);
                f16x4* Xo = reinterpret_cast<f16x4*>(a.ws + (buf ? g.o_X0 : g.o_X1));
#pragma unroll
                for (int p = 0; p < kParts; ++p) Xo[xs_index(g, p, b, n0) >> 2] = ph[p];
                if (!kState) continue;
                st_state<kNT>(reinterpret_cast<real4*>(a.ws + g.o_E) + t4, En);
                real4 hi, lo;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    hi[r] = Av[r].hi;
                    lo[r] = Av[r].lo;
                }
                st_state<kNT>(Ahw + t4, hi);
                st_state<kNT>(reinterpret_cast<real4*>(a.ws + g.o_Alo) + t4, lo);
            } else {
                Xn[(size_t)(4 * mt + gq) * g.Bp + b] = En;
                real4 av;
#pragma unroll
                for (int r = 0; r < 4; ++r) av[r] = Av[r].get();
                Ahw[t4] = av;
            }
        }
    }
}

template <typename Real, int DIAG = 0, int STAGES = 2, bool PF = false>
int run_large(const wc_params* p, int B, int N, const double* sc, const double* G, const double* sigmaE,
              const uint64_t* keys, double* E, double* I, double* A, int64_t step0, int64_t nsteps, double tau_ip,
              int64_t rec_every, int64_t rec_ld, void* recE, void* recI, void* recA, void* workspace,
              hipStream_t st) {
    LArgs a{};
    a.a_ee = p->a_ee; a.a_ei = p->a_ei; a.a_ii = p->a_ii; a.tauE = p->tauE; a.tauI = p->tauI;
    a.P = p->P; a.rhoE = p->rhoE; a.rE = p->rE; a.rI = p->rI; a.mu = p->mu; a.sigmaI = p->sigmaI;
    a.sqdtD = p->sqdtD; a.dtSim = p->dtSim; a.tau_ip = tau_ip;
    a.keys = keys; a.recE = recE; a.recI = recI; a.recA = recA; a.rec_ld = rec_ld; a.step0 = step0;
    a.ws = static_cast<char*>(workspace);
    a.g = geometry(B, N, sizeof(Real) == 4 ? WC_F32 : WC_F64);
    const Geo& g = a.g;
    if constexpr (sizeof(Real) == 4) {
        const int n = g.MT * g.NC * 64;
        float* scl = reinterpret_cast<float*>(a.ws + g.o_scl);
        hipLaunchKernelGGL(coupling_scale_kernel, dim3(1), dim3(1024), 0, st, sc, N, scl);
        hipLaunchKernelGGL(frag_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc, g, scl,
                           reinterpret_cast<f16x8*>(a.ws + g.o_frag));
    } else {
        const int n = g.MT * g.KC4 * 64;
        hipLaunchKernelGGL(frag_f64_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc, g,
                           reinterpret_cast<double*>(a.ws + g.o_frag));
    }
    const size_t cells = (size_t)g.Bp * g.Np;
    hipError_t se = hipMemsetAsync(a.ws + status_offset(B, N, sizeof(Real) == 4 ? WC_F32 : WC_F64), 0, 4, st);
    if (se != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(se));
    hipLaunchKernelGGL(prep_kernel<Real>, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, a, G, sigmaE, E,
                       I, A);
    if constexpr (sizeof(Real) == 4) {
        hipError_t me = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a.ws + g.o_uni), 1, 1, st);
        if (me != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(me));
        const size_t bn = (size_t)B * N;
        hipLaunchKernelGGL(uniform_params_kernel, dim3((unsigned)((bn + 255) / 256)), dim3(256), 0, st, a, G, sigmaE);
    }
    const int W = (g.Bp / kTile) * (g.Np / kTile);
    for (int64_t s = 0; s < nsteps; ++s) {
        const int rec_row = (rec_every > 0 && s % rec_every == 0) ? (int)(s / rec_every) : -1;
        hipLaunchKernelGGL((step_kernel<Real, DIAG, STAGES, PF>), dim3(W), dim3(256), 0, st, a, (int)s, rec_row,
                           (int)(s & 1));
    }
    const size_t bn = (size_t)B * N;
    hipLaunchKernelGGL(finish_kernel<Real>, dim3((unsigned)((bn + 255) / 256)), dim3(256), 0, st, a,
                       (int)(nsteps & 1), E, I, A);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? WC_OK : wc_set_err(WC_EHIP, hipGetErrorString(e));
}


// ============================================================================================
// Persistent fp32 integrator (round 5 layout): the state stays in registers for the whole call.
//
// One workgroup (8 waves) owns a tile of 128 nodes x 80 simulations for ALL nsteps steps: wave w
// holds node tile w (16 nodes) of the five 16-simulation tiles, i.e. 20 (node, sim) cells per lane
// -- E, I and the a_ie pair in VGPRs, G and the slope per simulation in LDS.  Every step the
// coupling of its 128 nodes needs the whole E image of its 80 simulations: the K loop (32-node
// chunks) runs the node block's OWN four chunks first, from LDS (the workgroup's E, written there
// by its own epilogue; their connectome rows stay resident in LDS), and then the other node blocks'
// chunks in cyclic order, two chunks (a pair) per workgroup barrier through a 3-stage LDS ring:
//   * the E image of the remote pairs comes from the workspace with 16-B sc1 buffer loads to
//     registers, issued TWO pairs ahead (and the first two as soon as the step's hand-off wait is
//     over, so that their round trip runs under the four local chunks' MFMAs);
//   * each wave streams its own node tile's connectome rows (read-only) two pairs ahead;
//   * the order is cyclic from chunk 4 nb for node block nb -- step_kernel accumulates in the same
//     order, so the two paths agree bit for bit.
// The epilogue is the packed pair update (cell_pair_f32, two cells per v_pk instruction), the
// step's Philox normals drawn there per simulation tile.
// Hand-off: MI355X_MICROARCH.md's fence-free form (its "Valid forms" consumer conditions (1)-(4)
// with row 1 of the sc1 hand-off table, whose store and load cells admit 4-, 8- or 16-B accesses;
// DESIGN.md 3.1b quotes them): the E image is stored write-through (16-B sc1 buffer stores) and every
// load of it is a 16-B sc1 buffer load to registers; every storing wave drains vmcnt before a
// workgroup barrier, after which ONE lane adds 1 to the simulation block's counter (relaxed,
// agent scope); the consumer's one lane polls that counter with relaxed agent-scope (sc1) loads,
// then a workgroup barrier releases the other waves.  Co-residency of the whole grid (one workgroup
// per CU) is guaranteed by the cooperative launch, which fails instead of running partly resident
// (the host then falls back to step_kernel).  Every wait is bounded: a timeout sets the status word,
// the state is poisoned with NaN (wc_integrate_status reports it).
// Double-buffered E image: a block writes E(s+1) into the buffer read at step s-1, which every
// block of its simulation block has finished reading (it passed that block's step-s wait).
constexpr int kPN = 128, kPS = 80, kPT = kPS / 16;  // nodes, simulations, simulation tiles per workgroup
constexpr int kPWaves = kPN / 16;                     // 8
constexpr int kPLoc = 4;                              // local K chunks (the node block's own nodes)
constexpr int kPStages = 3;                           // LDS ring of chunk pairs
constexpr uint32_t kSpinLimit = 1u << 22;             // polls per wait before giving up (~seconds)
constexpr int kPersistRetry = 1;                      // run_persistent: cooperative launch refused

struct PGeo {
    int B, N, Np, Bp, MT, NC, SBp, NBp;
    int nbx, gn, sbx;  // XCD placement: nbx node blocks x sbx simulation blocks per XCD (gn node groups); nbx = 0: plain order
    size_t o_frag, o_scl, o_x, o_cnt, o_err, total;
};

// blockIdx -> (simulation block, node block).  Workgroup b runs on XCD b % 8 (dispatch order;
// used for speed only, nothing depends on it): each XCD gets nbx node blocks of sbx simulation
// blocks, so its L2 holds nbx x 128 connectome rows across steps and each E-image line it
// fetches is read by nbx workgroups
void pplace(PGeo& g, int nbx) {
    g.nbx = 0;
    const int W = g.SBp * g.NBp;
    if (nbx <= 0 || W % 8 || g.NBp % nbx) return;
    const int gn = g.NBp / nbx;
    if (8 % gn || g.SBp % (8 / gn)) return;
    g.nbx = nbx;
    g.gn = gn;
    g.sbx = g.SBp / (8 / gn);
}

__device__ __forceinline__ void pblock(const PGeo& g, int& sb, int& nb) {
    const int b = blockIdx.x;
    if (g.nbx == 0) {
        sb = b % g.SBp;
        nb = b / g.SBp;
        return;
    }
    const int x = b & 7, r = b >> 3;
    nb = (x % g.gn) * g.nbx + r % g.nbx;
    sb = (x / g.gn) * g.sbx + r / g.nbx;
}

PGeo pgeometry(int B, int N) {
    PGeo g{};
    g.B = B;
    g.N = N;
    g.Np = (N + kPN - 1) / kPN * kPN;
    g.Bp = (B + kPS - 1) / kPS * kPS;
    g.MT = g.Np / 16;
    g.NC = g.Np / 32;
    g.SBp = g.Bp / kPS;
    g.NBp = g.Np / kPN;
    size_t o = 0;
    g.o_frag = o; o += al((size_t)g.MT * g.NC * kParts * 64 * 16);
    g.o_scl = o; o += al(2 * sizeof(float));
    g.o_x = o; o += al(2 * (size_t)g.Np * g.Bp * 4);   // two fp16x2 E images
    g.o_cnt = o; o += al((size_t)g.SBp * 64);           // one counter per simulation block, 64 B apart
    g.total = o;
    g.o_err = 0;  // set by status_offset (after both layouts)
    return g;
}

// The status word of the last N > 96 call on a workspace sits after both layouts (the step and the
// persistent path reuse the same workspace): each call clears it, a persistent call whose
// inter-workgroup wait timed out sets it; wc_integrate_status reads it (no host state anywhere).
size_t status_offset(int B, int N, int precision) {
    const size_t st = geometry(B, N, precision).total;
    if (precision != WC_F32) return st;
    const size_t pe = pgeometry(B, N).total;
    return st > pe ? st : pe;
}

struct PArgs {
    CellConsts kc;  // folded on the host (cell_consts): no fp64 constant math inside the step loop
    const uint64_t* keys;
    const double* G;
    const double* sigmaE;
    double* E;
    double* I;
    double* A;
    void* recE;
    void* recI;
    void* recA;
    int64_t rec_ld, rec_every, step0, nsteps;
    char* ws;
    PGeo g;
};

// E image unit (k-chunk c, simulation block sb, simulation tile t, half h) of 64 lanes x 16 B: lane
// (g, j) holds [hi | lo] (f16x4 each) of nodes 16 (2c + h) + 4g + r, r < 4, of simulation 80 sb +
// 16 t + j -- written whole by the wave of node tile 2c + h; the 10 units of a (chunk, simulation
// block) are 10 contiguous KB, and the staging splits each piece into the two parts' B fragments
__host__ __device__ __forceinline__ uint32_t pimg_unit16(const PGeo& g, int c, int sb, int t, int h) {
    return (uint32_t)((((size_t)c * g.SBp + sb) * kPT + t) * 2 + h);
}

// DIAG (timing ablations only, diag build, WCSDE_PERSISTENT=2..7; results are wrong): 1 = no MFMA,
// 2 = no epilogue arithmetic, 3 = no remote E-image loads (stale stages), 4 = no hand-off waits,
// 5 = half the B-fragment LDS reads (lo part reuses hi), 6 = a fifth of them (tile 0's for all)
// NRP_T >= 0: the number of remote chunk pairs (NC - 4) / 2 at compile time, the remote K loop
// fully unrolled (straight-line code keeps the compiler's vmcnt bookkeeping exact: a loop header
// merges states and waits for every load in flight); -1: a runtime loop, any N
template <int DIAG = 0, int NRP_T = -1>
__global__ void __launch_bounds__(kPWaves * 64, 1) persist_kernel(const PArgs a) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    // ring of chunk-pair stages [stage][chunk of the pair][part x sim tile][lane] (60 KB): stages 0
    // and 1 hold the local pairs at the start of a step (written by the epilogue), remote pair k
    // lands in stage (k + 2) % 3; the local chunks' connectome rows, resident (64 KB)
    __shared__ f16x8 ldsB[kPStages][2][kParts * kPT][64];
    __shared__ u2 ldsDummy[256][2];  // stage_pair's unit-less loads land here
    __shared__ f16x8 ldsA[kPLoc][kPWaves][kParts][64];
    __shared__ float2 ldsGS[kPS];
    __shared__ uint64_t ldsK[kPS];
    __shared__ int go, uni;
    const PGeo& g = a.g;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, j = lane & 15, gq = lane >> 4;
    int sb, nb;
    pblock(g, sb, nb);
    const int mt = nb * kPWaves + w;  // this wave's node tile
    const int n0 = 16 * mt + 4 * gq;
    const int c0 = kPLoc * nb;        // the node block's own chunks: c0 .. c0 + 3
    const int NRP = NRP_T >= 0 ? NRP_T : (g.NC - kPLoc) / 2;  // remote pairs (NC is a multiple of 4: even)
    const float gscale = reinterpret_cast<const float*>(a.ws + g.o_scl)[1];
    unsigned* cnt = reinterpret_cast<unsigned*>(a.ws + g.o_cnt) + sb * 16;
    unsigned* err = reinterpret_cast<unsigned*>(a.ws + g.o_err);
    const uint32_t img_bytes = (uint32_t)((size_t)g.Np * g.Bp * 4);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(a.ws + g.o_x, 0, (int)(2 * img_bytes), 0x00020000);
    const f16x8* F = reinterpret_cast<const f16x8*>(a.ws + g.o_frag);
    const f16x8* asrc = F + (size_t)mt * g.NC * kParts * 64 + lane;  // this wave's connectome rows, + c * 128

    // ---- state into registers (step_kernel's prep_kernel arithmetic); G and slope per
    // simulation when this workgroup's cells do not vary by node (every sweep but the maps
    // modes), else read per cell at each step ----
    if (tid == 0) uni = 1;
    if (tid < kPS) {
        const int b = sb * kPS + tid;
        const int bb = b < g.B ? b : g.B - 1;
        ldsK[tid] = a.keys[bb];
        ldsGS[tid] = b < g.B ? make_float2((float)a.G[(size_t)bb * g.N] * gscale, Tr<float>::slope(a.sigmaE[(size_t)bb * g.N]))
                             : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < kPLoc; ++i)
#pragma unroll
        for (int p = 0; p < kParts; ++p) ldsA[i][w][p][lane] = asrc[(size_t)(c0 + i) * kParts * 64 + p * 64];
    __syncthreads();
    f2v E[kPT][2], I[kPT][2], Ah[kPT][2], Al[kPT][2];  // cells (t, 2q + {0, 1}): nodes n0 + 2q, n0 + 2q + 1
    bool my_uni = true;
#pragma unroll
    for (int t = 0; t < kPT; ++t) {
        const int b = sb * kPS + 16 * t + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = n0 + r;
            const bool ok = b < g.B && n < g.N;
            const size_t o = ok ? (size_t)b * g.N + n : 0;
            AccA<true> acc0;
            acc0.set(ok ? a.A[o] : 0.0);
            E[t][r >> 1][r & 1] = ok ? (float)a.E[o] : 0.f;
            I[t][r >> 1][r & 1] = ok ? (float)a.I[o] : 0.f;
            Ah[t][r >> 1][r & 1] = acc0.hi;
            Al[t][r >> 1][r & 1] = acc0.lo;
            if (ok && (a.G[o] != a.G[(size_t)b * g.N] || a.sigmaE[o] != a.sigmaE[(size_t)b * g.N])) my_uni = false;
        }
    }
    if (!my_uni) uni = 0;  // benign race: every writer stores 0
    const bool pad0 = n0 >= g.N, pad1 = n0 + 1 >= g.N, pad2 = n0 + 2 >= g.N, pad3 = n0 + 3 >= g.N;

    // publish this wave's E tiles into image `buf` (sc1, write-through) and signal the simulation
    // block; then (after that barrier: every wave has finished reading the ring) write them into the
    // ring's local stages for this workgroup's next K loop
    auto publish = [&](int buf) {
        u4 piece[kPT];
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            const float ev[4] = {E[t][0].x, E[t][0].y, E[t][1].x, E[t][1].y};
            f16x4 ph[kParts];
            split2h(ev, ph[0], ph[1]);
            const u2 h0 = __builtin_bit_cast(u2, ph[0]), h1 = __builtin_bit_cast(u2, ph[1]);
            piece[t] = u4{h0.x, h0.y, h1.x, h1.y};
            const uint32_t unit = pimg_unit16(g, mt >> 1, sb, t, mt & 1);
            __builtin_amdgcn_raw_buffer_store_b128(piece[t], xrs, (int)(buf * img_bytes + (unit * 64 + lane) * 16), 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // local chunk i = w / 2 (node tiles 2i, 2i + 1 of the block), half h = w % 2: stage i / 2,
        // chunk-of-pair i % 2 -- the layout the staging gives the remote chunks
        const int i = w >> 1, hh = w & 1;
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            *reinterpret_cast<u2*>(reinterpret_cast<unsigned*>(&ldsB[i >> 1][i & 1][t][lane]) + 2 * hh) = u2{piece[t].x, piece[t].y};
            *reinterpret_cast<u2*>(reinterpret_cast<unsigned*>(&ldsB[i >> 1][i & 1][kPT + t][lane]) + 2 * hh) = u2{piece[t].z, piece[t].w};
        }
    };
    // consumer: one lane polls the counter (relaxed agent-scope = sc1 loads); the workgroup barrier
    // after it releases the other waves (and makes the local stages visible); bounded
    auto wait_for = [&](unsigned target) -> bool {
        if (tid == 0) {
            int ok = DIAG == 4;
            for (uint32_t it = 0; !ok && it < kSpinLimit; ++it) {
                if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
                    ok = 1;
                    break;
                }
                if ((it & 63) == 63 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            go = ok;
        }
        __syncthreads();
        return go != 0;
    };

    publish(0);
    const bool uni_wg = uni != 0;  // (the barrier inside publish ordered every store to it)
    const CellConsts kc = a.kc;
    CellConsts2 k2 = cell_consts2(kc);
    // the packed cell constants pinned in VGPR pairs (as SGPR pairs they crowd the scalar file, see rchunk)
    asm volatile("" : "+v"(k2.a_ee), "+v"(k2.Pm), "+v"(k2.cIe), "+v"(k2.cIi), "+v"(k2.cI0), "+v"(k2.knoise));
    asm volatile("" : "+v"(k2.dtE), "+v"(k2.dtI), "+v"(k2.dtA), "+v"(k2.cA), "+v"(k2.nrE), "+v"(k2.nrI));
    const size_t BN = (size_t)g.B * g.N;
    int rec_cnt = 0, rec_row = 0;

    // remote pair k: chunks (c0 + 4 + 2k) % NC and the next; thread tid stages units tid, tid + 512
    // and (tid < 256) tid + 1024 of the pair's 1280 (out-of-range buffer loads return 0 and move
    // nothing: every wave issues the same three loads)
    // Every load of the K loop is issued unconditionally, in the same order every iteration, so that
    // the compiler's in-order vmcnt bookkeeping stays exact (a load skipped on some path makes it wait
    // for everything): a load with nothing to fetch gets an out-of-range buffer offset (zeros, no
    // memory traffic).  Unit q of a pair for thread tid is unit ul = tid + 512 q of its 1280: byte
    // qo[q] of the image (pair base excluded) and, staged, the LDS bytes qs[q] of a stage (units
    // beyond 1280, q = 2 for tid >= 256, go to a dummy slot of their own).
    const uint32_t chunk_bytes = (uint32_t)(g.SBp * (kPT * 2 * 64 * 16));  // one k-chunk of the image
    const uint32_t sb_off = (uint32_t)(sb * (kPT * 2 * 64 * 16));
    const uint32_t oob = 2 * img_bytes;
    // (lane-linear: a wave loads one contiguous 1-KB unit; pairing a thread's units as the two 8-B
    // halves of one LDS slot was slower, docs/CHANGELOG.md round 5)
    uint32_t qo[3], qs[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int ul = tid + 512 * q;
        const int h = ul >= 640 ? 1 : 0;
        const int ulc = ul - 640 * h;
        const int u = ulc >> 6, ln = ulc & 63, t = u >> 1, hh = u & 1;
        qo[q] = (ul < 1280) ? h * chunk_bytes + ulc * 16 : oob;
        // byte offset in a stage of the hi half (the lo half is kPT * 1 KB further)
        qs[q] = (ul < 1280) ? (uint32_t)(((h * kParts * kPT + t) * 64 + ln) * 16 + 8 * hh) : 0u;
    }
    const __amdgpu_buffer_rsrc_t frs =
        __builtin_amdgcn_make_buffer_rsrc(a.ws + g.o_frag, 0, (int)((size_t)g.MT * g.NC * kParts * 64 * 16), 0x00020000);
    const uint32_t row_off = (uint32_t)(((size_t)mt * g.NC * kParts * 64 + lane) * 16);  // this wave's rows, chunk 0
    const uint32_t frag_oob = (uint32_t)((size_t)g.MT * g.NC * kParts * 64 * 16);
    constexpr int kLead = 2;  // remote pairs whose E image is in flight in registers
    u4 rb[kLead][3];
    f16x8 fa[2][2][kParts];  // rows of the pair [slot][chunk of the pair][part], one pair ahead
    // chunk index of remote pair k: (c0 + 4 + 2k) mod NC.  Its inputs are laundered at the top of
    // every step: as step-invariants the unrolled loop's ~30 per-pair offsets are hoisted into SGPRs,
    // overflow the file and push the buffer descriptors into VGPR lanes, re-read by 16 v_readlane
    // before every load group (313 readlanes per step before, 27 after, with the constants above)
    int c0v = c0, ncv = g.NC;
    uint32_t cbv = chunk_bytes, sbv = sb_off;
    auto rchunk = [&](int k) {
        const int c = c0v + kPLoc + 2 * k;
        return c < ncv ? c : c - ncv;
    };
    // (the pair's uniform base goes in the SGPR offset operand and the lane's part in the VGPR one, so
    // an address costs no VALU; a pair past the last, k >= NRP, loads from an out-of-range offset)
    auto load_rows = [&](int k, int slot) {
        const bool live_k = k < NRP;
        const int so = live_k ? (int)((uint32_t)rchunk(k) * (kParts * 64 * 16)) : 0;
        const uint32_t vo = live_k ? row_off : frag_oob;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int p = 0; p < kParts; ++p)
                fa[slot][h][p] = __builtin_bit_cast(
                    f16x8, __builtin_amdgcn_raw_buffer_load_b128(frs, (int)(vo + (uint32_t)((h * kParts + p) * 64 * 16)), so, 0));
    };
    auto load_pair = [&](int k, int slot, int buf) {
        const bool live_k = DIAG != 3 && k < NRP;
        const int so = live_k ? (int)(buf * img_bytes + (uint32_t)rchunk(k) * cbv + sbv) : 0;
#pragma unroll
        for (int q = 0; q < 3; ++q)
            rb[slot][q] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xrs, (int)(live_k ? qo[q] : oob), so, 16));
    };
    char* const ring = reinterpret_cast<char*>(&ldsB[0][0][0][0]);
    auto stage_pair = [&](int slot, int st) {
        if (DIAG == 3) return;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const u4 v = rb[slot][q];
            char* d = ring + (size_t)st * sizeof(ldsB[0]) + qs[q];
            char* dl = d + kPT * 64 * 16;
            if (q == 2) {  // (tid >= 256: no unit; its zeros go to a dummy slot, without a branch)
                d = tid < 256 ? d : reinterpret_cast<char*>(&ldsDummy[tid & 255][0]);
                dl = tid < 256 ? dl : reinterpret_cast<char*>(&ldsDummy[tid & 255][1]);
            }
            *reinterpret_cast<u2*>(d) = u2{v.x, v.y};
            *reinterpret_cast<u2*>(dl) = u2{v.z, v.w};
        }
    };
    // the MFMAs of one chunk: A from (a0, a1), B from ring stage st, chunk-of-pair h
    auto mfma_chunk = [&](f16x8 a0, f16x8 a1, int st, int h, f4 (&acc)[kPT]) {
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            // (DIAG 5: the lo part's B reads skipped, DIAG 6: one simulation tile's fragments for all
            // five -- the ablations of the LDS read traffic, 8 waves x 10 KB per chunk)
            const f16x8 fb0 = ldsB[st][h][DIAG == 6 ? 0 : t][lane];
            const f16x8 fb1 = DIAG == 5 ? fb0 : ldsB[st][h][kPT + (DIAG == 6 ? 0 : t)][lane];
            if (DIAG == 1) {
                acc[t][0] += (float)fb0[0] + (float)a0[0] + (float)fb1[1] + (float)a1[1];
                continue;
            }
            // small terms first (2^-11: lo.hi, hi.lo; 1: hi.hi), as in step_kernel
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, fb0, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, fb1, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, fb0, acc[t], 0, 0, 0);
        }
    };
    // remote pair k in ring stage st: its E image staged (loaded two pairs ago), one barrier, the
    // next pair's rows (into the other row slot) and the E image two pairs ahead issued, the MFMAs
    // (E-image register slot es = k mod kLead, row slot rs = k mod 2)
    auto remote_pair = [&](int k, int es, int rs, int st, int buf, f4 (&acc)[kPT]) {
        stage_pair(es, st);
        __syncthreads();
        load_rows(k + 1, rs ^ 1);
        load_pair(k + kLead, es, buf);
        mfma_chunk(fa[rs][0][0], fa[rs][0][1], st, 0, acc);
        mfma_chunk(fa[rs][1][0], fa[rs][1][1], st, 1, acc);
    };

    bool alive = true;
    for (int64_t s = 0; s < a.nsteps; ++s) {
        const int buf = (int)(s & 1);
        asm volatile("" : "+s"(c0v), "+s"(ncv), "+s"(cbv), "+s"(sbv));
        if (!wait_for((unsigned)g.NBp * (unsigned)(s + 1))) {
            alive = false;
            break;
        }
        const bool rec = a.rec_every > 0 && rec_cnt == 0;
        if (a.rec_every > 0) {
            if (rec_cnt == 0) rec_cnt = (int)a.rec_every;
            --rec_cnt;
        }
        load_pair(0, 0, buf);
        load_rows(0, 0);
#pragma unroll
        for (int k = 1; k < kLead; ++k) load_pair(k, k, buf);
        asm volatile("" ::: "memory");  // (the loads stay here, ahead of the local chunks' MFMAs)
        f4 acc[kPT];
#pragma unroll
        for (int t = 0; t < kPT; ++t) acc[t] = f4{0, 0, 0, 0};
        // local chunks (stages 0 and 1, rows from ldsA)
        const uint64_t gstep = (uint64_t)(a.step0 + s);
        f2v z[kPT][2];
        auto noise = [&](int t) {
            float zz[4];
            quad_normals_raw(gstep, (uint32_t)(4 * mt + gq), ldsK[16 * t + j], zz);
            z[t][0] = f2v{zz[0], zz[1]};
            z[t][1] = f2v{zz[2], zz[3]};
        };
#pragma unroll
        for (int i = 0; i < kPLoc; ++i) {
            mfma_chunk(ldsA[i][w][0][lane], ldsA[i][w][1][lane], i >> 1, i & 1, acc);
        }
        // remote pairs, two per iteration (the staging and row registers alternate)
        if constexpr (NRP_T >= 0) {
#pragma unroll
            for (int k = 0; k < NRP_T; ++k) remote_pair(k, k % kLead, k & 1, (k + 2) % kPStages, buf, acc);
        } else {
            int st = 2;  // remote pair k lands in ring stage (k + 2) mod 3
            for (int k = 0; k < NRP; k += 2) {
                remote_pair(k, 0, 0, st, buf, acc);
                st = st == kPStages - 1 ? 0 : st + 1;
                remote_pair(k + 1, 1, 1, st, buf, acc);
                st = st == kPStages - 1 ? 0 : st + 1;
            }
        }
        // ---- epilogue: the packed cell update on the D fragments (the state in registers) ----
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            __builtin_amdgcn_sched_barrier(0);  // one simulation tile at a time: bounded live ranges
            const int b = sb * kPS + 16 * t + j;
            const bool live = b < g.B;
            // record offsets and per-cell parameter addresses recomputed here (opaque N, ld):
            // hoisted out of the step loop they would pin dozens of VGPRs of 64-bit addresses
            int Nn = g.N;
            int64_t ld = a.rec_ld;
            asm volatile("" : "+s"(Nn), "+s"(ld));
            if (rec && live) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = n0 + r;
                    if (n < Nn) {
                        const size_t cc = (size_t)b * Nn + n;
                        const size_t o = ld ? cc * ld + rec_row : (size_t)rec_row * BN + cc;
                        static_cast<float*>(a.recE)[o] = E[t][r >> 1][r & 1];
                        if (a.recI) static_cast<float*>(a.recI)[o] = I[t][r >> 1][r & 1];
                        if (a.recA) static_cast<float*>(a.recA)[o] = (float)((double)Ah[t][r >> 1][r & 1] + (double)Al[t][r >> 1][r & 1]);
                    }
                }
            }
            if (DIAG == 2) {
#pragma unroll
                for (int q = 0; q < 2; ++q) E[t][q] += 1e-30f * f2v{acc[t][2 * q], acc[t][2 * q + 1]};
                continue;
            }
            noise(t);
            f2v gv, sv;
            f2v gv1, sv1;
            if (uni_wg) {
                const float2 gs = ldsGS[16 * t + j];
                gv = gv1 = f2v{gs.x, gs.x};
                sv = sv1 = f2v{gs.y, gs.y};
            } else {
                float gg[4], ss[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = n0 + r;
                    const bool ok = live && n < Nn;
                    const size_t o = ok ? (size_t)b * Nn + n : 0;
                    gg[r] = ok ? (float)a.G[o] * gscale : 0.f;
                    ss[r] = ok ? Tr<float>::slope(a.sigmaE[o]) : 0.f;
                }
                gv = f2v{gg[0], gg[1]};
                gv1 = f2v{gg[2], gg[3]};
                sv = f2v{ss[0], ss[1]};
                sv1 = f2v{ss[2], ss[3]};
            }
            cell_pair_f32(k2, E[t][0], I[t][0], Ah[t][0], Al[t][0], f2v{acc[t][0], acc[t][1]}, gv, sv, z[t][0], pad0,
                          pad1);
            cell_pair_f32(k2, E[t][1], I[t][1], Ah[t][1], Al[t][1], f2v{acc[t][2], acc[t][3]}, gv1, sv1, z[t][1], pad2,
                          pad3);
        }
        if (rec) ++rec_row;
        if (s + 1 < a.nsteps) publish(buf ^ 1);
    }
    // ---- state back to the caller's fp64 arrays (NaN if a wait timed out) ----
    const bool poisoned = !alive;
#pragma unroll
    for (int t = 0; t < kPT; ++t) {
        const int b = sb * kPS + 16 * t + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = n0 + r;
            if (b < g.B && n < g.N) {
                const size_t o = (size_t)b * g.N + n;
                a.E[o] = poisoned ? __builtin_nan("") : (double)E[t][r >> 1][r & 1];
                a.I[o] = poisoned ? __builtin_nan("") : (double)I[t][r >> 1][r & 1];
                a.A[o] = poisoned ? __builtin_nan("") : (double)Ah[t][r >> 1][r & 1] + (double)Al[t][r >> 1][r & 1];
            }
        }
    }
}

constexpr int kPThreads = kPWaves * 64;
template <int DIAG>
const void* persist_for(int nrp) {
    switch (nrp) {
        case 14: return (const void*)persist_kernel<DIAG, 14>;
        default: return (const void*)persist_kernel<DIAG, -1>;
    }
}

int cu_count_large() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return n;
}

// The product path for fp32 N > 96 whenever every workgroup gets a CU of its own (residency) and
// the image offsets fit the 32-bit buffer descriptors.  C5 bench: 28.2 us per step against the
// step kernel's 31.8.  WCSDE_PERSISTENT=0 forces step_kernel; in the diag build
// (libwcsde_diag.so) 2..5 select the timing ablations (wrong results).
bool persistent_ok(int B, int N) {
    const char* env = getenv("WCSDE_PERSISTENT");
    if (env && (env[0] < '1' || env[0] > '7')) return false;
    const PGeo g = pgeometry(B, N);
    if (2 * (size_t)g.Np * g.Bp * 4 >= (size_t)INT32_MAX) return false;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persist_for<0>((g.NC - kPLoc) / 2), kPThreads, 0) != hipSuccess ||
        occ < 1)
        return false;
    return g.SBp * g.NBp <= cu_count_large();
}

int run_persistent(const wc_params* p, int B, int N, const double* sc, const double* G, const double* sigmaE,
                   const uint64_t* keys, double* E, double* I, double* A, int64_t step0, int64_t nsteps,
                   double tau_ip, int64_t rec_every, int64_t rec_ld, void* recE, void* recI, void* recA,
                   void* workspace, hipStream_t st) {
    PArgs a{};
    a.kc = cell_consts(p->a_ee, p->a_ei, p->a_ii, p->P, p->rhoE, p->rE, p->rI, p->mu, p->sigmaI, p->sqdtD, p->dtSim,
                       p->tauE, p->tauI, tau_ip);
    a.keys = keys; a.G = G; a.sigmaE = sigmaE; a.E = E; a.I = I; a.A = A;
    a.recE = recE; a.recI = recI; a.recA = recA; a.rec_ld = rec_ld; a.rec_every = rec_every;
    a.step0 = step0; a.nsteps = nsteps;
    a.ws = static_cast<char*>(workspace);
    a.g = pgeometry(B, N);
    a.g.o_err = status_offset(B, N, WC_F32);
    // 4 node blocks x 8 simulation blocks per XCD measured 1.5-2% faster than the plain order and
    // than 1, 2 or 8 node blocks per XCD (C5 shard, tools/time_pmap.py); WCSDE_PMAP overrides
    const char* pm = getenv("WCSDE_PMAP");
    pplace(a.g, pm ? atoi(pm) : 4);
    const PGeo& g = a.g;
    // connectome image in the 128-node padding (frag_f16_kernel takes a Geo)
    Geo fg{};
    fg.N = N;
    fg.Np = g.Np;
    fg.MT = g.MT;
    fg.NC = g.NC;
    float* scl = reinterpret_cast<float*>(a.ws + g.o_scl);
    hipLaunchKernelGGL(coupling_scale_kernel, dim3(1), dim3(1024), 0, st, sc, N, scl);
    const int n = g.MT * g.NC * 64;
    hipLaunchKernelGGL(frag_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc, fg, scl,
                       reinterpret_cast<f16x8*>(a.ws + g.o_frag));
    hipError_t me = hipMemsetAsync(a.ws + g.o_cnt, 0, g.total - g.o_cnt, st);  // counters
    if (me == hipSuccess) me = hipMemsetAsync(a.ws + g.o_err, 0, 4, st);        // this call's status word
    if (me != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(me));
    const dim3 grid((unsigned)(g.SBp * g.NBp)), blk(kPThreads);
    const int nrp = (g.NC - kPLoc) / 2;
    const void* kern = persist_for<0>(nrp);
#ifdef WCSDE_DIAG
    const char* env = getenv("WCSDE_PERSISTENT");
    switch (env ? env[0] : '1') {
        case '2': kern = persist_for<1>(nrp); break;
        case '3': kern = persist_for<2>(nrp); break;
        case '4': kern = persist_for<3>(nrp); break;
        case '5': kern = persist_for<4>(nrp); break;
        case '6': kern = persist_for<5>(nrp); break;
        case '7': kern = persist_for<6>(nrp); break;
        default: break;
    }
#endif
    // cooperative: the whole grid is co-resident (the inter-workgroup waits need it) or the launch
    // fails -- e.g. another process holds CUs -- and the caller runs step_kernel instead
    void* kargs[] = {&a};
    // WCSDE_COOP=0 (profiling only): an ordinary launch of the same one-workgroup-per-CU grid, all
    // resident on an otherwise idle GPU; rocprofv3 runs of a process that made a cooperative launch
    // die in the runtime's teardown, an ordinary launch lets one run hold several
    // counter passes.  Nothing is guaranteed co-resident then: a wait that cannot be met times out
    // (status word, NaN state), it does not hang.
    const char* coop = getenv("WCSDE_COOP");
    hipError_t e = (coop && coop[0] == '0') ? hipLaunchKernel(kern, grid, blk, kargs, 0, st)
                                            : hipLaunchCooperativeKernel(kern, grid, blk, kargs, 0, st);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return kPersistRetry;
    }
    // no host synchronisation: a wait that timed out set the status word and poisoned E, I, a_ie with
    // NaN (which every later call on this state carries); wc_integrate_status reads the word when the
    // caller chooses (e.g. at the end of a batch)
    return WC_OK;
}

}  // namespace

// internal entry points used by wc_sde.hip's dispatcher
size_t wc_large_workspace_size(int B, int N, int precision) {
    return status_offset(B, N, precision) + al(4);  // both layouts (same workspace, reused) + the status word
}

int wc_large_status(const void* workspace, int B, int N, int precision, hipStream_t st) {
    unsigned word = 0;
    const char* w = static_cast<const char*>(workspace) + status_offset(B, N, precision);
    hipError_t e = hipMemcpyAsync(&word, w, sizeof(word), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return wc_set_err(WC_EHIP, hipGetErrorString(e));
    if (word)
        return wc_set_err(WC_EHIP, "wc_integrate: persistent N > 96 integrator: an inter-workgroup wait timed out "
                                   "(state poisoned with NaN)");
    return WC_OK;
}

int wc_large_integrate(const wc_params* p, int precision, int B, int N, const double* sc, const double* G,
                       const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                       int64_t nsteps, double tau_ip, int64_t rec_every, int64_t rec_ld, void* recE, void* recI,
                       void* recA, void* workspace, hipStream_t st) {
    if (precision == WC_F64)
        return run_large<double>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every, rec_ld,
                                 recE, recI, recA, workspace, st);
    if (nsteps > 1 && persistent_ok(B, N)) {
        const int rc = run_persistent(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every, rec_ld,
                                      recE, recI, recA, workspace, st);
        if (rc != kPersistRetry) return rc;  // else: the grid could not be made co-resident
    }
    return run_large<float>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, rec_every, rec_ld, recE,
                            recI, recA, workspace, st);
}

#ifdef WCSDE_DIAG
// ablation variants of the fp32 step kernel (wc_diag_integrate variants 100..107; diag build only)
int wc_large_diag(int variant, const wc_params* p, int B, int N, const double* sc, const double* G,
                  const double* sigmaE, const uint64_t* keys, double* E, double* I, double* A, int64_t step0,
                  int64_t nsteps, double tau_ip, void* workspace, hipStream_t st) {
    switch (variant) {
        case 100: return run_large<float, 0>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, 0, 0,
                                             nullptr, nullptr, nullptr, workspace, st);
        case 101: return run_large<float, 1>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, 0, 0,
                                             nullptr, nullptr, nullptr, workspace, st);
        case 102: return run_large<float, 2>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, 0, 0,
                                             nullptr, nullptr, nullptr, workspace, st);
        case 103: return run_large<float, 3>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, 0, 0,
                                             nullptr, nullptr, nullptr, workspace, st);
        case 104: return run_large<float, 0, 3, true>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip,
                                                      0, 0, nullptr, nullptr, nullptr, workspace, st);
        case 105: return run_large<float, 0, 2, true>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip,
                                                      0, 0, nullptr, nullptr, nullptr, workspace, st);
        case 106: return run_large<float, 0, 3, false>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip,
                                                       0, 0, nullptr, nullptr, nullptr, workspace, st);
        case 107: return run_large<float, 4>(p, B, N, sc, G, sigmaE, keys, E, I, A, step0, nsteps, tau_ip, 0, 0,
                                             nullptr, nullptr, nullptr, workspace, st);
        default: return wc_set_err(WC_EINVAL, "unknown large-N diagnostic variant");
    }
}
#endif  // WCSDE_DIAG
