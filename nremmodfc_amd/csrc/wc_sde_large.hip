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
// folded in for the raw Box-Muller normal, a_ie read as its high word), with every fusion
// explicit (contraction off inside).  step_kernel and persist_kernel both call this, so the two
// N > 96 paths give the same bits whatever the surrounding code lets the compiler fuse.
struct CellConsts {
    float a_ee, Pm, rhoE, rE, rI, cIe, cIi, cI0, knoise, dtE, dtI, dtA;
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
    const float tA = in0 * k.dtA;
    A.add(__builtin_fmaf(e0, tA, -k.rhoE * tA));
}
#pragma clang fp contract(on)

__host__ __device__ inline CellConsts cell_consts(double a_ee, double a_ei, double a_ii, double P, double rhoE,
                                                  double rE, double rI, double mu, double sigmaI, double sqdtD,
                                                  double dtSim, double tauE, double tauI, double tau_ip) {
    const double l2e = 1.4426950408889634;
    return CellConsts{(float)a_ee, (float)(P - mu), (float)rhoE, (float)rE, (float)rI, (float)(-a_ei * sigmaI * l2e),
                      (float)(a_ii * sigmaI * l2e), (float)(mu * sigmaI * l2e), (float)(sqdtD * (double)kSqrt2Ln2),
                      (float)(dtSim / tauE), (float)(dtSim / tauI), (float)(dtSim / tau_ip)};
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
        auto issue = [&](int c, int st) {
#pragma unroll
            for (int i = 0; i < kU; ++i) {
                __builtin_amdgcn_global_load_lds(asrc[i] + (size_t)c * kParts * 64, (lds_vptr)(&lds[st][0][aoff[i]]), 16,
                                                 0, 0);
                __builtin_amdgcn_global_load_lds(bsrc[i] + (size_t)c * bstep, (lds_vptr)(&lds[st][1][boff[i]]), 16, 0, 0);
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
// Persistent fp32 integrator (round 2): the state stays in registers for the whole call.
//
// One workgroup (8 waves) owns a tile of 128 nodes x 80 simulations for ALL nsteps steps:
// wave w holds node tile w (16 nodes) of the five 16-simulation tiles, i.e. 20 (node, sim)
// cells per lane -- E, I, the a_ie pair, G and the slope in VGPRs.  Each step it streams the
// connectome rows of its 128 nodes (read-only: LDS-DMA, as in step_kernel) and the whole E
// image of its 80 simulations, which the 8 node-block workgroups of the simulation block
// publish every step (every node's E feeds every node's coupling).  The hand-off follows
// MI355X_MICROARCH.md's fence-free form (its "Valid forms" consumer conditions (1)-(4) with
// row 1 of the sc1 hand-off table, whose store and load cells admit 4-, 8- or 16-B accesses;
// DESIGN.md 3.1b quotes them): the E image is stored write-through (16-B sc1 buffer stores
// under WC_PIMG16, the default; 8-B otherwise) and every load of it is a 16-B sc1 buffer load to
// registers; every storing wave drains vmcnt before a workgroup barrier, after which ONE lane
// adds 1 to the simulation block's counter (a relaxed agent-scope atomic add -- no release
// fence: the sc1 stores have left the CU once vmcnt drained); the consumer's one lane polls that
// counter with relaxed agent-scope (sc1) loads, then a workgroup barrier releases the other
// waves (no acquire fence: every image load bypasses the L1).  Co-residency of the whole grid
// (one workgroup per CU) is guaranteed by the cooperative launch, which fails instead of
// running partly resident (the host then falls back to step_kernel).  Every wait is still
// bounded: a timeout sets the error word, the state is poisoned with NaN, and the host reads
// the word back and returns WC_EHIP.
// Double-buffered E image: a block writes E(s+1) into the buffer read at step s-1, which
// every block of its simulation block has finished reading (it passed that block's step-s
// wait).  The arithmetic per cell -- K order of the MFMA chain, the epilogue expressions,
// the noise -- is step_kernel's, so both paths give the same bits.
constexpr int kPN = 128, kPS = 80, kPT = kPS / 16;  // nodes, simulations, simulation tiles per workgroup
constexpr int kPWaves = kPN / 16;                     // 8
constexpr uint32_t kSpinLimit = 1u << 22;             // polls per wait before giving up (~seconds)
constexpr int kPersistRetry = 1;                      // run_persistent: cooperative launch refused
#ifndef WC_PPAIR
#define WC_PPAIR 1
#endif
#ifndef WC_PEARLY
#define WC_PEARLY 1  // the next pair's operand loads issued before the pair's barrier
#endif
// K chunks of the connectome tile kept in LDS (112 KB of the 512 KB streamed per step; 8 chunks
// = 128 KB before the image stages were paired, WC_PPAIR)
constexpr int kPRes = WC_PPAIR ? 7 : 8;

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

// E image unit (k-chunk c, simulation block sb, part p, simulation tile t): 64 lanes x 16 B,
// lane (g, j) holding the 8 fp16 values of nodes 16(2c + h) + 4g + r (jj = 4h + r) of
// simulation 80 sb + 16 t + j -- the MFMA B-operand fragment, so a chunk of a block is 10
// contiguous KB
__host__ __device__ __forceinline__ uint32_t pimg_unit(const PGeo& g, int c, int sb, int p, int t) {
    return (uint32_t)((((size_t)c * g.SBp + sb) * kParts + p) * kPT + t);
}
#ifndef WC_PIMG16
#define WC_PIMG16 1  // the E image in 16-B units of one node tile (hi | lo), one store per lane and tile
                     // (0: 8-B halves of two tiles per unit; 4.5% slower, profiles/r03_c5_pimg16.log)
#endif
// WC_PIMG16 layout: unit (k-chunk c, simulation block sb, simulation tile t, half h) of 64 lanes x
// 16 B, lane (g, j) holding [hi | lo] of nodes 16 (2c + h) + 4g + r, r < 4, of simulation 80 sb +
// 16 t + j: the publishing wave (node tile 2c + h) writes whole 16-B pieces, the chunk of a block
// is still 10 contiguous KB, and the staging splits each piece into the two parts' B fragments
__host__ __device__ __forceinline__ uint32_t pimg_unit16(const PGeo& g, int c, int sb, int t, int h) {
    return (uint32_t)((((size_t)c * g.SBp + sb) * kPT + t) * 2 + h);
}

// DIAG (timing ablations only, diag build, WCSDE_PERSISTENT=2..7; results are wrong): 1 = no MFMA, 2 = no
// epilogue arithmetic, 3 = no K-loop operand loads, 4 = no hand-off waits, 5 = no loads for the step's
// first pair, 6 = no E-image loads (A rows still streamed)
template <int DIAG = 0>
__global__ void __launch_bounds__(kPWaves * 64, 1) persist_kernel(const PArgs a) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    // [stage][part x sim tile][lane] B (2 stages); per-simulation G, slope and keys.  The state and
    // the A fragments live in registers (~215 VGPRs: one workgroup per CU).
    // image stages: WC_PPAIR stages the two chunks of a pair behind one barrier (16 per step, not 32)
    __shared__ f16x8 ldsB[2][WC_PPAIR ? 2 : 1][kParts * kPT][64];
    __shared__ f16x8 ldsA[kPRes][kPWaves][kParts][64];  // the first kPRes K chunks of the connectome rows, resident
    __shared__ float2 ldsGS[kPS];
    __shared__ uint64_t ldsK[kPS];
    __shared__ int go, uni;
    const PGeo& g = a.g;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, j = lane & 15, gq = lane >> 4;
    int sb, nb;
    pblock(g, sb, nb);
    const int mt = nb * kPWaves + w;  // this wave's node tile
    const int n0 = 16 * mt + 4 * gq;
    const float* scl = reinterpret_cast<const float*>(a.ws + g.o_scl);
    const float gscale = scl[1];
    unsigned* cnt = reinterpret_cast<unsigned*>(a.ws + g.o_cnt) + sb * 16;
    unsigned* err = reinterpret_cast<unsigned*>(a.ws + g.o_err);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(a.ws + g.o_x, 0,
                                                                         (int)(2 * (size_t)g.Np * g.Bp * 4), 0x00020000);
    const uint32_t img_units = (uint32_t)((size_t)g.Np * g.Bp * 4 / 1024);  // 1-KB units (64 lanes x 16 B) per image

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
    __syncthreads();
    float E[kPT][4], I[kPT][4];
    AccA<true> Av[kPT][4];
    bool my_uni = true;
#pragma unroll
    for (int t = 0; t < kPT; ++t) {
        const int b = sb * kPS + 16 * t + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = n0 + r;
            const bool ok = b < g.B && n < g.N;
            const size_t o = ok ? (size_t)b * g.N + n : 0;
            E[t][r] = ok ? (float)a.E[o] : 0.f;
            I[t][r] = ok ? (float)a.I[o] : 0.f;
            Av[t][r].set(ok ? a.A[o] : 0.0);
            if (ok && (a.G[o] != a.G[(size_t)b * g.N] || a.sigmaE[o] != a.sigmaE[(size_t)b * g.N])) my_uni = false;
        }
    }
    if (!my_uni) uni = 0;  // benign race: every writer stores 0
    // publish this wave's E tiles into image `buf` and signal the simulation block:
    // write-through (sc1) stores, a vmcnt drain in every storing wave, a workgroup barrier, one
    // lane's relaxed agent-scope counter add (the fence-free form above: no release fence)
    auto publish = [&](int buf) {
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            f16x4 ph[kParts];
            split2h(E[t], ph[0], ph[1]);
#if WC_PIMG16
            typedef unsigned u4s __attribute__((ext_vector_type(4)));
            const u2 h0 = __builtin_bit_cast(u2, ph[0]), h1 = __builtin_bit_cast(u2, ph[1]);
            const uint32_t unit = buf * img_units + pimg_unit16(g, mt >> 1, sb, t, mt & 1);
            __builtin_amdgcn_raw_buffer_store_b128(u4s{h0.x, h0.y, h1.x, h1.y}, xrs, (int)((unit * 64 + lane) * 16), 0, 16);
#else
#pragma unroll
            for (int p = 0; p < kParts; ++p) {
                const uint32_t unit = buf * img_units + pimg_unit(g, mt >> 1, sb, p, t);
                const int off = (int)((unit * 64 + lane) * 16 + (mt & 1) * 8);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, ph[p]), xrs, off, 0, 16);
            }
#endif
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // consumer: one lane polls the counter (relaxed agent-scope = sc1 loads), then a workgroup
    // barrier before any wave loads the image, every such load sc1 (no acquire fence; bounded:
    // error word + exit)
    auto wait_for = [&](unsigned target) -> bool {
        if (DIAG == 4) {
            __syncthreads();
            return true;
        }
        if (tid == 0) {
            int ok = 0;
            for (uint32_t it = 0; it < kSpinLimit; ++it) {
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
    bool alive = wait_for((unsigned)g.NBp);
    const bool uni_wg = uni != 0;  // (the barriers inside publish/wait_for ordered every store to it)
    const f16x8* F = reinterpret_cast<const f16x8*>(a.ws + g.o_frag);
    CellConsts kc = a.kc;
    // the folded constants stay in VGPRs (wave-uniform values; as SGPRs they were spilled to VGPR
    // lanes and re-read every step)
    asm volatile("" : "+v"(kc.a_ee), "+v"(kc.Pm), "+v"(kc.rhoE), "+v"(kc.rE), "+v"(kc.rI), "+v"(kc.cIe));
    asm volatile("" : "+v"(kc.cIi), "+v"(kc.cI0), "+v"(kc.knoise), "+v"(kc.dtE), "+v"(kc.dtI), "+v"(kc.dtA));
    const size_t BN = (size_t)g.B * g.N;
    int rec_cnt = 0, rec_row = 0;
    // K loop operands, two chunks ahead, through registers: A = this wave's own node tile (units
    // 2w, 2w+1 of the read-only connectome image) straight into MFMA fragments; B = the chunk's
    // 640 E-image units, thread tid loading unit-lane tid (and 512 + tid for tid < 128), written
    // to one of two LDS stages once they land
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const f16x8* asrc = F + (size_t)mt * g.NC * kParts * 64 + lane;
    f16x8 fa[2][kParts];
    u4 rb[2][2];
    const int res = g.NC < kPRes ? g.NC : kPRes;  // chunks c < res come from ldsA (NC is a multiple of 4)
    for (int c = 0; c < res; ++c) {
        ldsA[c][w][0][lane] = asrc[(size_t)c * kParts * 64];
        ldsA[c][w][1][lane] = asrc[(size_t)c * kParts * 64 + 64];
    }
    auto load_chunk = [&](int c, int slot, int buf) {
        if (DIAG == 3) return;
        if (c >= res) {
            const f16x8* ap = asrc + (size_t)c * kParts * 64;
            fa[slot][0] = ap[0];
            fa[slot][1] = ap[64];
        }
        if (DIAG == 6) return;  // (ablation: no E-image loads, the A rows still streamed)
        const int xo = (int)(((buf * img_units + pimg_unit(g, c, sb, 0, 0)) * 64 + tid) * 16);
        rb[slot][0] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo, 0, 16));
        if (tid < 128) rb[slot][1] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo + 512 * 16, 0, 16));
    };
    // chunk c's MFMAs from image stage `st` (each wave reads only its own ldsA slice, written by
    // itself before the step loop)
    auto mfma_chunk = [&](int c, f16x8 a0, f16x8 a1, const f16x8 (*stg)[64], f4 (&acc)[kPT]) {
#pragma unroll
        for (int t = 0; t < kPT; ++t) {
            const f16x8 fb0 = stg[t][lane], fb1 = stg[kPT + t][lane];
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
    // WC_PPAIR: chunks c, c + 1 (a pair) staged together into pair stage (c / 2) & 1 behind ONE
    // barrier; that stage was last read two pairs ago, before the previous pair's barrier.  The
    // pair's A operands are taken before the next pair's loads overwrite fa.
    // one staged 16-B unit-lane ul (0..639) of a chunk into ldsB stage `st` (stage row h)
    auto stage_put = [&](int st, int h, int ul, u4 v) {
#if WC_PIMG16
        // unit (t, hh) = ul / 64: hi -> part 0's fragment of tile t, lo -> part 1's, half hh of each
        const int u = ul >> 6, ln = ul & 63, t = u >> 1, hh = u & 1;
        unsigned* b0 = reinterpret_cast<unsigned*>(&ldsB[st][h][t][ln]) + 2 * hh;
        unsigned* b1 = reinterpret_cast<unsigned*>(&ldsB[st][h][kPT + t][ln]) + 2 * hh;
        *reinterpret_cast<u2*>(b0) = u2{v.x, v.y};
        *reinterpret_cast<u2*>(b1) = u2{v.z, v.w};
#else
        reinterpret_cast<u4*>(&ldsB[st][h][0][0])[ul] = v;
#endif
    };
    auto do_pair = [&](int c, int buf, f4 (&acc)[kPT]) {
        const int ps = (c >> 1) & 1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            stage_put(ps, h, tid, rb[h][0]);
            if (tid < 128) stage_put(ps, h, 512 + tid, rb[h][1]);
        }
#if WC_PEARLY
        // the next pair's loads issued before the barrier (the staged registers are free once
        // their ds_writes have issued; the A operands of this pair taken first: each wave reads
        // only its own ldsA slice)
        const f16x8 a00 = c < res ? ldsA[c][w][0][lane] : fa[0][0];
        const f16x8 a01 = c < res ? ldsA[c][w][1][lane] : fa[0][1];
        const f16x8 a10 = c + 1 < res ? ldsA[c + 1][w][0][lane] : fa[1][0];
        const f16x8 a11 = c + 1 < res ? ldsA[c + 1][w][1][lane] : fa[1][1];
        if (c + 2 < g.NC) {
            load_chunk(c + 2, 0, buf);
            load_chunk(c + 3, 1, buf);
        }
        __syncthreads();
#else
        __syncthreads();
        const f16x8 a00 = c < res ? ldsA[c][w][0][lane] : fa[0][0];
        const f16x8 a01 = c < res ? ldsA[c][w][1][lane] : fa[0][1];
        const f16x8 a10 = c + 1 < res ? ldsA[c + 1][w][0][lane] : fa[1][0];
        const f16x8 a11 = c + 1 < res ? ldsA[c + 1][w][1][lane] : fa[1][1];
        if (c + 2 < g.NC) {
            load_chunk(c + 2, 0, buf);
            load_chunk(c + 3, 1, buf);
        }
#endif
        mfma_chunk(c, a00, a01, ldsB[ps][0], acc);
        mfma_chunk(c + 1, a10, a11, ldsB[ps][1], acc);
    };
    auto do_chunk = [&](int c, int slot, int buf, f4 (&acc)[kPT]) {
        stage_put(slot, 0, tid, rb[slot][0]);
        if (tid < 128) stage_put(slot, 0, 512 + tid, rb[slot][1]);
        __syncthreads();  // stage `slot` was last read at chunk c - 2, before the previous barrier
        // (each wave reads only its own ldsA slice, written by itself before the step loop)
        const f16x8 a0 = c < res ? ldsA[c][w][0][lane] : fa[slot][0];
        const f16x8 a1 = c < res ? ldsA[c][w][1][lane] : fa[slot][1];
        if (c + 2 < g.NC) load_chunk(c + 2, slot, buf);
        mfma_chunk(c, a0, a1, ldsB[slot][0], acc);
    };
    for (int64_t s = 0; s < a.nsteps && alive; ++s) {
        const int buf = (int)(s & 1);
        const bool rec = a.rec_every > 0 && rec_cnt == 0;
        if (a.rec_every > 0) {
            if (rec_cnt == 0) rec_cnt = (int)a.rec_every;
            --rec_cnt;
        }
        f4 acc[kPT];
#pragma unroll
        for (int t = 0; t < kPT; ++t) acc[t] = f4{0, 0, 0, 0};
        if (DIAG != 5) {  // (ablation 5: the step's first pair from stale registers, no exposed round trip)
            load_chunk(0, 0, buf);
            load_chunk(1, 1, buf);
        }
        for (int c = 0; c < g.NC; c += 2) {  // NC is a multiple of 4 (nodes padded to 128)
            if (WC_PPAIR) {
                do_pair(c, buf, acc);
            } else {
                do_chunk(c, 0, buf, acc);
                do_chunk(c + 1, 1, buf, acc);
            }
        }
        // ---- epilogue: step_kernel's update on the D fragments (the state in registers) ----
        const uint64_t gstep = (uint64_t)(a.step0 + s);
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
                        static_cast<float*>(a.recE)[o] = E[t][r];
                        if (a.recI) static_cast<float*>(a.recI)[o] = I[t][r];
                        if (a.recA) static_cast<float*>(a.recA)[o] = (float)Av[t][r].get();
                    }
                }
            }
            if (DIAG == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r) E[t][r] += 1e-30f * acc[t][r];
                continue;
            }
            float z[4];
            quad_normals_raw(gstep, (uint32_t)(4 * mt + gq), ldsK[16 * t + j], z);
            float gv[4], sv[4];
            if (uni_wg) {
                const float2 gs = ldsGS[16 * t + j];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    gv[r] = gs.x;
                    sv[r] = gs.y;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = n0 + r;
                    const bool ok = live && n < Nn;
                    const size_t o = ok ? (size_t)b * Nn + n : 0;
                    gv[r] = ok ? (float)a.G[o] * gscale : 0.f;
                    sv[r] = ok ? Tr<float>::slope(a.sigmaE[o]) : 0.f;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                cell_update_f32(kc, E[t][r], I[t][r], Av[t][r], acc[t][r], gv[r], sv[r], z[r], n0 + r >= g.N);
        }
        if (rec) ++rec_row;
        if (s + 1 < a.nsteps) {
            publish(buf ^ 1);
            alive = wait_for((unsigned)g.NBp * (unsigned)(s + 2));
        }
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
                a.E[o] = poisoned ? __builtin_nan("") : (double)E[t][r];
                a.I[o] = poisoned ? __builtin_nan("") : (double)I[t][r];
                a.A[o] = poisoned ? __builtin_nan("") : Av[t][r].get();
            }
        }
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
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)persist_kernel<0>, kPWaves * 64, 0) != hipSuccess ||
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
    const dim3 grid((unsigned)(g.SBp * g.NBp)), blk(kPWaves * 64);
    const void* kern = (const void*)persist_kernel<0>;
#ifdef WCSDE_DIAG
    const char* env = getenv("WCSDE_PERSISTENT");
    switch (env ? env[0] : '1') {
        case '2': kern = (const void*)persist_kernel<1>; break;
        case '3': kern = (const void*)persist_kernel<2>; break;
        case '4': kern = (const void*)persist_kernel<3>; break;
        case '5': kern = (const void*)persist_kernel<4>; break;
        case '6': kern = (const void*)persist_kernel<5>; break;
        case '7': kern = (const void*)persist_kernel<6>; break;
        default: break;
    }
#endif
    // cooperative: the whole grid is co-resident (the inter-workgroup waits need it) or the launch
    // fails -- e.g. another process holds CUs -- and the caller runs step_kernel instead
    void* kargs[] = {&a};
    hipError_t e = hipLaunchCooperativeKernel(kern, grid, blk, kargs, 0, st);
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
