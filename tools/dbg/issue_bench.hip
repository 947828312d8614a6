// Issue-cost microbenchmark (tools only): cycles per instruction for independent streams of
// v_mad_u64_u32, v_bitop3_b32, v_pk_fma_f32, v_fma_f32, v_exp_f32, at W waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define REP 256
template <int OP>
__global__ void __launch_bounds__(1024) kern(uint32_t* out, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 * 3 + 1, a2 = a0 * 5 + 2, a3 = a0 * 7 + 3, a4 = a0 ^ 0x55, a5 = a0 + 99, a6 = a0 * 11, a7 = a0 * 13;
    float f0 = a0 * 1e-3f, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v p0 = {f0, f1}, p1 = {f2, f3}, p2 = {f4, f5}, p3 = {f6, f7}, p4 = p0 + 1.f, p5 = p1 + 1.f, p6 = p2 + 1.f, p7 = p3 + 1.f;
    const uint32_t m = 0xD2511F53u;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < REP / 8; ++r) {
            if constexpr (OP == 0) {  // v_mad_u64_u32, 8 independent chains
                uint64_t q;
#define MAD(a) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(q) : "v"(a), "s"(m) : "vcc"); a = (uint32_t)(q >> 32) ^ (uint32_t)q;
                MAD(a0) MAD(a1) MAD(a2) MAD(a3) MAD(a4) MAD(a5) MAD(a6) MAD(a7)
            } else if constexpr (OP == 1) {  // v_bitop3
#define B3(a, b, c) a = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
                B3(a0, a1, a2) B3(a1, a2, a3) B3(a2, a3, a4) B3(a3, a4, a5) B3(a4, a5, a6) B3(a5, a6, a7) B3(a6, a7, a0) B3(a7, a0, a1)
            } else if constexpr (OP == 2) {  // v_pk_fma_f32
#define PF(a, b) a = __builtin_elementwise_fma(a, b, p7);
                PF(p0, p1) PF(p1, p2) PF(p2, p3) PF(p3, p4) PF(p4, p5) PF(p5, p6) PF(p6, p0) PF(p7, p1)
            } else if constexpr (OP == 3) {  // v_fma_f32
#define FF(a, b) a = __builtin_fmaf(a, b, f7);
                FF(f0, f1) FF(f1, f2) FF(f2, f3) FF(f3, f4) FF(f4, f5) FF(f5, f6) FF(f6, f0) FF(f7, f1)
            } else if constexpr (OP == 4) {  // v_exp_f32
#define EX(a) a = __builtin_amdgcn_exp2f(a);
                EX(f0) EX(f1) EX(f2) EX(f3) EX(f4) EX(f5) EX(f6) EX(f7)
            } else if constexpr (OP == 5) {  // v_mad_u64_u32 with a dedicated SGPR pair for the carry
                uint64_t q, cy;
#define MADS(a) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(q), "=s"(cy) : "v"(a), "s"(m)); a = (uint32_t)(q >> 32) ^ (uint32_t)q;
                MADS(a0) MADS(a1) MADS(a2) MADS(a3) MADS(a4) MADS(a5) MADS(a6) MADS(a7)
            } else if constexpr (OP == 6) {  // v_mul_hi_u32 + v_mul_lo_u32
#define MHL(a) { uint32_t h = __umulhi(a, m), l = a * m; a = h ^ l; }
                MHL(a0) MHL(a1) MHL(a2) MHL(a3) MHL(a4) MHL(a5) MHL(a6) MHL(a7)
            }
        }
    }
    long long t1 = clock64();
    uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7 + p0.x + p1.x + p2.y + p3.y + p4.x + p5.y + p6.x + p7.y);
    if (s == 0x12345678u) out[1 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (uint32_t)(t1 - t0);
}
int main() {
    uint32_t* d;
    hipMalloc(&d, 8192 * 4);
    const char* names[] = {"v_mad_u64_u32(vcc)", "v_bitop3_b32", "v_pk_fma_f32", "v_fma_f32", "v_exp_f32", "v_mad_u64_u32(sgpr)", "mul_hi+mul_lo"};
    for (int waves = 1; waves <= 16; waves *= 2) {
        for (int op = 0; op < 7; ++op) {
            auto k = op == 0 ? kern<0> : op == 1 ? kern<1> : op == 2 ? kern<2> : op == 3 ? kern<3> : op == 4 ? kern<4> : op == 5 ? kern<5> : kern<6>;
            int iters = 200;
            // waves per SIMD: blocks of min(1024, 256 waves) threads, 256 * waves / 4 waves per CU
            const int tpb = waves <= 4 ? 256 * waves : 1024, nb = 256 * (waves <= 4 ? 1 : waves / 4);
            hipLaunchKernelGGL(k, dim3(nb), dim3(tpb), 0, 0, d, 10);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k, dim3(nb), dim3(tpb), 0, 0, d, iters);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            uint32_t c;
            hipMemcpy(&c, d, 4, hipMemcpyDeviceToHost);
            // clock64 = shader clock cycles of wave 0; instructions issued per SIMD = waves * iters * REP
            // SIMD throughput from the kernel time: instructions per SIMD = waves * iters * REP, at 2.4 GHz
            printf("waves/SIMD=%2d %-22s wave0 %.2f cyc/instr; kernel %.3f ms -> %.2f cyc per instr per SIMD at 2.4 GHz\n",
                   waves, names[op], (double)c / (iters * REP), ms, ms * 1e-3 * 2.4e9 / (waves * (double)iters * REP));
        }
    }
    return 0;
}
