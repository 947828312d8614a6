// Read-rate probe for the Welch ring access pattern (tools/dbg, not product code): every wave
// reads one column's 4000-sample segment (16 KB contiguous, columns 24000 B apart, the node-major
// 6000-sample ring) with 8-B loads (the current welch_wave_kernel fetch, 512 B per wave
// instruction) or 16-B loads (1 KB per instruction), 8 waves per CU (one 512-thread workgroup,
// 128 KB of LDS reserved as the Welch kernel's), a column per wave at a time, the next column's
// loads issued before the current one is summed (the kernel's prefetch).  Prints GB/s.
//   hipcc --offload-arch=gfx950 -O3 tools/dbg/ring_read_bench.hip -o /tmp/rrb && /tmp/rrb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kLd = 6000, kSeg = 4000;

template <int W>  // bytes per lane per load: 8 or 16
__global__ void __launch_bounds__(512, 1) ring_read(const float* __restrict__ ring, long ncol, float* out, int seg0) {
    __shared__ float pad[32 * 1024];  // 128 KB: one workgroup per CU, as the Welch kernel
    typedef float vec __attribute__((ext_vector_type(W / 4)));
    constexpr int kPer = kSeg * 4 / (64 * W);  // loads per lane per column
    const int lane = threadIdx.x & 63;
    const long wv = (long)blockIdx.x * 8 + (threadIdx.x >> 6), nw = (long)gridDim.x * 8;
    float acc = 0.f;
    vec x[kPer];
    long c = wv;
    if (c < ncol) {
        const vec* col = reinterpret_cast<const vec*>(ring + c * kLd + seg0);
#pragma unroll
        for (int k = 0; k < kPer; ++k) x[k] = col[k * 64 + lane];
    }
    for (; c < ncol; c += nw) {
        vec y[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) y[k] = x[k];
        const long cn = c + nw < ncol ? c + nw : c;
        const vec* col = reinterpret_cast<const vec*>(ring + cn * kLd + seg0);
#pragma unroll
        for (int k = 0; k < kPer; ++k) x[k] = col[k * 64 + lane];
#pragma unroll
        for (int k = 0; k < kPer; ++k)
#pragma unroll
            for (int e = 0; e < W / 4; ++e) acc += y[k][e];
    }
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (acc == 1234.5f) out[0] = pad[(threadIdx.x + 1) & 511];
}

int main() {
    const long ncol = 1800000;
    float* ring;
    float* out;
    if (hipMalloc(&ring, (size_t)ncol * kLd * 4) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipEvent_t e0, e1;
    int cus = 0;
    if (hipMemset(ring, 0, (size_t)ncol * kLd * 4) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) {
        printf("setup failed\n");
        return 1;
    }
    for (int rep = 0; rep < 3; ++rep) {
        for (int w = 0; w < 2; ++w) {
            for (int grid_mul : {1, 4}) {
                const int grid = cus * grid_mul;
                (void)hipEventRecord(e0);
                if (w == 0)
                    hipLaunchKernelGGL(ring_read<8>, dim3(grid), dim3(512), 0, 0, ring, ncol, out, 2000);
                else
                    hipLaunchKernelGGL(ring_read<16>, dim3(grid), dim3(512), 0, 0, ring, ncol, out, 2000);
                float ms = 0;
                if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                    hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
                    printf("launch failed\n");
                    return 1;
                }
                printf("rep %d, %2d-B loads, grid %d: %.3f ms, %.0f GB/s\n", rep, w ? 16 : 8, grid, ms,
                       ncol * kSeg * 4.0 / ms / 1e6);
            }
        }
    }
    return 0;
}
