// Vector-memory cost of the level kernel's 2-byte access patterns on gfx950: one wave-wide int16
// load per step over (a) 64 consecutive elements 128-byte aligned, (b) the same at an odd element
// offset, (c) two contiguous segments (row break at lane 40) at unrelated addresses, each either
// cache-resident (4 MB window) or streamed from HBM (1 GB window).  Cycles per load per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_pat(const short *buf, size_t window, int iters, int mode, int *out) {
    const int lane = threadIdx.x & 63;
    const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int acc = 0;
    unsigned long long x = wave * 0x9E3779B97F4A7C15ull;
#pragma unroll 4
    for (int it = 0; it < iters; ++it) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        const size_t base = (size_t)(x >> 20) & (window - 1);  // window: power of two (elements)
        size_t e;
        if (mode == 0) e = (base & ~(size_t)63) + lane;                // aligned 128 B
        else if (mode == 1) e = base + lane;                          // any offset
        else e = lane < 40 ? base + lane : ((base * 7919) & (window - 1)) + lane;  // two segments
        acc += buf[e];
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
    const size_t big = (size_t)1 << 30;
    short *buf;
    int *out;
    if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, big);
    int ncu = 256, clk = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const int iters = 2048, blocks = ncu * 6;  // 24 waves per CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[3] = {"aligned 64 x int16", "unaligned 64 x int16", "two segments"};
    for (size_t window : {(size_t)2 << 20, big / 4}) {  // elements; buffer has slack past the window
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(k_pat, dim3(blocks), dim3(256), 0, 0, buf, window, iters, mode, out);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_pat, dim3(blocks), dim3(256), 0, 0, buf, window, iters, mode, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double loads_per_cu = (double)blocks * 4 * iters / ncu;
            printf("%-22s window %6zu MB: %.2f cycles/load/CU\n", names[mode], (window * 2) >> 20,
                   ms * 1e-3 * clk * 1e3 / loads_per_cu);
        }
    }
    return 0;
}
