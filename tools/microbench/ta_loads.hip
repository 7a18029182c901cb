// Vector-memory issue cost on gfx950 for loads of 2/4/8/16 bytes per lane (cache-resident data).
// Each wave issues ITER loads of one width over a small (L1/L2-resident) window; the kernel time
// divided by the number of wave-loads per CU gives the cycles per load instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int W>
struct Vec;
template <> struct Vec<2> { using T = short; };
template <> struct Vec<4> { using T = int; };
template <> struct Vec<8> { using T = int2; };
template <> struct Vec<16> { using T = int4; };

__device__ __forceinline__ int fold(short v) { return v; }
__device__ __forceinline__ int fold(int v) { return v; }
__device__ __forceinline__ int fold(int2 v) { return v.x ^ v.y; }
__device__ __forceinline__ int fold(int4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int W>
__global__ __launch_bounds__(256) void k_load(const char *buf, int iters, int misalign, int stride_lanes, int *out) {
    using T = typename Vec<W>::T;
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    // each wave walks its own 16 KB window (L1-resident after the first pass)
    const char *base = buf + (size_t)(wave & 255) * 16384 + misalign;  // misalign: byte shift of every load
    int acc = 0;
#pragma unroll 8
    for (int it = 0; it < iters; ++it) {
        const int off = ((it * 64 * stride_lanes) & 8191) + lane * W * stride_lanes;
        acc += fold(*(const T *)(base + (off & ~(W - 1))));
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
    char *buf;
    int *out;
    hipMalloc(&buf, 256 * 16384 + 4096);
    hipMemset(buf, 1, 256 * 16384 + 4096);
    hipMalloc(&out, 4);
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const int iters = 4096, blocks = ncu * 8;  // 32 waves per CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto kern, int mis, int stride) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, iters, mis, stride, out);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, iters, mis, stride, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double loads_per_cu = 5.0 * blocks * 4.0 * iters / ncu;
        printf("%-22s misalign %2d stride %d : %.2f cycles/load/CU (clock %d MHz)\n", name, mis, stride,
               ms * 1e-3 * clk * 1e3 / loads_per_cu, clk / 1000);
    };
    for (int stride : {1, 2}) {
        run("2B short", k_load<2>, 0, stride);
        run("2B short", k_load<2>, 64, stride);
        run("2B short", k_load<2>, 2, stride);
        run("4B int", k_load<4>, 0, stride);
        run("4B int", k_load<4>, 64, stride);
        run("4B int", k_load<4>, 2, stride);
        run("8B int2", k_load<8>, 0, stride);
        run("16B int4", k_load<16>, 0, stride);
    }
    return 0;
}
