// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the CCJ kernels use:
// each kernel streams a 1 GiB buffer exactly once (2-, 4- or 16-byte loads per lane, coalesced) or
// writes it once with 2-byte stores.  rocprofv3 --pmc FETCH_SIZE (KB) over these dispatches, divided
// by 1 GiB, is the counter-to-bytes factor for that width (tools/gpu_profile.sh).
// k_window: the partial-line patterns of k_iloop / k_ppush (one 64-lane 2-byte load per wave, each
// wave on fresh lines 4 KiB apart): `lanes` x 2 bytes at a byte offset `mis` into a 128-byte line
// (aligned: 1 line; misaligned: 2 lines each partly used; 32 lanes: half a line).  FETCH_SIZE over
// the 262144 waves, against 128 bytes per distinct line touched, says whether a partly used line is
// fetched (and counted) whole or as 64-byte halves.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T *buf, size_t n, int *out) {
    int acc = 0;
    for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < n; x += (size_t)gridDim.x * blockDim.x) {
        const T v = buf[x];
        const int *p = (const int *)&v;
        acc ^= (sizeof(T) >= 4) ? p[0] : (int)*(const short *)&v;
    }
    if (acc == 0x12345678) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_write16(short *buf, size_t n) {
    for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < n; x += (size_t)gridDim.x * blockDim.x)
        buf[x] = (short)x;
}

__global__ __launch_bounds__(256) void k_window(const short *buf, int lanes, int mis, int *out) {
    const size_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    int acc = 0;
    if (lane < lanes) acc = buf[(w * 4096 + (size_t)mis) / 2 + lane];
    if (acc == 12345) out[0] = acc;  // a value a short can hold, so the load stays
}

int main() {
    const size_t bytes = 1ull << 30;
    char *buf;
    int *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const int blocks = 256 * 16;
    hipLaunchKernelGGL(k_read<short>, dim3(blocks), dim3(256), 0, 0, (const short *)buf, bytes / 2, out);
    hipLaunchKernelGGL(k_read<int>, dim3(blocks), dim3(256), 0, 0, (const int *)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read<int4>, dim3(blocks), dim3(256), 0, 0, (const int4 *)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_write16, dim3(blocks), dim3(256), 0, 0, (short *)buf, bytes / 2);
    // 262144 waves (1 GiB / 4 KiB), 65536 workgroups: aligned 128 B, misaligned by 64 / 2 / 126 bytes
    // (2 lines each), and 32 lanes (64 B) aligned
    const int cases[5][2] = {{64, 0}, {64, 64}, {64, 2}, {64, 126}, {32, 0}};
    for (auto &c : cases) {
        hipMemset(buf, 1, bytes);  // evict the previous kernel's lines from L2 / MALL
        hipLaunchKernelGGL(k_window, dim3(65536), dim3(256), 0, 0, (const short *)buf, c[0], c[1], out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("streamed %zu bytes per kernel\n", bytes);
    return 0;
}
