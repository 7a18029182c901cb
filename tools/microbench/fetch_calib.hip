// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the CCJ kernels use:
// each kernel streams a 1 GiB buffer exactly once (2-, 4- or 16-byte loads per lane, coalesced) or
// writes it once with 2-byte stores.  rocprofv3 --pmc FETCH_SIZE (KB) over these dispatches, divided
// by 1 GiB, is the counter-to-bytes factor for that width (tools/gpu_profile.sh).
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
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("streamed %zu bytes per kernel\n", bytes);
    return 0;
}
