// Where does global_load_lds_ushort put each lane's 2 bytes in LDS?  Fills LDS with a marker,
// loads 64 consecutive int16 (values 1000+lane) with one LDS-DMA instruction at LDS offset 0 and
// dumps the first 256 bytes of LDS as int16.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const short *src, short *out) {
    __shared__ short buf[256];
    const int lane = threadIdx.x;
    for (int x = lane; x < 256; x += 64) buf[x] = -1;
    __syncthreads();
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + lane),
                                     (__attribute__((address_space(3))) void *)&buf[0], 2, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int x = lane; x < 256; x += 64) out[x] = buf[x];
}
int main() {
    short h[64], o[256], *ds, *dout;
    for (int i = 0; i < 64; ++i) h[i] = (short)(1000 + i);
    hipMalloc(&ds, 128); hipMalloc(&dout, 512);
    hipMemcpy(ds, h, 128, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout);
    hipMemcpy(o, dout, 512, hipMemcpyDeviceToHost);
    for (int i = 0; i < 256; ++i) printf("%d%c", o[i], i % 16 == 15 ? '\n' : ' ');
    return 0;
}
