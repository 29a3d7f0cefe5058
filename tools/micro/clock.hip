// Shader clock under a one-wave load: s_memtime (core clock counter) against
// s_memrealtime (100 MHz) around a dependent VALU chain; and the same chain's
// cost in core cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(unsigned long long *out, int iters, int busy_blocks)
{
    if (blockIdx.x > 0) {  // optional extra load on other CUs
        int v = threadIdx.x;
        for (int i = 0; i < iters; i++)
            v = v * 1664525 + 1013904223;
        if (v == 12345)
            out[8] = v;
        return;
    }
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    int v = threadIdx.x;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            v = v * 1664525 + 1013904223;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = (unsigned long long)v;
    }
}

int main()
{
    unsigned long long *d, h[9];
    hipMalloc(&d, 9 * 8);
    for (int busy : {1, 256, 1024}) {
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(spin, dim3(busy), dim3(64), 0, 0, d, 20000, busy);
            hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
            const double secs = h[1] / 100e6;
            std::printf("blocks %4d: %llu core clocks in %.1f us -> %.0f MHz; %.2f clocks per dependent mad\n", busy,
                        h[0], secs * 1e6, h[0] / secs / 1e6, (double)h[0] / (20000.0 * 16 * 2));
        }
    }
    return 0;
}
