// Dependent random-load latency against the working-set size (32 MB .. 4 GB):
// the node table of a large search is far beyond the 32 MB of latency.hip,
// so its probes may pay address-translation misses on top of HBM latency.
// hipcc --offload-arch=gfx950 -O3 tools/micro/tlb.hip -o tools/micro/tlb
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(const unsigned long long *buf, unsigned long long mask, int iters, unsigned long long *out,
                      int lanes)
{
    const unsigned long long salt = (threadIdx.x + 1) * 0xD1B54A32D192ED03ull;
    unsigned long long idx = (salt >> 17) & mask;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < iters && (int)threadIdx.x < lanes; k++) {
        unsigned long long x = (buf[idx * 16] ^ salt) + k;  // one 128-B line per element
        x ^= x >> 31;
        x *= 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        idx = x & mask;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0)
        out[0] = t1 - t0;
    if (idx == ~0ull)
        out[1] = idx;
}

int main()
{
    const unsigned long long max_bytes = 4ull << 30;
    unsigned long long *buf, *out;
    if (hipMalloc(&buf, max_bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess)
        return 1;
    if (hipMemset(buf, 0, max_bytes) != hipSuccess)
        return 1;
    for (unsigned long long mb : {32ull, 256ull, 1024ull, 4096ull}) {
        const unsigned long long lines = (mb << 20) / 128;
        for (int lanes : {1, 16, 64}) {
            const int iters = 2000;
            hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, buf, lines - 1, 100, out, lanes);
            hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, buf, lines - 1, iters, out, lanes);
            unsigned long long r = 0;
            if (hipMemcpy(&r, out, 8, hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            std::printf("set %5llu MB lanes %2d  %7.1f ns per dependent load\n", mb, lanes, r * 10.0 / iters);
        }
    }
    return 0;
}
