// Dependent-chain latency of the memory operations the search kernel uses,
// on one wave of one block (the regime of a narrow-frontier search level).
// hipcc --offload-arch=gfx950 -O3 tools/micro/latency.hip -o tools/micro/latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memrealtime(); }

enum { kPlain, kCas64, kAdd64, kCasWg64, kSc1Load, kLds, kCas32, kMin64, kExch64, kMinWg64, kAddWg64, kModes };
static const char *kNames[] = {"plain load", "agent CAS64", "agent add64", "wg CAS64", "sc1 load", "LDS load",
                               "agent CAS32", "agent min64", "agent exch64", "wg min64", "wg add64"};

__global__ void chain(unsigned long long *buf, unsigned long long n, int mode, int iters, unsigned long long *out,
                      int lanes)
{
    __shared__ unsigned long long lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x)
        lds[i] = (i * 1031 + 7) & 4095;
    __syncthreads();
    const unsigned long long mask = n - 1;  // n is a power of two
    const unsigned long long salt = (threadIdx.x + 64ull * blockIdx.x) * 0xD1B54A32D192ED03ull + 1;
    unsigned long long idx = (salt >> 17) & mask;
    unsigned long long t0 = clk();
    for (int k = 0; k < iters && (int)threadIdx.x < lanes; k++) {
        unsigned long long v = 0;
        unsigned long long *p = &buf[idx];
        switch (mode) {
        case kPlain: v = *p; break;
        case kCas64: v = atomicCAS(p, 0xdeadull, 0xbeefull); break;
        case kAdd64: v = atomicAdd(p, 2ull); break;
        case kCasWg64: {
            unsigned long long e = 0xdeadull;
            __hip_atomic_compare_exchange_strong(p, &e, 0xbeefull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            v = e;
            break;
        }
        case kSc1Load: v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break;
        case kLds: v = lds[idx & 4095]; break;
        case kCas32: v = atomicCAS(reinterpret_cast<unsigned *>(p), 0xdeadu, 0xbeefu); break;
        case kMin64: v = atomicMin(p, ~1ull); break;
        case kExch64: v = atomicExch(p, idx * 2654435761ull); break;
        case kMinWg64: v = __hip_atomic_fetch_min(p, ~1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); break;
        case kAddWg64: v = __hip_atomic_fetch_add(p, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); break;
        }
        // next address depends on the value; the per-lane salt keeps lanes
        // that meet at one address from following each other afterwards
        unsigned long long x = (v ^ salt) + k;
        x ^= x >> 31;
        x *= 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        idx = x & mask;
    }
    unsigned long long t1 = clk();
    if (threadIdx.x == 0)
        out[blockIdx.x] = t1 - t0;
    if (idx == n)  // never (idx <= mask): keeps the chain live
        out[1000] = idx;
}

int main()
{
    const unsigned long long n = 1ull << 22;  // 32 MB of 8-B words
    unsigned long long *buf, *out;
    if (hipMalloc(&buf, n * 8) != hipSuccess || hipMalloc(&out, 1024 * 8) != hipSuccess)
        return 1;
    std::vector<unsigned long long> h(n);
    for (unsigned long long i = 0; i < n; i++)
        h[i] = i * 2654435761ull;
    if (hipMemcpy(buf, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess)
        return 1;
    for (unsigned long long set : {n, 1ull << 15}) {
        for (int cfg = 0; cfg < 3; cfg++) {
            const int blocks = cfg == 2 ? 64 : 1, lanes = cfg == 0 ? 1 : 64;
            for (int mode = 0; mode < kModes; mode++) {
                const int iters = 1000;
                hipLaunchKernelGGL(chain, dim3(blocks), dim3(64), 0, 0, buf, set, mode, 50, out, lanes);  // warm
                hipLaunchKernelGGL(chain, dim3(blocks), dim3(64), 0, 0, buf, set, mode, iters, out, lanes);
                unsigned long long r[64];
                if (hipMemcpy(r, out, 8 * blocks, hipMemcpyDeviceToHost) != hipSuccess)
                    return 1;
                double avg = 0;
                for (int b = 0; b < blocks; b++)
                    avg += r[b];
                avg /= blocks;
                std::printf("set %8llu KB blocks %2d lanes %2d %-14s %7.1f ns per dependent op\n", set * 8 / 1024,
                            blocks, lanes, kNames[mode], avg * 10.0 / iters);
            }
        }
    }
    return 0;
}
