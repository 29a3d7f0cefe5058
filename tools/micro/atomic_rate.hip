// Chip-wide rate of random 8-B operations on a large device array (the node
// table's access pattern): plain loads, non-returning and returning
// agent-scope atomicMin, and returning CAS, each lane walking its own random
// sequence with `inflight` independent operations per iteration.  Prints
// operations per second and the equivalent 64-B-line rate, to place the
// expand kernel's per-launch relax count against a measured ceiling.
//   hipcc --offload-arch=gfx950 -O3 atomic_rate.hip -o atomic_rate_bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ unsigned long long next(unsigned long long x)
{
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
}

template <int OP, int K>
__global__ __launch_bounds__(256) void rate(unsigned long long *tab, unsigned long long mask, int iters,
                                            unsigned long long *sink)
{
    unsigned long long s[K];
#pragma unroll
    for (int k = 0; k < K; k++)
        s[k] = 0x9E3779B97F4A7C15ull * (blockIdx.x * 256ull + threadIdx.x + 1) + k * 0x632BE59BD9B4E019ull;
    unsigned long long acc = 0;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            s[k] = next(s[k]);
            unsigned long long *p = tab + (s[k] & mask);
            if (OP == 0) {
                acc += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (OP == 1) {
                __hip_atomic_fetch_min(p, s[k] >> 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (OP == 2) {
                acc += __hip_atomic_fetch_min(p, s[k] >> 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                unsigned long long e = 0;
                __hip_atomic_compare_exchange_strong(p, &e, s[k] | 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                acc += e;
            }
        }
    }
    if (acc == 42)
        sink[0] = acc;
}

template <int OP, int K>
void run(const char *name, unsigned long long *tab, unsigned long long mask, unsigned long long *sink, int blocks)
{
    const int iters = 64;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    rate<OP, K><<<blocks, 256>>>(tab, mask, iters, sink);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    rate<OP, K><<<blocks, 256>>>(tab, mask, iters, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double ops = (double)blocks * 256 * iters * K;
    std::printf("%-26s inflight %d blocks %5d: %7.2f G ops/s (%6.1f GB/s of 64-B lines) in %.3f ms\n", name, K, blocks,
                ops / ms * 1e-6, ops * 64 / ms * 1e-6, ms);
}

int main()
{
    const unsigned long long words = 1ull << 28;  // 2 GB, beyond the MALL
    unsigned long long *tab = nullptr, *sink = nullptr;
    CHECK(hipMalloc(&tab, words * 8));
    CHECK(hipMalloc(&sink, 8));
    CHECK(hipMemset(tab, 0xff, words * 8));
    for (int blocks : {1024, 4096}) {
        run<0, 1>("load", tab, words - 1, sink, blocks);
        run<0, 4>("load", tab, words - 1, sink, blocks);
        run<1, 1>("atomicMin (no return)", tab, words - 1, sink, blocks);
        run<1, 4>("atomicMin (no return)", tab, words - 1, sink, blocks);
        run<2, 1>("atomicMin (returning)", tab, words - 1, sink, blocks);
        run<2, 4>("atomicMin (returning)", tab, words - 1, sink, blocks);
        run<3, 1>("CAS (returning)", tab, words - 1, sink, blocks);
        run<3, 4>("CAS (returning)", tab, words - 1, sink, blocks);
    }
    // a table of kinase's learned size (2^25 slots x 32 B = 1 GB; one word per slot here)
    for (int blocks : {1024, 4096}) {
        run<2, 4>("atomicMin ret, 32M words", tab, (1ull << 25) - 1, sink, blocks);
        run<0, 4>("load, 32M words", tab, (1ull << 25) - 1, sink, blocks);
    }
    return 0;
}
