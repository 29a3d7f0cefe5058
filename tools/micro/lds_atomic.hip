// Dependent-chain cost of LDS operations on one wave, by active lanes and
// address pattern: read, write+read, CAS32 (returning), min64 (returning),
// min64 (no return) + read.  Used to shape the LDS-resident search's relax.
#include <hip/hip_runtime.h>
#include <cstdio>

#define LDSP __attribute__((address_space(3)))

template <int OP>
__global__ void probe(unsigned long long *out, int iters, int active, int spread)
{
    __shared__ unsigned int tab[8192];
    __shared__ unsigned long long tab64[4096];
    const int lane = threadIdx.x;
    for (int k = lane; k < 8192; k += 64)
        tab[k] = 0;
    for (int k = lane; k < 4096; k += 64)
        tab64[k] = ~0ull;
    __syncthreads();
    LDSP unsigned int *t = (LDSP unsigned int *)tab;
    LDSP unsigned long long *t64 = (LDSP unsigned long long *)tab64;
    unsigned int idx = (lane * 2654435761u) % 4093u;  // scattered slots
    if (!spread)
        idx = lane;  // consecutive slots
    unsigned int acc = 0;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (lane < active) {
        for (int i = 0; i < iters; i++) {
            unsigned int v;
            if (OP == 0) {
                v = t[idx];
            } else if (OP == 1) {
                unsigned int e = 0;
                __hip_atomic_compare_exchange_strong(&t[idx], &e, (unsigned)(i + 1), __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                v = e;
            } else if (OP == 2) {
                v = (unsigned int)__hip_atomic_fetch_min(&t64[idx], (unsigned long long)(1000000 - i),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (OP == 3) {
                __hip_atomic_fetch_min(&t64[idx], (unsigned long long)(1000000 - i), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                v = (unsigned int)t64[idx];
            } else {
                t[idx] = i;
                v = t[idx];
            }
            acc += v;
            idx = (idx + (v & 1)) & 4095u;  // dependent address
        }
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
        out[0] = r1 - r0;
    if (acc == 0xdeadbeef)
        out[1] = acc;
}

int main()
{
    unsigned long long *d, h;
    hipMalloc(&d, 16);
    const char *names[] = {"read", "CAS32 rtn", "min64 rtn", "min64 + read", "write + read"};
    const int iters = 2000;
    for (int op = 0; op < 5; op++)
        for (int spread = 0; spread < 2; spread++)
            for (int active : {1, 8, 32, 64}) {
                switch (op) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, d, iters, active, spread); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, iters, active, spread); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, iters, active, spread); break;
                case 3: hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, d, iters, active, spread); break;
                default: hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, d, iters, active, spread); break;
                }
                (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
                std::printf("%-14s %s lanes %2d: %6.1f ns per dependent step\n", names[op],
                            spread ? "scattered  " : "consecutive", active, h * 10.0 / iters);
            }
    return 0;
}
