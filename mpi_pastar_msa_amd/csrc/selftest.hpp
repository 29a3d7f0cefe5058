// selftest.hpp -- device self-tests of the open list's reserve / store
// hand-over (kernels.hpp: queue_reserve, queue_store), run through
// pastar_gpu_selftest_queue.  They call the search's own functions on the
// search's own buffers; every wait in them is bounded, so each kernel ends
// whatever the outcome.
#pragma once

#include "lists.hpp"

namespace pastar {
namespace dev {

constexpr int kSelfN = 16;  // entries each block stores per bucket

__device__ __forceinline__ uint32_t selftest_tag(int block, int which, int lane)
{
    return (uint32_t)(block * 1000 + which * 100 + lane);
}

// Polls *flag until it is set, at most `limit` times.
__device__ __forceinline__ void selftest_wait(const SearchArgs &a, unsigned *flag, unsigned limit)
{
    for (unsigned poll = 0; poll < limit; poll++) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        __builtin_amdgcn_s_sleep(4);
    }
    atomicOr(&a.ctl->fault, (int)kSiteSelftest);
}

// Crossed reservations.  Two workgroups X (block 0) and Z (block 1) append
// kSelfN entries each to sub-queue 0 of buckets b1 and b2, both empty:
//   X reserves in b2, then (after Z has reserved in both) in b1;
//   Z reserves in b1, then in b2,
// so Z holds the first positions of b1 and X those of b2 (flags[] orders the
// reservations; its waits are bounded).  Then each block stores, first into
// the bucket where it came second: X into b1, Z into b2, and only then into
// the other.  Position 0 opens a sub-queue's first chunk, so each block's
// first stores need the chunk the other block opens.  With chunks opened at
// reservation time (queue_reserve) both ids are published before any store;
// were a chunk opened by the store of its first position, X's first stores
// would wait for Z's second and Z's first for X's second.
__global__ __launch_bounds__(64) void selftest_crossed_kernel(SearchArgs a, int b1, int b2, unsigned *flags,
                                                             unsigned handshake_limit)
{
    const int lane = lane_id();
    const bool X = blockIdx.x == 0;
    unsigned long long r1 = 0, r2 = 0;
    if (lane == 0) {
        if (X) {
            r2 = queue_reserve(a, b2, 0, kSelfN);
            __hip_atomic_store(&flags[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            selftest_wait(a, &flags[1], handshake_limit);
            r1 = queue_reserve(a, b1, 0, kSelfN);
        } else {
            selftest_wait(a, &flags[0], handshake_limit);
            r1 = queue_reserve(a, b1, 0, kSelfN);
            r2 = queue_reserve(a, b2, 0, kSelfN);
            __hip_atomic_store(&flags[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    r1 = bcast_lane(r1, 0);
    r2 = bcast_lane(r2, 0);
    for (int it = 0; it < 2; it++) {
        const bool into_b1 = X == (it == 0);
        if (lane < kSelfN) {
            const Entry e = {selftest_tag(blockIdx.x, into_b1 ? 1 : 2, lane), 0};
            queue_store(a, into_b1 ? b1 : b2, 0, (into_b1 ? r1 : r2) + lane, e, a.stats);
        }
    }
}

// What selftest_crossed_kernel must have left: in b1 Z's entries at positions
// 0..kSelfN-1 and X's behind them, in b2 the other way round.  out[0] counts
// wrong or missing entries, out[1] the entries checked.
__global__ __launch_bounds__(64) void selftest_crossed_check_kernel(SearchArgs a, int b1, int b2,
                                                                   unsigned long long *out)
{
    const int lane = lane_id();
    unsigned bad = 0, seen = 0;
    if (lane < 2 * kSelfN) {
        for (int which = 1; which <= 2; which++) {
            const int b = which == 1 ? b1 : b2;
            const int first_block = which == 1 ? 1 : 0;
            const int block = lane < kSelfN ? first_block : 1 - first_block;
            Entry e;
            if (!queue_entry(a, b, 0, (unsigned long long)lane, e) || e.slot != selftest_tag(block, which, lane % kSelfN))
                bad++;
            seen++;
        }
        if (a.q->W[b1][0] != 2 * kSelfN || a.q->W[b2][0] != 2 * kSelfN)
            bad++;
    }
    bad = wave_sum(bad);
    seen = wave_sum(seen);
    if (lane == 0) {
        out[0] = bad;
        out[1] = seen;
    }
}

// A store into a chunk nobody opened: the host has moved sub-queue (b, 0)'s
// cursor to `lost` (> 0, inside chunk 0) without opening the chunk, as if a
// reserver had vanished between its cursor add and its publication.  The
// stores wait Ctl::spin_limit polls (set low by the host), flag the fault word
// and drop their entries; the kernel ends.
__global__ __launch_bounds__(64) void selftest_lost_opener_kernel(SearchArgs a, int b)
{
    const int lane = lane_id();
    unsigned long long r = 0;
    if (lane == 0)
        r = queue_reserve(a, b, 0, kSelfN);
    r = bcast_lane(r, 0);
    if (lane < kSelfN)
        queue_store(a, b, 0, r + lane, Entry{selftest_tag(0, 3, lane), 0}, a.stats);
}

}  // namespace dev
}  // namespace pastar
