// lists.hpp -- the OpenList / ClosedList of the reference (PriorityList.h:
// 52-122, PAStar.cpp:92, 219-250) as host-driven operations on the device
// node table and f-bucket queues the batched search uses (kernels.hpp), so a
// host loop shaped like worker_inner (PAStar.cpp:320-401) can drive them one
// call at a time (include/pastar_gpu.h "OpenList / ClosedList").
//
// One table slot holds a node of both lists (Open U Closed): best = g << 32 |
// parent mask, aux = closed g | h << 32.  A node is
//   open    iff best.g < closed g   (it has a live queue entry: f = best.g + h;
//                                    closed g is INT_MAX: an enqueue that
//                                    improves a closed node resets it)
//   closed  iff closed g <= best.g  (closed g != INT_MAX)
//   absent  iff its slot is unclaimed or best == ~0 (erased)
#pragma once

#include "kernels.hpp"

namespace pastar {
namespace dev {

constexpr int kListThreads = 256;

template <int KW>
__device__ __forceinline__ void pack_key_dev(const DevProblem &P, const uint16_t *pos, uint64_t (&key)[KW])
{
#pragma unroll
    for (int w = 0; w < KW; w++)
        key[w] = w < P.kw ? kMark : 0;
    for (int i = 0; i < P.n; i++) {
        const uint64_t v = (uint64_t)pos[i] << P.kshift[i];
#pragma unroll
        for (int w = 0; w < KW; w++)
            if (w == P.kword[i])
                key[w] += v;
    }
}

template <int KW>
__device__ __forceinline__ void unpack_key_dev(const DevProblem &P, const uint64_t *key, uint16_t *pos)
{
    for (int i = 0; i < P.n; i++) {
        uint64_t word = key[0];
#pragma unroll
        for (int w = 1; w < KW; w++)
            if (w == P.kword[i])
                word = key[w];
        pos[i] = (uint16_t)((word >> P.kshift[i]) & ((1ull << P.kbits[i]) - 1ull));
    }
    for (int i = P.n; i < PASTAR_MAX_SEQ; i++)
        pos[i] = 0;
}

// PAStar::enqueue (PAStar.cpp:219-237) for a host batch: each node is relaxed
// into the table (a ClosedList node with g <= the new g, or an OpenList node
// with f <= the new f, keeps its record: the relax improves only on a
// strictly smaller g, h being a function of the coordinate), and an improved
// one gets a queue entry (conditional_enqueue, PriorityList.h:104-113).
// added[i] = 1 when node i entered the OpenList; out[0] counts reopenings
// (a closed node improved), out[1] table probe-limit failures.
template <int KW>
__global__ __launch_bounds__(kListThreads) void lists_enqueue_kernel(SearchArgs a, const pastar_node *__restrict__ in,
                                                                    int count, int32_t *__restrict__ added,
                                                                    unsigned long long *__restrict__ out)
{
    const DevProblem &P = *a.P;
    constexpr int SW = slot_words<KW>();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < count;
    bool improved = false, claimed = false;
    int64_t slot = 0;
    int f = 0;
    if (active) {
        const pastar_node nd = in[i];
        uint64_t key[KW];
        pack_key_dev<KW>(P, nd.pos, key);
        f = nd.f;
        slot = relax<KW, 1>(a.table, a.cap_mask, key, nd.g, nd.parent_mask, nd.f - nd.g, improved, claimed, false,
                            SlotWords<KW, 1>{});
        if (slot < 0) {
            if (slot == -2)
                atomicOr(&a.ctl->fault, (int)kSiteRelaxTail);
            improved = false;
            atomicAdd(&out[1], 1ull);
        } else if (improved) {
            // a ClosedList node improved: it leaves the ClosedList here
            // (ClosedList[tid].erase, PAStar.cpp:230) and is counted once
            // (nodes_reopen, :231), whichever of several improving entries
            // of one batch gets there first; its later dequeue then closes
            // an open node and counts nothing
            int *closed = reinterpret_cast<int *>(a.table + (uint64_t)slot * SW + KW + 1);
            if (*closed != kIntMax && atomicExch(closed, kIntMax) != kIntMax)
                atomicAdd(&out[0], 1ull);
        }
        added[i] = improved ? 1 : 0;
    }
    const int w = a.ctl->band_log2, f0 = a.ctl->f0;
    // every lane of the wave takes part in the append; entries may land
    // below the lowest bucket in use (host batches are not f-ordered)
    queue_append(a, improved, bucket_of(f, f0, w), Entry{(uint32_t)(slot < 0 ? 0 : slot), f}, a.stats, true);
}

// Entry at queue position p of (bucket b, sub-queue sq), or false when the
// position was reserved but never written (pool exhausted).
__device__ __forceinline__ bool queue_entry(const SearchArgs &a, int b, int sq, unsigned long long p, Entry &e)
{
    const uint32_t c = a.chunk_tab[((size_t)b * kSub + sq) * a.maxch + (p >> kChunkLog2)];
    if (c == 0 || c == kNoChunk)
        return false;
    e = a.pool[(size_t)(c - 1) * kChunk + (p & (kChunk - 1))];
    return true;
}

// PriorityList::dequeue (PriorityList.h:84-93) in batches, with the worker's
// ClosedList insert (worker_inner, PAStar.cpp:336-351): the lowest bucket
// holding live entries is scanned for its minimum f, and up to `max` nodes
// with that f leave the OpenList for the ClosedList (closed g = g).  peek:
// get_highest_priority (:116-122) only.  One block; res[0] = nodes out,
// res[1] = their f (INT_MAX when the OpenList is empty), res[2] = reopenings.
template <int KW>
__global__ __launch_bounds__(kListThreads) void lists_dequeue_kernel(SearchArgs a, pastar_node *__restrict__ out,
                                                                    int max, int peek, int *__restrict__ res)
{
    const DevProblem &P = *a.P;
    constexpr int SW = slot_words<KW>();
    const int tid = threadIdx.x;
    __shared__ unsigned long long r0[kSub], n_sq[kSub + 1];
    __shared__ int fmin_s, taken_s, reopen_s;
    __shared__ unsigned nlive_s;
    int b = ld_agent(&a.ctl->cur_b);
    if (b < 0)
        b = 0;
    int result_f = kIntMax;
    if (tid == 0) {  // an empty OpenList never enters the bucket loop
        taken_s = 0;
        reopen_s = 0;
    }
    __syncthreads();
    for (; b < kBuckets; b++) {
        if (tid < kSub) {
            const unsigned long long r = ld_agent(&a.q->R[b][tid]), w = ld_agent(&a.q->W[b][tid]);
            r0[tid] = r;
            n_sq[tid + 1] = w > r ? w - r : 0;
        }
        if (tid == 0) {
            n_sq[0] = 0;
            fmin_s = kIntMax;
            nlive_s = 0;
            taken_s = 0;
            reopen_s = 0;
        }
        __syncthreads();
        if (tid == 0)
            for (int sq = 0; sq < kSub; sq++)
                n_sq[sq + 1] += n_sq[sq];
        __syncthreads();
        const unsigned long long total = n_sq[kSub];
        // pass 1: the minimum f of the live entries
        for (unsigned long long k = tid; k < total; k += kListThreads) {
            int sq = 0;
            while (n_sq[sq + 1] <= k)
                sq++;
            Entry e;
            if (!queue_entry(a, b, sq, r0[sq] + (k - n_sq[sq]), e))
                continue;
            const uint64_t *s = a.table + (uint64_t)e.slot * SW;
            const uint64_t best = s[KW], aux = s[KW + 1];
            const int g = (int)(best >> 32), h = (int)(aux >> 32), closed = (int)(uint32_t)aux;
            if (best != ~0ull && g + h == e.f && g < closed) {
                atomicMin(&fmin_s, e.f);
                atomicAdd(&nlive_s, 1u);
            }
        }
        __syncthreads();
        if (nlive_s == 0) {
            // every entry of the bucket is stale or closed: consumed
            if (!peek && tid < kSub)
                st_agent(&a.q->R[b][tid], r0[tid] + (n_sq[tid + 1] - n_sq[tid]));
            __syncthreads();
            continue;
        }
        result_f = fmin_s;
        if (!peek) {
            // pass 2: up to max nodes of that f, each closed once (two live
            // entries of one node, from one enqueue batch, race on closed g)
            for (unsigned long long k = tid; k < total; k += kListThreads) {
                int sq = 0;
                while (n_sq[sq + 1] <= k)
                    sq++;
                Entry e;
                if (!queue_entry(a, b, sq, r0[sq] + (k - n_sq[sq]), e) || e.f != result_f)
                    continue;
                uint64_t *s = a.table + (uint64_t)e.slot * SW;
                const uint64_t best = s[KW], aux = s[KW + 1];
                const int g = (int)(best >> 32), h = (int)(aux >> 32);
                if (best == ~0ull || g + h != e.f || g >= (int)(uint32_t)aux)
                    continue;
                if (atomicAdd(&taken_s, 0) >= max)
                    continue;
                const int old = atomicMin(reinterpret_cast<int *>(s + KW + 1), g);
                if (old <= g)
                    continue;  // another entry of this node closed it
                const int at = atomicAdd(&taken_s, 1);
                if (at >= max) {
                    atomicMax(reinterpret_cast<int *>(s + KW + 1), old);  // over the limit: stays open
                    continue;
                }
                if (old != kIntMax)
                    atomicAdd(&reopen_s, 1);
                pastar_node nd;
                unpack_key_dev<KW>(P, s, nd.pos);
                nd.g = g;
                nd.f = e.f;
                nd.parent_mask = (int)(uint32_t)best;
                out[at] = nd;
            }
            __syncthreads();
            // entries ahead of the first live one are never looked at again:
            // each sub-queue's R moves past its leading run of dead entries
            // (stale, closed, or taken just now), so a bucket that drains
            // one node per call is not rescanned from its start every time
            if (tid < kSub) {
                const unsigned long long end = r0[tid] + (n_sq[tid + 1] - n_sq[tid]);
                unsigned long long r = r0[tid];
                for (; r < end; r++) {
                    Entry e;
                    if (!queue_entry(a, b, tid, r, e))
                        continue;  // reserved, never written: dead
                    const uint64_t *s = a.table + (uint64_t)e.slot * SW;
                    const uint64_t best = ld_agent(&s[KW]), aux = ld_agent(&s[KW + 1]);
                    const int g = (int)(best >> 32), h = (int)(aux >> 32);
                    if (best != ~0ull && g + h == e.f && g < (int)(uint32_t)aux)
                        break;  // live: stays
                }
                if (r != r0[tid])
                    st_agent(&a.q->R[b][tid], r);
            }
        }
        break;
    }
    if (tid == 0) {
        if (!peek)
            st_agent(&a.ctl->cur_b, b);
        res[0] = peek ? 0 : (taken_s < max ? taken_s : max);
        res[1] = result_f;
        res[2] = peek ? 0 : reopen_s;
    }
}

// OpenList / ClosedList sizes (PriorityList::size, ClosedList map size): nodes
// by state.  out[0] open, out[1] closed.
template <int KW>
__global__ __launch_bounds__(kListThreads) void lists_census_kernel(const uint64_t *__restrict__ table, uint64_t nslots,
                                                                   unsigned long long *__restrict__ out)
{
    constexpr int SW = slot_words<KW>();
    unsigned long long open = 0, closed = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t *s = table + i * SW;
        if (!s[0] || s[KW] == ~0ull)
            continue;
        const int g = (int)(s[KW] >> 32), c = (int)(uint32_t)s[KW + 1];
        open += g < c;
        closed += c != kIntMax && c <= g;
    }
    open = wave_sum(open);
    closed = wave_sum(closed);
    if (lane_id() == 0) {
        if (open)
            atomicAdd(&out[0], open);
        if (closed)
            atomicAdd(&out[1], closed);
    }
}

// find / erase of one coordinate.  res[0] = 0 absent, 1 open, 2 closed;
// res[1] = best, res[2] = aux.  erase_which (1 open, 2 closed): a node found
// in that list leaves both (its record is cleared: queue entries go stale).
template <int KW>
__global__ void lists_find_kernel(SearchArgs a, const uint16_t *__restrict__ pos, int erase_which,
                                  unsigned long long *__restrict__ res)
{
    const DevProblem &P = *a.P;
    constexpr int SW = slot_words<KW>();
    uint64_t key[KW];
    pack_key_dev<KW>(P, pos, key);
    const int64_t slot = lookup<KW>(a.table, a.cap_mask, key);
    res[0] = 0;
    if (slot < 0)
        return;
    uint64_t *s = a.table + (uint64_t)slot * SW;
    const uint64_t best = s[KW], aux = s[KW + 1];
    if (best == ~0ull)
        return;
    const int g = (int)(best >> 32), c = (int)(uint32_t)aux;
    const int where = g < c ? 1 : 2;
    res[0] = where;
    res[1] = best;
    res[2] = aux;
    if (erase_which == where) {
        s[KW] = ~0ull;
        s[KW + 1] = (aux & 0xffffffff00000000ull) | (uint32_t)kIntMax;
    }
}

}  // namespace dev
}  // namespace pastar
