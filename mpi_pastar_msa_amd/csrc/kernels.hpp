// kernels.hpp -- gfx950 kernels of the PAStar engine (see device.hpp for the
// data layout and DESIGN.md for the roofline of each kernel).
#pragma once

#include "device.hpp"
#include "pastar_gpu.h"

namespace pastar {
namespace dev {

// ---------------------------------------------------------------------------
// Table initialisation: keys 0, best = ~0, closed_g = INT_MAX, h = 0.
// ---------------------------------------------------------------------------
template <int SW>
__global__ __launch_bounds__(kBlock) void init_table_kernel(uint64_t *__restrict__ table, uint64_t nslots, int kw)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) {
        uint64_t *s = table + i * SW;
#pragma unroll
        for (int w = 0; w < SW; w++) {
            uint64_t v = 0;
            if (w == kw)
                v = ~0ull;
            else if (w == kw + 1)
                v = (uint64_t)kIntMax;
            s[w] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// PairAlign::Align as an anti-diagonal wavefront (PairAlign.cpp:107-171).
// One workgroup per pair; cell (i, j) depends on (i+1, j), (i, j+1) and
// (i+1, j+1), so every anti-diagonal i + j = d is independent.  The last
// three diagonals live in LDS (value + affine direction), indexed by row i;
// every cell is written once to the pair's H block.
// ---------------------------------------------------------------------------
enum { kNoGap = 0, kGapX = 1, kGapY = 2 };

__global__ __launch_bounds__(kBlock) void pairalign_kernel(const DevProblem *__restrict__ Pp, int32_t *__restrict__ H)
{
    const DevProblem &P = *Pp;
    const int p = blockIdx.x;
    const int x = P.pair_x[p], y = P.pair_y[p];
    const int L1 = P.len[x], L2 = P.len[y];
    const int GO = P.gap_open, GE = P.gap_ext;
    const uint8_t *s1 = P.codes + P.seq_off[x];
    const uint8_t *s2 = P.codes + P.seq_off[y];
    int32_t *M = H + P.h_off[p];
    const int W = L2 + 1;
    extern __shared__ int lds[];
    int *val = lds;                                       // [3][L1 + 1]
    unsigned char *dir = (unsigned char *)(lds + 3 * (L1 + 1));  // [3][L1 + 1]
    for (int d = L1 + L2; d >= 0; d--) {
        const int r0 = d % 3, r1 = (d + 1) % 3, r2 = (d + 2) % 3;
        const int ilo = d - L2 > 0 ? d - L2 : 0;
        const int ihi = d < L1 ? d : L1;
        for (int i = ilo + (int)threadIdx.x; i <= ihi; i += blockDim.x) {
            const int j = d - i;
            int m, a;
            if (i == L1 && j == L2) {
                m = 0;
                a = kNoGap;
            } else if (i == L1) {
                m = (j == L2 - 1) ? GO : val[r1 * (L1 + 1) + L1] + GE;
                a = kGapY;
            } else if (j == L2) {
                m = (i == L1 - 1) ? GO : val[r1 * (L1 + 1) + i + 1] + GE;
                a = kGapX;
            } else {
                const int down = val[r1 * (L1 + 1) + i + 1];  // (i+1, j)
                const int adown = dir[r1 * (L1 + 1) + i + 1];
                const int right = val[r1 * (L1 + 1) + i];     // (i, j+1)
                const int aright = dir[r1 * (L1 + 1) + i];
                const int c0 = down + (adown == kGapX ? GE : GO);
                const int c1 = right + (aright == kGapY ? GE : GO);
                if (c0 < c1) {
                    m = c0;
                    a = kGapX;
                } else {
                    m = c1;
                    a = kGapY;
                }
                const int c2 = val[r2 * (L1 + 1) + i + 1] + P.sub[s1[i] * P.alpha + s2[j]];
                if (c2 < m) {
                    m = c2;
                    a = kNoGap;
                }
            }
            val[r0 * (L1 + 1) + i] = m;
            dir[r0 * (L1 + 1) + i] = (unsigned char)a;
            M[(int64_t)i * W + j] = m;
        }
        __syncthreads();
    }
}

// h for a list of coordinates (HeuristicHPair::calculate_h), test/ABI helper.
__global__ void h_kernel(const DevProblem *__restrict__ Pp, const uint16_t *__restrict__ pos, int count,
                         int32_t *__restrict__ out)
{
    const DevProblem &P = *Pp;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count)
        return;
    const uint16_t *c = pos + (size_t)k * PASTAR_MAX_SEQ;
    int h = 0;
    for (int p = 0; p < P.npairs; p++) {
        const int x = P.pair_x[p], y = P.pair_y[p];
        h += P.H[P.h_off[p] + (int64_t)c[x] * P.h_row[p] + c[y]] * P.weight[p];
    }
    out[k] = h;
}

// ---------------------------------------------------------------------------
// Batched Node::getNeigh for the ABI (pastar_gpu_expand): every border-valid
// neighbour of each input node in increasing mask order, compacted within the
// node's lane group by ballot + prefix popcount.  Shares the parent staging
// and cost code with the search kernel.
// ---------------------------------------------------------------------------
template <int N, int KW>
__global__ __launch_bounds__(kBlock) void expand_api_kernel(const DevProblem *__restrict__ Pp,
                                                            const pastar_node *__restrict__ in, int n_in,
                                                            const int64_t *__restrict__ out_off, int vec_size,
                                                            pastar_node *__restrict__ out,
                                                            int32_t *__restrict__ out_owner,
                                                            int32_t *__restrict__ out_src)
{
    const DevProblem &P = *Pp;
    const int n = N ? N : P.n;
    const int npairs = P.npairs;
    const int lpn = (1 << n) < 64 ? (1 << n) : 64;
    const int npw = 64 / lpn;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int group = lane / lpn, glane = lane % lpn;
    __shared__ int2 terms_all[kWaves][kTPerWave];
    int2 *terms = &terms_all[wave][group * 4 * npairs];
    const uint64_t gmask = (lpn == 64 ? ~0ull : ((1ull << lpn) - 1ull)) << (group * lpn);
    const int per_block = kWaves * npw;
    for (int chunk = blockIdx.x; chunk * per_block < n_in; chunk += gridDim.x) {
        const int node = chunk * per_block + wave * npw + group;
        const bool active = node < n_in;
        Parent<N, KW> par;
        par.g = 0;
        par.pmask = 0;
        par.blocked = 0;
#pragma unroll
        for (int i = 0; i < Parent<N, KW>::NMAX; i++)
            par.pos[i] = 0;
        if (active) {
            const pastar_node &nd = in[node];
#pragma unroll
            for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
                par.pos[i] = (N || i < n) ? nd.pos[i] : 0;
                if ((N || i < n) && par.pos[i] >= P.len[i])
                    par.blocked |= 1 << i;
            }
            par.g = nd.g;
            par.pmask = nd.parent_mask;
            stage_terms<N, KW>(P, n, npairs, par, terms, glane, lpn);
        }
        __syncthreads();
        int64_t run = active ? out_off[node] : 0;
        const int masks = 1 << n;
        for (int r = 0; r * lpn < masks; r++) {
            const int m = r * lpn + glane;
            const bool valid = active && m >= 1 && m < masks && !(m & par.blocked);
            const uint64_t bal = __ballot(valid) & gmask;
            if (valid) {
                const int rank = __popcll(bal & ((1ull << lane) - 1ull));
                const int2 dc = child_cost<N>(P, npairs, terms, m);
                pastar_node c;
                int cp[Parent<N, KW>::NMAX];
#pragma unroll
                for (int i = 0; i < PASTAR_MAX_SEQ; i++)
                    c.pos[i] = 0;
#pragma unroll
                for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
                    cp[i] = par.pos[i] + ((m >> i) & 1);
                    if (N || i < n)
                        c.pos[i] = (uint16_t)cp[i];
                }
                c.g = par.g + dc.x;
                c.f = c.g + dc.y;
                c.parent_mask = m;
                const int64_t o = run + rank;
                out[o] = c;
                out_owner[o] = owner_dev<Parent<N, KW>::NMAX>(P, n, cp, vec_size);
                out_src[o] = node;
            }
            run += __popcll(bal);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Search kernels
// ---------------------------------------------------------------------------
__device__ __forceinline__ void hist_add(unsigned int *h, int f, int base)
{
    int b = f - base;
    b = b < 0 ? 0 : (b > kHistBins - 1 ? kHistBins - 1 : b);
    atomicAdd(&h[b], 1u);
}

__device__ __forceinline__ void hist_flush(unsigned int *lds_hist, unsigned int *global_hist)
{
    __syncthreads();
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) {
        const unsigned int v = lds_hist[b];
        if (v)
            atomicAdd(&global_hist[b], v);
    }
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

// Split the near pile: f <= t -> batch (at most kmax), t < f < bound -> the
// next near pile (with its f histogram relative to `base`), f >= bound -> drop.
// Block 0 also clears the other parity's StepStats for the next step.
__global__ __launch_bounds__(kBlock) void partition_kernel(const Entry *__restrict__ in, unsigned long long n,
                                                           int t, int bound, int base,
                                                           unsigned long long kmax, Entry *__restrict__ batch,
                                                           Entry *__restrict__ keep, unsigned long long keep_cap,
                                                           StepStats *__restrict__ st, StepStats *__restrict__ st_next)
{
    __shared__ unsigned int lh[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        lh[b] = 0;
    if (blockIdx.x == 0) {
        unsigned long long *z = (unsigned long long *)st_next;
        const int words = (int)(sizeof(StepStats) / 8);
        for (int w = threadIdx.x; w < words; w += blockDim.x)
            z[w] = 0;
    }
    __syncthreads();
    unsigned long long dropped = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long start = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long iters = (n + stride - 1) / stride;
    const int lane = lane_id();
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = start + it * stride;
        Entry e = {0, 0};
        const bool in_range = i < n;
        if (in_range)
            e = in[i];
        const bool drop = in_range && e.f >= bound;
        const bool sel = in_range && !drop && e.f <= t;
        dropped += drop;
        const uint64_t mask = __ballot(sel);
        unsigned long long bbase = 0;
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            if (lane == leader)
                bbase = atomicAdd(&st->batch_count, (unsigned long long)__popcll(mask));
            bbase = __shfl(bbase, leader);
        }
        const unsigned long long idx = bbase + __popcll(mask & ((1ull << lane) - 1ull));
        const bool to_batch = sel && idx < kmax;
        if (to_batch)
            batch[idx] = e;
        const bool to_keep = in_range && !drop && !to_batch;
        if (to_keep)
            hist_add(lh, e.f, base);
        wave_append(to_keep, &st->near_count, keep, keep_cap, e, &st->overflow);
    }
    dropped = wave_sum(dropped);
    if (lane == 0 && dropped)
        atomicAdd(&st->dropped, dropped);
    hist_flush(lh, st->hist);
}

struct SearchArgs {
    const DevProblem *P;
    uint64_t *table;
    uint64_t cap_mask;
    const Entry *batch;
    unsigned long long kmax;
    StepStats *st;
    Entry *near_out;
    unsigned long long near_cap;
    Entry *far_out;
    unsigned long long *far_n;
    unsigned long long far_cap;
    void *outbox;  // Remote<KW>[n_shards][outbox_cap]
    unsigned long long outbox_cap;
    int *goal_g;
    int t_near, bound, base, pad;
};

// Route one child: relax locally or post it to its owner shard; append the
// improved ones to the near / far pile.  All lanes of the wave must call it.
template <int KW>
__device__ __forceinline__ void route_child(const SearchArgs &a, const DevProblem &P, bool valid, bool local,
                                            int owner, const uint64_t (&ck)[KW], int g, int h, int m,
                                            unsigned int *lh, unsigned long long &claimed,
                                            unsigned long long &ovf)
{
    bool improved = false, cl = false;
    int64_t slot = 0;
    if (valid && local) {
        slot = relax<KW>(a.table, a.cap_mask, ck, g, m, h, improved, cl);
        if (slot < 0) {
            ovf++;
            improved = false;
        }
        claimed += cl;
        if (improved) {
            bool goal = true;
#pragma unroll
            for (int w = 0; w < KW; w++)
                goal &= (ck[w] == P.goal_key[w]);
            if (goal)
                atomicMin(a.goal_g, g);
        }
    }
    const int f = g + h;
    const Entry e = {(uint32_t)slot, f};
    const bool near = improved && f < a.t_near;
    const bool far = improved && f >= a.t_near;
    if (near)
        hist_add(lh, f, a.base);
    wave_append(near, &a.st->near_count, a.near_out, a.near_cap, e, &a.st->overflow);
    wave_append(far, a.far_n, a.far_out, a.far_cap, e, &a.st->overflow);
    if (P.n_shards > 1) {
        const bool remote = valid && !local;
        Remote<KW> rec;
#pragma unroll
        for (int w = 0; w < KW; w++)
            rec.key[w] = ck[w];
        rec.g = g;
        rec.h = h;
        rec.pmask = m;
        rec.pad = 0;
        Remote<KW> *ob = (Remote<KW> *)a.outbox;
        for (int d = 0; d < P.n_shards; d++)
            wave_append(remote && owner == d, &a.st->outbox_count[d], ob + (size_t)d * a.outbox_cap,
                        a.outbox_cap, rec, &a.st->overflow);
    }
}

// One search step: expand every entry of the batch (worker_inner's dequeue,
// closed check and getNeigh, PAStar.cpp:320-401) and relax its neighbours
// into the node table (PAStar::enqueue + conditional_enqueue, :219-237).
template <int N, int KW>
__global__ __launch_bounds__(kBlock) void expand_kernel(SearchArgs a)
{
    constexpr int SW = slot_words<KW>();
    const DevProblem &P = *a.P;
    const int n = N ? N : P.n;
    const int npairs = P.npairs;
    const int lpn = (1 << n) < 64 ? (1 << n) : 64;
    const int npw = 64 / lpn;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int group = lane / lpn, glane = lane % lpn;
    const int leader_lane = group * lpn;
    __shared__ int2 terms_all[kWaves][kTPerWave];
    __shared__ unsigned int lh[kHistBins];
    int2 *terms = &terms_all[wave][group * 4 * npairs];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        lh[b] = 0;
    const unsigned long long nb = a.st->batch_count < a.kmax ? a.st->batch_count : a.kmax;
    int bound = *(volatile int *)a.goal_g;
    bound = bound < a.bound ? bound : a.bound;
    unsigned long long expanded = 0, reopen = 0, generated = 0, claimed = 0, ovf = 0, stale = 0;
    const int per_block = kWaves * npw;
    const int masks = 1 << n;
    __syncthreads();
    for (unsigned long long chunk = blockIdx.x; chunk * per_block < nb; chunk += gridDim.x) {
        const unsigned long long node = chunk * per_block + wave * npw + group;
        bool ok = node < nb;
        Parent<N, KW> par;
        par.g = 0;
        par.pmask = 0;
        par.blocked = 0;
#pragma unroll
        for (int w = 0; w < KW; w++)
            par.key[w] = 0;
        if (ok) {
            const Entry e = a.batch[node];
            const uint64_t *s = a.table + (uint64_t)e.slot * SW;
#pragma unroll
            for (int w = 0; w < KW; w++)
                par.key[w] = s[w];
            const uint64_t best = s[KW];
            const int h = (int)(s[KW + 1] >> 32);
            par.g = (int)(best >> 32);
            par.pmask = (int)(uint32_t)best;
            ok = (par.g + h == e.f) && e.f < bound;
            int verdict = ok ? 1 : 0;
            if (ok && glane == 0) {
                const int old = atomicMin((int *)(a.table + (uint64_t)e.slot * SW + KW + 1), par.g);
                verdict = old <= par.g ? 0 : (old != kIntMax ? 2 : 1);
            }
            verdict = __shfl(verdict, leader_lane);
            ok = verdict != 0;
            if (glane == 0) {
                expanded += ok;
                reopen += verdict == 2;
                stale += !ok;
            }
        }
        if (ok) {
            decode_key<N, KW>(P, n, par.key, par.pos);
#pragma unroll
            for (int i = 0; i < Parent<N, KW>::NMAX; i++)
                if ((N || i < n) && par.pos[i] >= P.len[i])
                    par.blocked |= 1 << i;
            stage_terms<N, KW>(P, n, npairs, par, terms, glane, lpn);
        }
        __syncthreads();
        for (int r = 0; r * lpn < masks; r++) {
            const int m = r * lpn + glane;
            bool valid = ok && m >= 1 && m < masks && !(m & par.blocked);
            int g = 0, h = 0, owner = P.shard;
            uint64_t ck[KW];
#pragma unroll
            for (int w = 0; w < KW; w++)
                ck[w] = 0;
            if (valid) {
                const int2 dc = child_cost<N>(P, npairs, terms, m);
                g = par.g + dc.x;
                h = dc.y;
                generated++;
                if (g + h >= bound)
                    valid = false;
            }
            if (valid) {
                child_key<N, KW>(P, n, par.key, m, ck);
                if (P.n_shards > 1) {
                    int cp[Parent<N, KW>::NMAX];
#pragma unroll
                    for (int i = 0; i < Parent<N, KW>::NMAX; i++)
                        cp[i] = par.pos[i] + ((m >> i) & 1);
                    owner = owner_dev<Parent<N, KW>::NMAX>(P, n, cp, P.n_shards);
                }
            }
            route_child<KW>(a, P, valid, owner == P.shard, owner, ck, g, h, m, lh, claimed, ovf);
        }
        __syncthreads();
    }
    hist_flush(lh, a.st->hist);
    expanded = wave_sum(expanded);
    reopen = wave_sum(reopen);
    generated = wave_sum(generated);
    claimed = wave_sum(claimed);
    ovf = wave_sum(ovf);
    stale = wave_sum(stale);
    if (lane == 0) {
        if (expanded)
            atomicAdd(&a.st->expanded, expanded);
        if (reopen)
            atomicAdd(&a.st->reopen, reopen);
        if (generated)
            atomicAdd(&a.st->generated, generated);
        if (claimed)
            atomicAdd(&a.st->claimed, claimed);
        if (ovf)
            atomicAdd(&a.st->overflow, ovf);
        if (stale)
            atomicAdd(&a.st->dropped, stale);
    }
}

// Relax nodes received from other shards (the owner side of the RCCL
// exchange; replaces PAStarMessageProcesser -> enqueue, PAStar.cpp:241-250).
template <int KW>
__global__ __launch_bounds__(kBlock) void insert_remote_kernel(SearchArgs a, const Remote<KW> *__restrict__ recs,
                                                               unsigned long long count)
{
    const DevProblem &P = *a.P;
    __shared__ unsigned int lh[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        lh[b] = 0;
    __syncthreads();
    int bound = *(volatile int *)a.goal_g;
    bound = bound < a.bound ? bound : a.bound;
    unsigned long long claimed = 0, ovf = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long iters = (count + stride - 1) / stride;
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x + it * stride;
        bool valid = i < count;
        uint64_t ck[KW];
        int g = 0, h = 0, m = 0;
#pragma unroll
        for (int w = 0; w < KW; w++)
            ck[w] = 0;
        if (valid) {
            const Remote<KW> r = recs[i];
#pragma unroll
            for (int w = 0; w < KW; w++)
                ck[w] = r.key[w];
            g = r.g;
            h = r.h;
            m = r.pmask;
            valid = g + h < bound;
        }
        route_child<KW>(a, P, valid, true, P.shard, ck, g, h, m, lh, claimed, ovf);
    }
    hist_flush(lh, a.st->hist);
    claimed = wave_sum(claimed);
    ovf = wave_sum(ovf);
    if (lane_id() == 0) {
        if (claimed)
            atomicAdd(&a.st->claimed, claimed);
        if (ovf)
            atomicAdd(&a.st->overflow, ovf);
    }
}

// Far pile statistics: min f and live count over f < bound.
__global__ __launch_bounds__(kBlock) void far_min_kernel(const Entry *__restrict__ far, unsigned long long n,
                                                         int bound, FarStats *__restrict__ fs)
{
    int mn = kIntMax;
    unsigned long long live = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int f = far[i].f;
        if (f < bound) {
            mn = f < mn ? f : mn;
            live++;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int v = __shfl_xor(mn, o);
        mn = v < mn ? v : mn;
    }
    live = wave_sum(live);
    if (lane_id() == 0) {
        if (mn != kIntMax)
            atomicMin(&fs->min_f, mn);
        if (live)
            atomicAdd(&fs->live, live);
    }
}

__global__ __launch_bounds__(kBlock) void far_hist_kernel(const Entry *__restrict__ far, unsigned long long n,
                                                          int bound, int base, FarStats *__restrict__ fs)
{
    __shared__ unsigned int lh[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        lh[b] = 0;
    __syncthreads();
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int f = far[i].f;
        if (f < bound)
            hist_add(lh, f, base);
    }
    hist_flush(lh, fs->hist);
}

// Move far entries with f < t_near into the near pile (appended after
// `near_off` existing entries, histogram relative to `base`); keep
// t_near <= f < bound in the other far buffer; drop f >= bound.
__global__ __launch_bounds__(kBlock) void far_partition_kernel(const Entry *__restrict__ in, unsigned long long n,
                                                               int t_near, int bound, int base,
                                                               Entry *__restrict__ near_out,
                                                               unsigned long long near_cap,
                                                               Entry *__restrict__ far_out,
                                                               unsigned long long far_cap, StepStats *__restrict__ st)
{
    __shared__ unsigned int lh[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        lh[b] = 0;
    __syncthreads();
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long iters = (n + stride - 1) / stride;
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x + it * stride;
        Entry e = {0, 0};
        const bool in_range = i < n;
        if (in_range)
            e = in[i];
        const bool live = in_range && e.f < bound;
        const bool to_near = live && e.f < t_near;
        const bool to_far = live && e.f >= t_near;
        if (to_near)
            hist_add(lh, e.f, base);
        wave_append(to_near, &st->near_count, near_out, near_cap, e, &st->overflow);
        wave_append(to_far, &st->far_count, far_out, far_cap, e, &st->overflow);
    }
    hist_flush(lh, st->hist);
}

// Backtrace walk (backtrace.cpp:47-69): from `start`, follow parent masks,
// writing them to `masks`, until the origin, `max` steps, or (local_only) a
// parent owned by another shard.  Single lane.  info = {steps, status}.
template <int N, int KW>
__global__ void walk_kernel(const DevProblem *__restrict__ Pp, const uint64_t *__restrict__ table, uint64_t cap_mask,
                            const uint64_t *__restrict__ start, int max, int local_only,
                            int32_t *__restrict__ masks, uint64_t *__restrict__ last_key, int *__restrict__ info)
{
    const DevProblem &P = *Pp;
    const int n = N ? N : P.n;
    constexpr int SW = slot_words<KW>();
    uint64_t key[KW];
#pragma unroll
    for (int w = 0; w < KW; w++)
        key[w] = start[w];
    int steps = 0, status = 0;
    for (;;) {
        bool origin = true;
#pragma unroll
        for (int w = 0; w < KW; w++)
            origin &= key[w] == P.origin_key[w];
        if (origin) {
            status = 1;
            break;
        }
        if (steps >= max) {
            status = 2;
            break;
        }
        const int64_t s = lookup<KW>(table, cap_mask, key);
        if (s < 0) {
            status = -1;
            break;
        }
        const int m = (int)(uint32_t)table[(uint64_t)s * SW + KW];
        masks[steps++] = m;
        int pos[Parent<N, KW>::NMAX];
        decode_key<N, KW>(P, n, key, pos);
#pragma unroll
        for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
            if ((N == 0 && i >= n) || !((m >> i) & 1))
                continue;
            pos[i] -= 1;
            const uint64_t dec = 1ull << P.kshift[i];
            const int w = P.kword[i];
#pragma unroll
            for (int k = 0; k < KW; k++)
                if (w == k)
                    key[k] -= dec;
        }
        if (local_only && P.n_shards > 1 && owner_dev<Parent<N, KW>::NMAX>(P, n, pos, P.n_shards) != P.shard) {
            status = 3;
            break;
        }
    }
#pragma unroll
    for (int w = 0; w < KW; w++)
        last_key[w] = key[w];
    info[0] = steps;
    info[1] = status;
}

template <int KW>
__global__ void lookup_kernel(const uint64_t *__restrict__ table, uint64_t cap_mask, const uint64_t *__restrict__ key_in,
                              uint64_t *__restrict__ out)
{
    constexpr int SW = slot_words<KW>();
    uint64_t key[KW];
#pragma unroll
    for (int w = 0; w < KW; w++)
        key[w] = key_in[w];
    const int64_t s = lookup<KW>(table, cap_mask, key);
    if (s < 0) {
        out[0] = 0;
        return;
    }
    out[0] = 1;
    out[1] = table[(uint64_t)s * SW + KW];
    out[2] = table[(uint64_t)s * SW + KW + 1];
}

__global__ __launch_bounds__(kBlock) void count_table_kernel(const uint64_t *__restrict__ table, uint64_t nslots, int sw,
                                                             int kw, unsigned long long *__restrict__ out)
{
    unsigned long long used = 0, closed = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) {
        const uint64_t *s = table + i * sw;
        if (s[0]) {
            used++;
            closed += (int)(uint32_t)s[kw + 1] != kIntMax;
        }
    }
    used = wave_sum(used);
    closed = wave_sum(closed);
    if (lane_id() == 0) {
        atomicAdd(&out[0], used);
        atomicAdd(&out[1], closed);
    }
}

}  // namespace dev
}  // namespace pastar
