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

enum { kNoGap = 0, kGapX = 1, kGapY = 2 };  // PairAlign affine directions

// ---------------------------------------------------------------------------
// PairAlign::Align (PairAlign.cpp:107-171), one workgroup of kPaWaves
// wavefronts per pair, no block barriers in the sweep.  Rows are taken in
// bands of 64 from the bottom, lane l holding row bottom - 63 + l; a band
// sweeps the columns right to left with lane l lagging 63 - l steps behind
// lane 63, so the cell below, (i+1, j), is what lane l+1 produced one step
// earlier (a DPP wave shift) and the diagonal one, (i+1, j+1), the value
// received the step before.  Band k runs on wave k % kPaWaves and lags band
// k-1 by 64 steps: lane 63 reads the row below from band k-1's top row in
// LDS (ring of kPaWaves rows), gated by band k-1's published step count.
// Writes the pair's H block and its search form HC ({H * w, cost * w}).
// ---------------------------------------------------------------------------
constexpr int kPaWaves = 4;

__device__ __forceinline__ int from_lane_above(int v)
{
    // lane l receives lane l + 1's value (wave_shl:1; lane 63 gets 0)
    return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false);
}

// as from_lane_above, lane 63 receiving kPaInf (the row below the table)
constexpr int kPaInf = 0x3fffffff;
__device__ __forceinline__ int from_lane_above_inf(int v)
{
    return __builtin_amdgcn_update_dpp(kPaInf, v, 0x130, 0xf, 0xf, false);
}

__host__ __device__ constexpr size_t pairalign_lds_bytes(int maxl2, int alpha, bool sub_lds)
{
    return (size_t)kPaWaves * (maxl2 + 1) * 5 + (size_t)(maxl2 + 1) + (sub_lds ? (size_t)alpha * alpha * 4 : 0) +
           kPaWaves * 4 + 64;
}

// SUB_LDS: the distance table is staged in LDS (every read in the sweep is
// then an LDS read, and the per-step waits never include the stores).
// WRITE_H: also store the plain table H (only pastar_gpu_pair_table reads it;
// the search and h read HC).
// EQ_GAPS: gap open == gap extension (the reference's constants, Cost.h:13):
// the gap direction cannot change a value, so it is not tracked (a third
// fewer instructions per cell on the dependent chain).
//
// Stores: a lane owns one row, so a per-step store touches 64 rows (64 cache
// lines) for 4-8 B each and the CU's address path, not HBM, bounds the sweep.
// The HC cells of kPaChunk consecutive steps are therefore kept in registers
// and stored as one run of kPaChunk * 8 B per lane (16-B vector stores).
constexpr int kPaChunk = 8;
typedef int pa_v4i __attribute__((ext_vector_type(4), aligned(8)));

template <bool SUB_LDS, bool WRITE_H, bool EQ_GAPS>
__global__ __launch_bounds__(64 * kPaWaves) void pairalign_wave_kernel(const DevProblem *__restrict__ Pp,
                                                                       int32_t *__restrict__ H,
                                                                       int2 *__restrict__ HC,
                                                                       int *__restrict__ fault, unsigned spin_limit)
{
    static_assert(kPaChunk == 8, "the progress handshake runs every 8 steps, once per chunk");
    const DevProblem &P = *Pp;
    const int p = blockIdx.x;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int x = P.pair_x[p], y = P.pair_y[p], wgt = P.weight[p];
    const int L1 = P.len[x], L2 = P.len[y];
    // the search form alone with equal gap costs: the sweep runs in weighted
    // units (w * H: min and + commute with w >= 0, so every cell equals H * w)
    // on a distance table staged pre-weighted, with no multiply in the loop
    constexpr bool WEIGHTED = EQ_GAPS && !WRITE_H && SUB_LDS;
    const int GO = WEIGHTED ? P.gap_open * wgt : P.gap_open, GE = P.gap_ext;
    const int alpha = P.alpha;
    const uint8_t *s1 = P.codes + P.seq_off[x];
    const uint8_t *s2g = P.codes + P.seq_off[y];
    int32_t *M = H + P.h_off[p];
    int2 *C = HC + P.h_off[p];
    const int W = L2 + 1;
    extern __shared__ int lds[];
    int *bval = lds;                                              // [kPaWaves][L2 + 1] band top rows
    int *sub = bval + kPaWaves * W;                               // [alpha * alpha] when staged
    // [kPaWaves] band << 16 | steps done: an LDS-qualified pointer with
    // workgroup-scope atomics, so the handshake is ds_read / ds_write (a
    // volatile generic pointer compiles to flat accesses, and the wait after
    // each flat store then also waits for the chunk's HBM stores)
    typedef __attribute__((address_space(3))) int lds_int;
    lds_int *progress = (lds_int *)(sub + (SUB_LDS ? alpha * alpha : 0));
    uint8_t *bdir = (uint8_t *)(sub + (SUB_LDS ? alpha * alpha : 0) + kPaWaves);  // [kPaWaves][L2 + 1]
    uint8_t *s2 = bdir + kPaWaves * W;                            // [L2 + 1] codes of sequence y
    for (int k = threadIdx.x; k <= L2; k += blockDim.x)
        s2[k] = s2g[k];
    if (SUB_LDS)
        for (int k = threadIdx.x; k < alpha * alpha; k += blockDim.x)
            sub[k] = WEIGHTED ? P.sub[k] * wgt : P.sub[k];
    if (threadIdx.x < kPaWaves)
        __hip_atomic_store(&progress[threadIdx.x], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int32_t *subp;
    if constexpr (SUB_LDS)
        subp = sub;
    else
        subp = P.sub;
    __syncthreads();
    const int nbands = L1 / 64 + 1;  // rows L1 .. 0
    for (int band = wave; band < nbands; band += kPaWaves) {
        const int bottom = L1 - 64 * band;
        const int i = bottom - (63 - lane);
        const bool row_ok = i >= 0;
        const int cx = row_ok ? (int)s1[i] : 0;  // code 0 at i == L1 (string end)
        const int *crow = subp + cx * alpha;
        const bool last_row = i == L1, row_above_last = i == L1 - 1;
        const bool use_lds_below = lane == 63 && band > 0;
        const int *below = bval + ((band + kPaWaves - 1) % kPaWaves) * W;
        const uint8_t *belowd = bdir + ((band + kPaWaves - 1) % kPaWaves) * W;
        int *top = bval + (band % kPaWaves) * W;
        uint8_t *topd = bdir + (band % kPaWaves) * W;
        lds_int *prev_progress = progress + (band + kPaWaves - 1) % kPaWaves;
        lds_int *my_progress = progress + band % kPaWaves;
        int32_t *Mrow = M + (int64_t)(row_ok ? i : 0) * W;
        int2 *Crow = C + (int64_t)(row_ok ? i : 0) * W;
        // EQ_GAPS: the cells past the last row and column are +inf, so the
        // plain recurrence reproduces the borders (PairAlign.cpp:142-160:
        // +30 per step from the corner) and only the corner is seeded
        int m = EQ_GAPS ? kPaInf : 0, a = kNoGap;        // this lane's cell of the previous step: (i, j + 1)
        int down = EQ_GAPS ? kPaInf : 0, adown = kNoGap;  // (i + 1, j)
        int diag = 0;                   // (i + 1, j + 1)
        int j = L2 + 63 - lane;         // column of step t: L2 - (t - (63 - lane))
        int cost = (j >= 0 && j <= L2) ? crow[s2[j]] : 0;  // one step ahead
        const int nsteps = L2 + 64;
        for (int t0 = 0; t0 < nsteps; t0 += kPaChunk) {
            if (band > 0 && t0 <= L2) {
                // lane 63 reads column L2 - t of band - 1's top row, written
                // by its lane 0 at its step t + 63; one check covers 8 steps
                const int need = ((band - 1) << 16) | (t0 + 71 < nsteps ? t0 + 71 : nsteps);
                // (band - 1 runs on another wave of this workgroup and waits
                // only on band - 2, ..., band 0 on nothing; bounded all the same:
                // a wait that runs out flags the fault word and goes on with
                // whatever the row holds)
                unsigned poll = 0;
                while (__hip_atomic_load(prev_progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
                    if (++poll > spin_limit) {
                        if (lane == 0)
                            atomicOr(fault, (int)kSitePairAlign);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                asm volatile("" ::: "memory");  // the row reads below stay after the wait
            }
            const int j0 = j;  // this lane's column at step t0
            // the chunk's LDS operands, issued together ahead of the DP chain
            // (one LDS round trip per chunk, not two per step): the previous
            // band's top row (lane 63) and the distance row for columns
            // j0 - 1 .. j0 - 8 (the cost of step u + 1)
            int lb[kPaChunk], lbd[kPaChunk], nc[kPaChunk];
            if constexpr (EQ_GAPS) {
                // unclamped: a column outside the table only feeds cells
                // outside the table (a lane's column is its neighbour's of
                // the step before, minus one), so what those reads return
                // is never used; lb is lane 63's row below (+inf under the
                // table), the old value of the DPP shift below
#pragma unroll
                for (int u = 0; u < kPaChunk; u++) {
                    lb[u] = band > 0 ? below[j0 - u] : kPaInf;
                    lbd[u] = 0;
                    nc[u] = s2[j0 - u - 1];
                }
            } else {
#pragma unroll
                for (int u = 0; u < kPaChunk; u++) {
                    const int jj = j0 - u;
                    const int jc = jj < 0 ? 0 : (jj > L2 ? L2 : jj);
                    const int jn = jj - 1 < 0 ? 0 : (jj - 1 > L2 ? L2 : jj - 1);
                    lb[u] = below[jc];
                    lbd[u] = belowd[jc];
                    nc[u] = s2[jn];
                }
            }
#pragma unroll
            for (int u = 0; u < kPaChunk; u++)
                nc[u] = crow[nc[u]];
            int2 cb[kPaChunk];
            int tb[kPaChunk], tbd[kPaChunk];
#pragma unroll
            for (int u = 0; u < kPaChunk; u++, j--) {
                // row i + 1 at column j: produced last step by the lane above
                // (lane 63: the previous band's top row); (i + 1, j + 1) is
                // last step's (i + 1, j).  Branch-free: every lane computes,
                // only cells inside the table are kept.  Steps past the sweep
                // (t >= nsteps) have j < 0 on every lane and change nothing.
                const bool in = row_ok && j >= 0 && j <= L2;
                int mm, aa = kNoGap;
                const int cost_here = cost;
                cost = nc[u];
                if constexpr (EQ_GAPS) {
                    // lane 63 has no lane above: the shift leaves it the old
                    // value, the previous band's top row (or +inf)
                    diag = down;
                    down = __builtin_amdgcn_update_dpp(lb[u], m, 0x130, 0xf, 0xf, false);
                    const int right = m;
                    mm = (down < right ? down : right) + GO;
                    const int c2 = diag + cost_here;
                    mm = c2 < mm ? c2 : mm;
                    mm = (last_row && t0 + u == 0) ? 0 : mm;  // the corner (L1, L2)
                } else {
                    const int m_up = from_lane_above(m), a_up = from_lane_above(a);
                    diag = down;
                    down = use_lds_below ? lb[u] : m_up;
                    adown = use_lds_below ? lbd[u] : a_up;
                    const int right = m, aright = a;
                    const int c0 = down + (adown == kGapX ? GE : GO);
                    const int c1 = right + (aright == kGapY ? GE : GO);
                    mm = c0 < c1 ? c0 : c1;
                    aa = c0 < c1 ? kGapX : kGapY;
                    const int c2 = diag + cost_here;
                    aa = c2 < mm ? kNoGap : aa;
                    mm = c2 < mm ? c2 : mm;
                    const bool last_col = j == L2;
                    // borders (PairAlign.cpp:142-160)
                    const int m_lastcol = row_above_last ? GO : down + GE;
                    const int m_lastrow = (j == L2 - 1) ? GO : right + GE;
                    mm = last_row ? (last_col ? 0 : m_lastrow) : (last_col ? m_lastcol : mm);
                    aa = last_row ? (last_col ? kNoGap : kGapY) : (last_col ? kGapX : aa);
                }
                // unsigned: cells outside the table may hold +inf, never stored
                if constexpr (WEIGHTED)
                    cb[u] = make_int2(mm, cost_here);
                else
                    cb[u] = make_int2((int)((unsigned)mm * (unsigned)wgt), cost_here * wgt);
                // a column left of the table only feeds cells left of it:
                // only the columns right of it must stay +inf
                m = (EQ_GAPS ? j <= L2 : in) ? mm : m;
                a = EQ_GAPS ? 0 : (in ? aa : a);
                tb[u] = m;
                tbd[u] = a;
                if constexpr (WRITE_H)
                    if (in)
                        Mrow[j] = mm;
            }
            // lane 0's cells are the band's top row, which the next band
            // reads: stored once per chunk, then the chunk is published
            if (lane == 0) {
#pragma unroll
                for (int u = 0; u < kPaChunk; u++) {
                    const int jj = j0 - u;
                    if (row_ok && jj >= 0 && jj <= L2) {
                        top[jj] = tb[u];
                        if constexpr (!EQ_GAPS)
                            topd[jj] = (uint8_t)tbd[u];
                    }
                }
                // the row's LDS writes stay before the publication (a wave's
                // LDS operations complete in order)
                asm volatile("" ::: "memory");
                __hip_atomic_store(my_progress, (band << 16) | (t0 + kPaChunk < nsteps ? t0 + kPaChunk : nsteps),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            // the chunk's cells of this lane's row are columns j0 - 7 .. j0
            const int jlo = j0 - (kPaChunk - 1);
            if (row_ok && jlo >= 0 && j0 <= L2) {
                pa_v4i *dst = reinterpret_cast<pa_v4i *>(Crow + jlo);
#pragma unroll
                for (int k = 0; k < kPaChunk / 2; k++) {
                    const int2 lo = cb[kPaChunk - 1 - 2 * k], hi = cb[kPaChunk - 2 - 2 * k];
                    dst[k] = pa_v4i{lo.x, lo.y, hi.x, hi.y};
                }
            } else if (row_ok) {
#pragma unroll
                for (int u = 0; u < kPaChunk; u++) {
                    const int jj = j0 - u;
                    if (jj >= 0 && jj <= L2)
                        Crow[jj] = cb[u];
                }
            }
        }
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
        h += P.HC[P.h_off[p] + (int64_t)c[x] * P.h_row[p] + c[y]].x;  // H * w
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
    __shared__ PairConst pc[kMaxPairs];
    int2 *terms = &terms_all[wave][group * 4 * npairs];
    const uint64_t gmask = (lpn == 64 ? ~0ull : ((1ull << (lpn & 63)) - 1ull)) << (group * lpn);
    const int per_block = kWaves * npw;
    stage_pairs(P, pc);
    __syncthreads();
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
            stage_terms<N, KW>(P, n, npairs, pc, par, terms, glane, lpn);
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
// Search kernels.
//
// Open list: f-bucketed FIFO queues.  Bucket b holds the open entries with
// f in [f0 + b*band, f0 + (b+1)*band) (the last bucket also everything
// above).  Each bucket is split into kSub sub-queues (a block appends to
// sub-queue blockIdx % kSub, so an append counter is shared by one XCD's
// blocks only), and a sub-queue is a list of kChunk-entry chunks taken from a
// pool by a bump allocator.  Positions are 64-bit counters: W (reserved by
// appends) and R (consumed by batches).  Nothing is ever rewritten.
//
// One step is two launches that read their plan from the device-resident
// Ctl block, so runs of steps are replayed as one hipGraph:
//   select  (1 block): book-keeping, find the lowest bucket with entries,
//                      cut a batch of at most kmax entries from it
//   expand           : expand the batch, relax children, append improved ones
// ---------------------------------------------------------------------------
constexpr int kSub = 32;           // sub-queues per bucket
constexpr int kBuckets = 2048;     // f buckets
constexpr int kChunkLog2 = 12;     // entries per chunk = 4096 (32 KB)
constexpr int kChunk = 1 << kChunkLog2;
constexpr uint32_t kNoChunk = 0xffffffffu;
constexpr int kWide = 4;                   // buckets a thin batch may span
constexpr int kRanges = kWide * kSub;      // (bucket, sub-queue) ranges of a batch
constexpr int kArrive = 64;                // first-level arrival counters of expand

enum { kFailNear = 1, kFailFar = 2, kFailTable = 4, kFailOut = 8 };  // near = chunk pool, far = chunk table

__host__ __device__ inline int fail_bits(unsigned long long near, unsigned long long far, unsigned long long table,
                                          unsigned long long out)
{
    return (near ? kFailNear : 0) | (far ? kFailFar : 0) | (table ? kFailTable : 0) | (out ? kFailOut : 0);
}

// Device-resident control block.  Grouped by access: the read-mostly words
// every expand block loads at its start, then each atomically updated word
// on a cache line of its own (a hot atomic line shared with words that every
// block reads slows every launch), then the last block's diagnostics.
struct Ctl {
    // ---- read by every block, written by select ----
    int status;     // 0 running, 1 done, 2 capacity exhausted, 3 step limit, 4 a bounded device wait ran out
    int band_log2;  // bucket width = 2^band_log2
    int f0;         // f of bucket 0 (h of the origin)
    int batch_b;    // first bucket of the current batch
    int batch_nb;   // buckets the current batch was cut from
    int depth;      // expansion levels per launch (block-local continuation)
    int deep_rounds;  // continuation only when a level may take >= this many rounds
    int n_shards;
    int timing;     // profile bits: 1 launch timing, 2 select phases, 4 expand phases
    int fuse;       // 1: the last expand block also runs select for the next step
    int fail_mask;  // kFail* bits of the capacity that ran out
    int has_work;   // select found a live bucket (multi-shard termination)
    int low_found;  // that bucket (kBuckets: none)
    int xwindow;    // sharded: buckets above the shards' common lowest live bucket a batch may be cut from
    int debug;      // 1: select validates its scan start (diagnostics)
    int deep_blocks;  // block-rounds per continuation level across the chip (kDeepBlocks by default)
    int prune_f;      // children with f >= this are not generated (an upper bound of the optimum + 1; kIntMax: none)
    int partial_k;    // partial expansion: children with f at or past the batch's last bucket + this many buckets
                      // wait until their parent is taken again (negative: every child at once)
    int partial_ahead;  // that parent is queued this many buckets before its first waiting child's
    int partial_two;    // a parent taken again: 1 (default) generates every child it has left; 0 the same window
                        // again; 2 a window that doubles its reach past the parent's f (tuning probes)
    unsigned long long kmax;
    unsigned long long pool_chunks, maxch;
    unsigned long long table_slots;
    unsigned long long n_batch;
    unsigned long long kmin;  // a batch smaller than this may pull the next buckets
    unsigned long long b_start[kRanges], b_prefix[kRanges + 1];
    // ---- select's running totals ----
    long long steps, max_steps;
    unsigned long long expanded, reopen, generated, claimed, dropped, parents;
    unsigned long long part_queued, part_taken;  // partial expansion: parents queued again / taken again
    // ---- atomics, one line each ----
    alignas(128) unsigned long long pool_top;  // chunk bump allocator
    alignas(128) int cur_b;  // lowest bucket that may hold entries (f_min only grows)
    // lowest bucket appended to by kernels that run beside select (the sharded
    // search's insert kernel on the side stream): select takes it by exchange
    // and starts its scan there, so a lowering can never be lost under
    // select's own store of cur_b (kBuckets: none)
    alignas(128) int low_b;
    // arrival counters of the expand blocks (two levels: blockIdx % kArrive,
    // then the groups), reset by the last block
    alignas(128) unsigned arrive_top;
    alignas(128) unsigned arrive[kArrive];
    // ---- last block only: expand-kernel timing on the 100 MHz device clock
    // (s_memrealtime): the first kArrive blocks stamp their start (blocks are
    // dispatched in index order), the last block to finish takes the earliest
    // stamp and its own end, and sums over the launches ----
    alignas(128) unsigned long long k_start, k_end, expand_ticks, timed_launches;
    unsigned long long select_ticks, gap_ticks, prev_end;
    unsigned long long phase_ticks[8];  // profile: select phases (diagnostics)
    unsigned long long body_ticks[18];  // profile: expand phases of block 0 (diagnostics; 10, 11: dive counts; 12..: dive phases)
    unsigned long long body_launches;
    // profile (PASTAR_PHASE_TIMERS builds): per-block chain statistics,
    // {blocks, sum levels, max levels, sum rounds, max rounds, max ticks},
    // then continuation levels by parents: 1, 2..4, 5..16, more
    unsigned long long blk_stats[10];
    int dbg_hits, dbg_bucket, dbg_cur, dbg_win, dbg_step;
    int fault_sites;  // status 4: the kSite* bits select found in the fault word
    // kSite* bits of bounded device waits that ran out (device.hpp), ORed in
    // by the waiter: sticky, kept across the per-search upload of this block
    // (search_init_kernel skips the word), cleared by the host when it
    // reports the fault.  The PairAlign kernel, which runs before a search's
    // setup, flags its band wait here too.
    alignas(128) int fault;
    unsigned spin_limit;  // polls a queue store waits for its chunk id (kSpinLimit; tests lower it)
    unsigned long long dbg_w, dbg_r;
};

__device__ __forceinline__ unsigned long long device_clock() { return __builtin_amdgcn_s_memrealtime(); }

// Cursor arrays indexed [bucket][sub-queue] but stored sub-queue-major: the
// 32 sub-queues of one bucket (appended to by blocks of different XCDs at
// once) sit on 32 different cache lines.
struct CursorArray {
    unsigned long long d[kSub][kBuckets];
    struct Row {
        unsigned long long *p;
        __host__ __device__ unsigned long long &operator[](int sq) const { return p[(size_t)sq * kBuckets]; }
    };
    struct CRow {
        const unsigned long long *p;
        __host__ __device__ const unsigned long long &operator[](int sq) const { return p[(size_t)sq * kBuckets]; }
    };
    __host__ __device__ Row operator[](int b) { return Row{&d[0][b]}; }
    __host__ __device__ CRow operator[](int b) const { return CRow{&d[0][b]}; }
};

struct Queues {
    CursorArray W;  // reserved by appends
    CursorArray R;  // consumed by batches
};

constexpr int kMaxExpandBlocks = 4096;
// register budget of expand_kernel<N, KW>: waves per SIMD it must fit, which
// is also its resident blocks per CU (a block is one wave on each SIMD)
// (5 for N <= 5 spills 36-72 B per lane and ran kinase 20% slower)
#ifndef PASTAR_WIDE_WAVES
#define PASTAR_WIDE_WAVES 4
#endif
__host__ __device__ constexpr int expand_waves_per_eu(int n, int) { return n >= 7 ? PASTAR_WIDE_WAVES : 4; }
constexpr int kTraceSteps = 4096;

struct SearchArgs {
    const DevProblem *P;
    Ctl *ctl;  // (also holds the fault word and the store wait's poll limit: values the hot loops never
               // touch stay out of the kernel arguments, which live in scalar registers for the whole launch)
    unsigned long long *stamps;  // [kArrive] start stamps of the first blocks
    int *trace;                  // debug: [kTraceSteps][8] per-step select trace (nullptr: off)
    uint64_t *table;
    uint64_t cap_mask;
    Queues *q;
    uint32_t *chunk_tab;  // [kBuckets][kSub][maxch], chunk id + 1
    Entry *pool;          // [pool_chunks][kChunk]
    StepStats *stats;
    int *goal_g;
    void *outbox;  // Remote<KW>[n_shards][outbox_cap]: a ring per destination shard
    unsigned long long outbox_cap;  // a power of two
    int *lower;    // the word an append below the lowest bucket in use lowers: Ctl::cur_b, or Ctl::low_b
                   // for appends that run beside a select (the sharded search's insert kernel)
    XState *x;     // shard exchange state (nullptr: one-shard search)
    int step;      // this launch's step (its slot of XState's per-step values)
    // the open-list capacities (= Ctl's), as kernel arguments: an append
    // then computes its chunk-table address without a load of the control
    // block ahead of the chunk-table read
    unsigned long long maxch, pool_chunks;
};

// (DPP lane moves, no LDS round trips; every lane of the wave must be active)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void wave_sum_step64(unsigned &lo, unsigned &hi)
{
    const unsigned l2 = (unsigned)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, ROW_MASK, 0xf, false);
    const unsigned h2 = (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, ROW_MASK, 0xf, false);
    const unsigned long long t = (((unsigned long long)hi << 32) | lo) + (((unsigned long long)h2 << 32) | l2);
    lo = (unsigned)t;
    hi = (unsigned)(t >> 32);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
    // an inclusive row scan (row_shr 1, 2, 4, 8), then row_bcast 15 and 31: lane 63 holds the total
    unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
    wave_sum_step64<0x111, 0xf>(lo, hi);
    wave_sum_step64<0x112, 0xf>(lo, hi);
    wave_sum_step64<0x114, 0xf>(lo, hi);
    wave_sum_step64<0x118, 0xf>(lo, hi);
    wave_sum_step64<0x142, 0xa>(lo, hi);
    wave_sum_step64<0x143, 0xc>(lo, hi);
    const unsigned tl = (unsigned)__builtin_amdgcn_readlane((int)lo, 63), th = (unsigned)__builtin_amdgcn_readlane((int)hi, 63);
    return ((unsigned long long)th << 32) | tl;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) { return (unsigned)wave_sum_i32((int)v); }

// Wave-aggregated append to a destination's outbox ring: one atomic per wave
// on the ring's append position; a record that would overrun what the pack
// kernel has consumed (r, read possibly stale, i.e. low: conservative) is
// counted as an outbox overflow.  Must be reached by every lane of the wave.
template <typename T>
__device__ __forceinline__ void ring_append(bool pred, unsigned long long *w, const unsigned long long *r_pub, T *ring,
                                            unsigned long long cap, const T &v, unsigned long long *overflow)
{
    const uint64_t mask = __ballot(pred);
    if (!mask)
        return;
    const int lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    unsigned long long base = 0, r = 0;
    if (lane == leader) {
        base = atomicAdd(w, (unsigned long long)__popcll(mask));
        r = __hip_atomic_load(r_pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    base = bcast_lane(base, leader);
    r = bcast_lane(r, leader);
    if (pred) {
        const unsigned long long pos = base + __popcll(mask & ((1ull << lane) - 1ull));
        if (pos - r < cap)
            ring[pos & (cap - 1)] = v;
        else
            atomicAdd(overflow, 1ull);
    }
}

// Loads of words other blocks of the same launch update with atomics (the
// fused select runs in the last expand block): coherent across XCDs.
template <typename T>
__device__ __forceinline__ T ld_agent(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stores to words that other launches update with atomics (cursors, cur_b,
// counters): atomic too, so that a plain store's copy in one XCD's L2 can
// never land over a later atomic update from another XCD.
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int bucket_of(int f, int f0, int w)
{
    const long long b = ((long long)f - f0) >> w;
    return b < 0 ? 0 : (b >= kBuckets ? kBuckets - 1 : (int)b);
}

// Reserve n consecutive positions of sub-queue (b, sq) (n <= kChunk; one
// lane) and open every chunk whose first position falls in the reserved
// range: its id is taken from the pool and published in the chunk table
// before this lane does anything else.  A store into a chunk (queue_store)
// waits for that publication, so what a store waits on is always one lane
// that has finished its cursor add and whose next instructions are the pool
// add and the publication, with no wait of its own in between: stores can
// form no circular wait, in whatever order blocks reserve ranges of several
// buckets and store into them.  (The chunk id is the only datum handed over,
// so the publication is relaxed: an agent-scope release or acquire would
// write back or invalidate the L2 on every append.)
__device__ __forceinline__ unsigned long long queue_reserve(const SearchArgs &a, int b, int sq, unsigned n)
{
    const unsigned long long base = atomicAdd(&a.q->W[b][sq], (unsigned long long)n);
    // (n <= kChunk: at most one chunk starts inside the range; the rare
    // path reads its capacities from the control block, not from kernel
    // arguments that would sit in scalar registers for the whole launch)
    const unsigned to_next = (unsigned)(-(long long)base) & (kChunk - 1);  // positions up to the next chunk start
    if (to_next < n) {
        const unsigned long long k = (base + to_next) >> kChunkLog2;
        Ctl *ctl = a.ctl;
        if (k < a.maxch) {
            const unsigned long long id = atomicAdd(&ctl->pool_top, 1ull);
            const uint32_t c = id < ctl->pool_chunks ? (uint32_t)(id + 1) : kNoChunk;
            __hip_atomic_store(a.chunk_tab + ((size_t)b * kSub + sq) * a.maxch + k, c, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    return base;
}

// Write entry e at position p (reserved by queue_reserve) of sub-queue
// (b, sq).  The chunk's id is read from the chunk table; a position whose
// chunk's reserver has not published yet waits for it, at most
// a.spin_limit polls (see queue_reserve: the reserver never waits).
__device__ __forceinline__ void queue_store(const SearchArgs &a, int b, int sq, unsigned long long p, const Entry &e,
                                            StepStats *st)
{
    const unsigned long long k = p >> kChunkLog2;
    const unsigned off = (unsigned)(p & (kChunk - 1));
    const unsigned long long maxch = a.maxch;
    if (k >= maxch) {
        atomicAdd(&st->ovf_far, 1ull);
        return;
    }
    uint32_t *tp = a.chunk_tab + ((size_t)b * kSub + sq) * maxch + k;
    uint32_t c = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c == 0) {
        const unsigned limit = a.ctl->spin_limit;
        for (unsigned poll = 0; poll < limit && c == 0; poll++) {
            __builtin_amdgcn_s_sleep(1);
            c = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (c == 0) {  // the wait ran out: flag it, drop the entry
            atomicOr(&a.ctl->fault, (int)kSiteQueueStore);
            return;
        }
    }
    if (c == kNoChunk) {
        atomicAdd(&st->ovf_near, 1ull);
        return;
    }
    a.pool[(size_t)(c - 1) * kChunk + off] = e;
}

// Wave-aggregated append of the predicated lanes' entries to their buckets:
// one atomic per distinct bucket in the wave.  Every lane must call it.
// may_lower: entries can land below cur_b (records from other shards; a
// shard's own children never fall below the bucket of their parent).
__device__ __forceinline__ void queue_append(const SearchArgs &a, bool pred, int b, const Entry &e, StepStats *st,
                                             bool may_lower)
{
    const int sq = blockIdx.x % kSub;
    const int lane = lane_id();
    uint64_t pending = __ballot(pred);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int bl = bcast_lane(b, leader);
        const uint64_t m = __ballot(pred && b == bl) & pending;
        unsigned long long base = 0;
        if (lane == leader) {
            base = queue_reserve(a, bl, sq, (unsigned)__popcll(m));
            // entries from other shards may land below this shard's minimum:
            // lowered after the cursor add has returned (the reservation is
            // performed before whoever sees the lowered word reads the cursor)
            if (may_lower) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (bl < ld_agent(a.lower))
                    atomicMin(a.lower, bl);
            }
#ifdef PASTAR_TRACE_APPENDS
            if (a.trace) {
                const long long stp = ld_agent(&a.ctl->steps);
                if (stp < kTraceSteps)
                    atomicMin(&a.trace[stp * 8 + 6], bl);  // lowest bucket appended after select `stp`
            }
#endif
        }
        base = bcast_lane(base, leader);
        if ((m >> lane) & 1ull)
            queue_store(a, bl, sq, base + __popcll(m & ((1ull << lane) - 1ull)), e, st);
        pending &= ~m;
    }
}

// Block-local continuation queue (LDS): improved children whose f lies in
// the current batch's buckets are expanded by the same block in the same
// launch, up to `depth` levels, instead of waiting for the next step.
#ifndef PASTAR_LOCAL_CAP
#define PASTAR_LOCAL_CAP 128
#endif
constexpr int kLocalCap = PASTAR_LOCAL_CAP;
constexpr int kDeepBlocks = 1024;  // block-rounds per continuation level across the chip (profiles/r2_tune_deep_blocks.txt)
// A continuation entry carries the parent as relaxed (key, g, h, mask), so
// the next level needs no table read before it stages the pair terms.
template <int KW>
struct LEntry {
    uint64_t key[KW];
    uint32_t slot;
    int g, h, pmask;
};

template <int KW>
struct LocalPush {
    LEntry<KW> *buf;  // nullptr: disabled
    int *count;
    int f_limit;
    int cap;     // entries one level may take (a block's width per round)
    Entry *out;  // block's outgoing buffer for the open list, appended once
    int *out_n;  // at the end of the launch (nullptr: append at once)
    // A kernel that runs beside a select (the sharded search's insert with
    // xchg_lag = 1) must not append to the open list itself: a select could
    // cut a position that is reserved but not yet written.  Its entries go to
    // a staging array instead, which a launch on the select's own stream
    // appends later (xdrain_kernel).
    Entry *stage;
    unsigned long long *stage_n;
    unsigned long long stage_cap;
};

constexpr int kOutCap = 1024;  // entries a block defers to its final append
static_assert(kOutCap <= kChunk, "one reservation opens at most one chunk");

// A group leader's verdict (0, 1, 2) to every lane of its group, by two
// ballots (no LDS round trip; the leader lane is per group, not uniform)
__device__ __forceinline__ int group_verdict(int verdict, int leader_lane)
{
    const uint64_t one = __ballot(verdict == 1), two = __ballot(verdict == 2);
    return ((two >> leader_lane) & 1ull) ? 2 : (int)((one >> leader_lane) & 1ull);
}

// Block barrier for LDS data only: outstanding global stores (closed marks,
// queue entries) need not land before the block moves on.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Open-list append of the predicated lanes' entries: into the block's
// deferred buffer while it has room (one cursor atomic per bucket for the
// whole block at the end of the launch), else at once.  Every lane of the
// wave must call it.
template <int KW>
__device__ __forceinline__ void open_append(const SearchArgs &a, const LocalPush<KW> &lp, bool pred, int b,
                                            const Entry &e, StepStats *st, bool may_lower)
{
    if (lp.stage) {
        wave_append(pred, lp.stage_n, lp.stage, lp.stage_cap, e, &st->ovf_near);
        return;
    }
    if (lp.out) {
        const uint64_t mask = __ballot(pred);
        if (mask) {
            const int lane = lane_id();
            const int leader = __ffsll((long long)mask) - 1;
            int base = 0;
            if (lane == leader)
                base = atomicAdd(lp.out_n, __popcll(mask));
            base = bcast_lane(base, leader);
            if (pred) {
                const int pos = base + __popcll(mask & ((1ull << lane) - 1ull));
                if (pos < kOutCap) {
                    lp.out[pos] = e;
                    pred = false;
                }
            }
        }
    }
    queue_append(a, pred, b, e, st, may_lower);
}

// Queue an improved child of this shard: into the block-local continuation
// queue when its f lies in the batch's buckets and the queue has room, else
// into the open list.  Every lane of the wave must call it.
template <int KW>
__device__ __forceinline__ void queue_improved(const SearchArgs &a, StepStats *st, int f0, int w, bool pred,
                                               int64_t slot, const uint64_t (&ck)[KW], int g, int h, int m,
                                               const LocalPush<KW> &lp, bool may_lower = false)
{
    const int f = g + h;
    const Entry e = {(uint32_t)slot, f};
    bool global = pred;
    if (lp.buf) {
        const bool want = pred && f < lp.f_limit;
        const uint64_t mask = __ballot(want);
        if (mask) {
            const int lane = lane_id();
            const int leader = __ffsll((long long)mask) - 1;
            int base = 0;
            if (lane == leader)
                base = atomicAdd(lp.count, __popcll(mask));
            base = bcast_lane(base, leader);
            if (want) {
                const int pos = base + __popcll(mask & ((1ull << lane) - 1ull));
                if (pos < lp.cap) {
                    LEntry<KW> le;
#pragma unroll
                    for (int k = 0; k < KW; k++)
                        le.key[k] = ck[k];
                    le.slot = (uint32_t)slot;
                    le.g = g;
                    le.h = h;
                    le.pmask = m;
                    lp.buf[pos] = le;
                    global = false;
                }
            }
        }
    }
    open_append(a, lp, global, bucket_of(f, f0, w), e, st, may_lower);
}

// Route one child: relax locally or post it to its owner shard; queue the
// improved ones (block-local continuation queue first, when it qualifies).
// All lanes of the wave must call it.
// SH = false: the one-shard search (no owner routing, no outbox code)
template <int KW, int PFS = 1, bool SH = true, typename PP>
__device__ __forceinline__ void route_child(const SearchArgs &a, const PP &P, StepStats *st, int f0, int w,
                                            bool valid, bool local, int owner, const uint64_t (&ck)[KW], int g, int h,
                                            int m, unsigned &claimed, unsigned &ovf,
                                            const LocalPush<KW> &lp, bool remote_in = false, bool has_pre = false,
                                            const SlotWords<KW, PFS> &pre = SlotWords<KW, PFS>{})
{
    bool improved = false, cl = false;
    int64_t slot = 0;
    // Sharded search: a child owned by another shard is relaxed into this
    // shard's table too (a record of the best g this shard has sent for it)
    // and goes to its owner only when that improved: each shard sends a
    // node once per improvement it finds, not once per parent, which cuts
    // the exchange by the number of parents a shard holds of one node.  The
    // owner's table alone is authoritative for the node (open list,
    // closed mark, backtrace).
    // Ties count: a record with the best g this shard has seen and a
    // smaller parent mask is sent too, so the owner ends with the smallest
    // mask over all shards' parents, as the one-shard table does.
    const bool filter = SH && P.n_shards > 1;
    bool lowered = false;
    if (valid && (local || filter)) {
        slot = relax<KW, PFS>(a.table, a.cap_mask, ck, g, m, h, improved, cl, has_pre, pre, &lowered);
        if (slot < 0) {
            if (slot == -2)
                atomicOr(&a.ctl->fault, (int)kSiteRelaxTail);
            ovf++;
            improved = false;
            lowered = false;
        }
        claimed += cl;
        if (improved) {
            bool goal = true;
#pragma unroll
            for (int k = 0; k < KW; k++)
                goal &= (ck[k] == P.goal_key[k]);
            if (goal)
                atomicMin(a.goal_g, g);
        }
    }
    queue_improved<KW>(a, st, f0, w, improved && local, slot, ck, g, h, m, lp, remote_in);
    if (SH && P.n_shards > 1) {
        const bool remote = valid && !local && lowered;
        Remote<KW> rec;
#pragma unroll
        for (int k = 0; k < KW; k++)
            rec.key[k] = ck[k];
        rec.g = g;
        rec.h = h;
        rec.pmask = m;
        rec.flags = 0;
        Remote<KW> *ob = (Remote<KW> *)a.outbox;
        for (int d = 0; d < P.n_shards; d++)
            ring_append(remote && owner == d, &a.x->w[d], &a.x->r_pub[d], ob + (size_t)d * a.outbox_cap, a.outbox_cap,
                        rec, &st->ovf_out);
    }
}


// select: account the previous step, then cut the next batch from the lowest
// bucket holding entries below the best goal (PAStar::check_stop's
// termination, PAStar.cpp:480-547: the goal is accepted once no open node has
// f below its g).  Run by one whole block of kBlock threads: as its own
// launch (sharded search, where the exchange sits between expand and
// select) or as the tail of the last expand block (one shard).
// The control words select needs that the caller has already loaded (the
// expand kernel reads them at its start anyway).
struct SelView {
    unsigned long long n_batch, kmax, kmin, table_slots, maxch;
    int batch_b, batch_nb, band_log2, f0, timing, depth;
};

__device__ __forceinline__ SelView load_view(const Ctl *ctl)
{
    SelView v;
    v.n_batch = ctl->n_batch;
    v.kmax = ctl->kmax;
    v.kmin = ctl->kmin;
    v.table_slots = ctl->table_slots;
    v.maxch = ctl->maxch;
    v.batch_b = ctl->batch_b;
    v.batch_nb = ctl->batch_nb;
    v.depth = ctl->depth;
    v.band_log2 = ctl->band_log2;
    v.f0 = ctl->f0;
    v.timing = ctl->timing;
    return v;
}

// Requires ctl->status == 0 on entry.  X: the sharded search (a.x set): its
// window, backpressure and insert-side counters compile out of the one-shard
// search's fused select.
template <bool X>
__device__ __forceinline__ void select_block(const SearchArgs &a, const SelView &v)
{
    Ctl *ctl = a.ctl;
    StepStats *st = a.stats;
    const int tid = threadIdx.x;
    constexpr int kWin = kBlock / kSub;  // buckets per scan window
    static_assert(kStatRows == 64, "one wave sums the stat rows");
    static_assert(kWin >= kWide, "the first window covers a batch's buckets");
    static_assert(kRanges == 128 && kSub % 2 == 0, "one wave cuts the batch, two ranges per lane");
    __shared__ int found, found2, goal_s, cur_s, fail_s, fault_s, low_s, gmin_s;
    __shared__ unsigned long long claimed_b_s;
    __shared__ unsigned long long wv[kBlock], rv[kBlock];
    __shared__ unsigned long long sums[kStFields], ovf[3];
    const bool prof = v.timing & 2;
    unsigned long long tp0 = prof ? device_clock() : 0, tp;
#define PHASE(k)                                      \
    if (prof && tid == 0) {                           \
        tp = device_clock();                          \
        ctl->phase_ticks[k] += tp - tp0;              \
        tp0 = tp;                                     \
    }
    const int w = v.band_log2, f0 = v.f0;
    const int b_win = v.batch_b;

    // Phase 1, one round trip: the step's statistics, the goal, cur_b, the
    // running totals, and the cursors of the kWin buckets from the last
    // batch's first bucket (children never fall below their parent's bucket,
    // f being monotone under the consistent HPair heuristic; entries from
    // other shards can, and lower cur_b, which the scan below then starts
    // from)
    unsigned long long acc[6];
    if (tid == 0) {
        acc[0] = ctl->expanded;
        acc[1] = ctl->reopen;
        acc[2] = ctl->generated;
        acc[3] = ctl->claimed;
        acc[4] = ctl->dropped;
        acc[5] = ctl->parents;
    }
    {
        const int bb = b_win + tid / kSub, sq = tid % kSub;
        wv[tid] = bb < kBuckets ? ld_agent(&a.q->W[bb][sq]) : 0;
        rv[tid] = bb < kBuckets ? ld_agent(&a.q->R[bb][sq]) : 0;
    }
    if (tid < kStatRows) {
        unsigned long long sv[kStFields];
#pragma unroll
        for (int f = 0; f < kStFields; f++)
            sv[f] = ld_agent(&st->row[tid][f]);
#pragma unroll
        for (int f = 0; f < kStFields; f++)
            sv[f] = wave_sum(sv[f]);
        if (tid == 0) {
#pragma unroll
            for (int f = 0; f < kStFields; f++)
                sums[f] = sv[f];
        }
    } else if (tid == kStatRows) {
        goal_s = ld_agent(a.goal_g);
    } else if (tid == kStatRows + 1) {
        cur_s = ld_agent(&ctl->cur_b);
    } else if (tid >= kStatRows + 2 && tid < kStatRows + 5) {
        const unsigned long long *o[3] = {&st->ovf_near, &st->ovf_far, &st->ovf_out};
        ovf[tid - kStatRows - 2] = ld_agent(o[tid - kStatRows - 2]);
    } else if (tid == kStatRows + 5) {
        found = kBuckets;
        found2 = kBuckets;
    } else if (tid == kStatRows + 6) {
        fault_s = ld_agent(&ctl->fault);
    } else if (tid == kStatRows + 7) {
        low_s = ld_agent(&ctl->low_b) < kBuckets ? atomicExch(&ctl->low_b, kBuckets) : kBuckets;
        claimed_b_s = X ? a.x->claimed_b : 0;
        gmin_s = X ? ld_agent(&a.x->gmin_b) : kBuckets;
    }
    __syncthreads();
    PHASE(0)
    if (tid == 0) {
        const unsigned long long claimed = acc[3] + sums[kStClaimed];
        ctl->expanded = acc[0] + sums[kStExpanded];
        ctl->reopen = acc[1] + sums[kStReopen];
        ctl->generated = acc[2] + sums[kStGenerated];
        ctl->claimed = claimed;
        ctl->dropped = acc[4] + sums[kStDropped];
        if (sums[kStPartQueued] | sums[kStPartTaken]) {  // (partial expansion only: read-modify-write off the common path)
            ctl->part_queued += sums[kStPartQueued];
            ctl->part_taken += sums[kStPartTaken];
        }
        ctl->parents = acc[5] + v.n_batch;
        int fm = fail_bits(ovf[0], ovf[1], sums[kStOvfTable], ovf[2]);
        if ((claimed + claimed_b_s) * 10 > v.table_slots * 7)
            fm |= kFailTable;
        if (fm) {
            atomicOr(&ctl->fail_mask, fm);
            ctl->status = 2;
        }
        if (fault_s) {  // a bounded device wait ran out: the search's state is no longer exact
            ctl->fault_sites = fault_s;
            ctl->status = 4;
        }
        fail_s = fm | fault_s;
    }
    const int goal = goal_s;
    const int limit = goal == kIntMax ? kBuckets - 1 : bucket_of(goal, f0, w);
    // Sharded search: a batch is cut only from the kWide buckets above the
    // lowest live bucket of ALL shards (as of their last select; every
    // shard's header carries its own).  A shard whose own buckets lie higher
    // waits: what it would expand from them now, it would mostly expand
    // again once the cheaper paths through the other shards' lower buckets
    // arrive (syn8x400 at 8 shards: 27-46 M expansions for 5.8 M without
    // the window).  limit still decides whether the shard has work at all.
    const int xwin = X ? ctl->xwindow : kBuckets;
    const int limit_take = (X && gmin_s < kBuckets && gmin_s + xwin - 1 < limit) ? gmin_s + xwin - 1 : limit;
    const int start_c = cur_s < b_win ? cur_s : b_win;
    const int start = low_s < start_c ? low_s : start_c;
    if (start == b_win) {
        const int bb = b_win + tid / kSub;
        if (bb <= limit && wv[tid] > rv[tid])
            atomicMin(&found, bb);
    }
    __syncthreads();
    PHASE(1)
    // every wave decides on phase 2 from this value; phase 2 writes its own
    // found2, so a fast wave's scan cannot change a slow wave's decision
    const int found1 = found;
    if (fail_s)
        return;
    unsigned long long *z = (unsigned long long *)st;
    for (int k = tid; k < (int)(sizeof(StepStats) / 8); k += blockDim.x)
        st_agent(&z[k], 0ull);
    if (ctl->debug && tid < kSub) {  // diagnostics: entries below the scan start?
        for (int bb = 0; bb < start; bb++) {
            const unsigned long long wq = ld_agent(&a.q->W[bb][tid]), rq = ld_agent(&a.q->R[bb][tid]);
            if (wq > rq) {
                if (atomicAdd(&ctl->dbg_hits, 1) == 0) {
                    ctl->dbg_bucket = bb;
                    ctl->dbg_cur = cur_s;
                    ctl->dbg_win = b_win;
                    ctl->dbg_step = (int)ctl->steps;
                    ctl->dbg_w = wq;
                    ctl->dbg_r = rq;
                }
                break;
            }
        }
    }
    // Phase 2 (rare): scan on past the window, or from a lower cur_b
    int bfound = found1;
    if (found1 == kBuckets) {
        for (int b0 = start == b_win ? b_win + kWin : start; b0 <= limit; b0 += kWin) {
            const int b = b0 + tid / kSub, sq = tid % kSub;
            if (b <= limit && ld_agent(&a.q->W[b][sq]) > ld_agent(&a.q->R[b][sq]))
                atomicMin(&found2, b);
            __syncthreads();
            bfound = found2;
            __syncthreads();  // every wave has read it before the next round writes it
            if (bfound < kBuckets)
                break;
        }
    }
    const int b = bfound;
    if (a.trace && tid == 0) {
        const long long stp = ctl->steps;
        if (stp < kTraceSteps) {
            int *t = a.trace + stp * 8;
            t[0] = (int)stp;
            t[1] = cur_s;
            t[2] = b_win;
            t[3] = start;
            t[4] = limit;
            t[5] = b;
        }
    }
    if (b < kBuckets && b > limit_take) {
        // live entries, but above the shards' common window: an idle step
        if (tid == 0) {
            ctl->n_batch = 0;
            ctl->has_work = 1;
            ctl->low_found = b;
            st_agent(&ctl->cur_b, b);
            const long long steps = ctl->steps + 1;
            ctl->steps = steps;
            if (ctl->max_steps && steps >= ctl->max_steps)
                ctl->status = 3;
        }
        return;
    }
    if (b >= kBuckets) {
        if (tid == 0) {
            ctl->n_batch = 0;
            ctl->has_work = 0;
            ctl->low_found = kBuckets;
            const long long steps = ctl->steps + 1;
            ctl->steps = steps;
            // one shard: done; the sharded protocol decides on the host
            // from every shard's has_work
            int status = ctl->fuse ? 1 : 0;
            if (ctl->max_steps && steps >= ctl->max_steps && !status)
                status = 3;
            if (status)
                ctl->status = status;
        }
        return;
    }
    PHASE(2)
    // Cut the batch: ranges r = (bucket b + r / kSub, sub-queue r % kSub),
    // r = 0..127, in order, at most kmax entries; bucket k > 0 joins only
    // while the buckets before it hold fewer than kmin entries (a thin
    // batch pulls the next buckets, up to kWide).  One wave, two
    // consecutive ranges per lane, a wave prefix sum; cursors already read
    // in phase 1 are reused.
    if (tid < 64) {
        unsigned long long rs[2], av[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int r = 2 * tid + j;
            const int bb = b + r / kSub, sq = r % kSub;
            const bool in = bb <= limit_take && bb < kBuckets;
            unsigned long long rsv = 0, wr = 0;
            if (in) {
                if (start == b_win && bb < b_win + kWin) {
                    const int wi = (bb - b_win) * kSub + sq;
                    rsv = rv[wi];
                    wr = wv[wi];
                } else {
                    rsv = ld_agent(&a.q->R[bb][sq]);
                    wr = ld_agent(&a.q->W[bb][sq]);
                }
            }
            rs[j] = rsv;
            av[j] = wr - rsv;
        }
        const unsigned long long s2 = av[0] + av[1];
        unsigned long long inc = s2;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(inc, o);
            if (tid >= o)
                inc += y;
        }
        const unsigned long long ex0 = inc - s2, ex1 = ex0 + av[0];
        const int k = (2 * tid) / kSub;                       // bucket offset of both ranges
        const unsigned long long bstart = __shfl(ex0, k * (kSub / 2));  // entries before bucket k
        // (sharded: a shard holds about 1 / n_shards of a thin bucket)
        const unsigned long long kmin = X ? v.kmin / (unsigned long long)ctl->n_shards : v.kmin;
        const bool incl = k == 0 || bstart < kmin;
        const int n_incl = __popcll(__ballot(incl && (tid % (kSub / 2)) == 0 && b + k <= limit_take));
        // sharded: no more parents than the outbox rings can take children
        // of (a ring holds what the exchange has not carried off yet): the
        // least free ring, spread over the other shards, at half the masks
        // a parent can have (an overflow past this estimate restarts the
        // search with larger rings)
        unsigned long long kmax = v.kmax;
        if (X && ctl->n_shards > 1) {
            unsigned long long free_min = ~0ull;
            for (int d = 0; d < ctl->n_shards; d++) {
                if (d == a.P->shard)
                    continue;
                const unsigned long long used = ld_agent(&a.x->w[d]) - ld_agent(&a.x->r_pub[d]);
                const unsigned long long fr = used < a.outbox_cap ? a.outbox_cap - used : 0;
                free_min = fr < free_min ? fr : free_min;
            }
            const unsigned long long masks = (1ull << a.P->n) - 1;
            const unsigned long long lim = free_min * (unsigned long long)(ctl->n_shards - 1) * 2 / masks;
            kmax = lim < kmax ? lim : kmax;
        }
        const unsigned long long t0 = incl ? (ex0 < kmax ? (av[0] < kmax - ex0 ? av[0] : kmax - ex0) : 0) : 0;
        const unsigned long long t1 = incl ? (ex1 < kmax ? (av[1] < kmax - ex1 ? av[1] : kmax - ex1) : 0) : 0;
        const unsigned long long total = wave_sum(t0 + t1);
        const unsigned long long p0 = incl ? (ex0 < kmax ? ex0 : kmax) : total;
        const unsigned long long p1 = incl ? (ex1 < kmax ? ex1 : kmax) : total;
        const int r0 = 2 * tid;
        ctl->b_start[r0] = t0 ? rs[0] : 0;
        ctl->b_start[r0 + 1] = t1 ? rs[1] : 0;
        ctl->b_prefix[r0] = p0;
        ctl->b_prefix[r0 + 1] = p1;
        if (t0)
            st_agent(&a.q->R[b + r0 / kSub][r0 % kSub], rs[0] + t0);
        if (t1)
            st_agent(&a.q->R[b + (r0 + 1) / kSub][(r0 + 1) % kSub], rs[1] + t1);
        if (tid == 0) {
            ctl->b_prefix[kRanges] = total;
            ctl->n_batch = total;
            ctl->batch_b = b;
            ctl->batch_nb = n_incl > 0 ? n_incl : 1;
            st_agent(&ctl->cur_b, b);
            ctl->has_work = 1;
            ctl->low_found = b;
            const long long steps = ctl->steps + 1;
            ctl->steps = steps;
            if (ctl->max_steps && steps >= ctl->max_steps)
                ctl->status = 3;
        }
    }
    PHASE(3)
#undef PHASE
}

__global__ __launch_bounds__(kBlock) void select_kernel(SearchArgs a)
{
    if (!a.ctl->status) {
        if (a.x)
            select_block<true>(a, load_view(a.ctl));
        else
            select_block<false>(a, load_view(a.ctl));
    }
    if (!a.x)
        return;
    // Sharded search: what this shard tells the others about step a.step,
    // sampled here once, by one thread, before the step's expansion: the
    // pack kernel copies it into every block header, whatever else changes
    // meanwhile (the side stream may set the status, the next step's select
    // may run beside the pack).
    __syncthreads();
    if (threadIdx.x == 0) {
        const Ctl *ctl = a.ctl;
        const int status = ld_agent(&ctl->status);
        XState::StepInfo si;
        si.n_batch = status == 0 ? ctl->n_batch : 0;
        si.has_work = status == 0 && ctl->has_work;
        si.low_b = si.has_work ? ctl->low_found : kBuckets;
        si.goal = ld_agent(a.goal_g);
        int fl = 0;
        if (status == 2)
            fl |= ctl->fail_mask & 0xff ? ctl->fail_mask & 0xff : kFailTable;
        else if (status == 3)
            fl |= 0x100;
        else if (status == 4)
            fl |= 0x200;
        fl |= ld_agent(&a.x->fail_b);  // the insert kernel's overflows (folded by the pack kernel)
        if (ld_agent(&ctl->fault))
            fl |= 0x200;
        si.fail = fl;
        a.x->info[a.step & (kXSlots - 1)] = si;
    }
}

// A batch parent's slot words: key, best, aux.
template <int KW>
struct PSlot {
    uint64_t key[KW];
    uint64_t best, aux;
};

template <int KW>
__device__ __forceinline__ PSlot<KW> load_pslot(const uint64_t *__restrict__ table, uint32_t slot)
{
    constexpr int SW = slot_words<KW>();
    const uint64_t *s = table + (uint64_t)slot * SW;
    PSlot<KW> o;
#pragma unroll
    for (int k = 0; k < KW; k++)
        o.key[k] = s[k];
    o.best = s[KW];
    o.aux = s[KW + 1];
    return o;
}

// Range of batch entry i (wave-uniform call): the batch's range prefix is
// held two entries per lane (pf_lo = prefix[2 lane], pf_hi = prefix[2 lane +
// 1], constant for the launch), so "the last range r with prefix[r] <= i" is
// a count of set ballot bits, for each of the wave's npw entries in turn --
// no chain of dependent LDS reads.  Empty ranges repeat a prefix value and
// are skipped the same way the binary search skips them.
__device__ __forceinline__ int batch_range(uint32_t pf_lo, uint32_t pf_hi, unsigned long long i, int npw, int lpn)
{
    const int lane = lane_id();
    int r = 0;
    for (int g = 0; g < npw; g++) {
        const unsigned long long ig = bcast_lane(i, g * lpn);
        const int cnt = __popcll(__ballot(pf_lo <= ig)) + __popcll(__ballot(pf_hi <= ig));
        if (lane / lpn == g)
            r = cnt - 1;
    }
    return r;
}

// Entry i of the current batch, in range r.
__device__ __forceinline__ Entry batch_entry_at(const SearchArgs &a, const SelView &v, const uint32_t *prefix,
                                                const unsigned long long *bstart, unsigned long long i, int r)
{
    const int bb = v.batch_b + r / kSub, sq = r % kSub;
    const unsigned long long p = bstart[r] + (i - prefix[r]);
    const uint32_t c = a.chunk_tab[((size_t)bb * kSub + sq) * v.maxch + (p >> kChunkLog2)];
    return a.pool[(size_t)(c - 1) * kChunk + (p & (kChunk - 1))];
}


// ---------------------------------------------------------------------------
// The dive (N = 4, 1-word keys): several continuation levels per memory round
// trip.  A block-local chain is bound by latency: a level costs two dependent
// memory round trips (the parent's pair cells, then the children's claim or
// atomicMin) and a pass over one wave's worth of instructions.  When a level's
// few parents sit close together, every node within kDiveW steps of them lies
// in one small window of the lattice: the window's pair cells ((kDiveW + 1)^2
// per pair) come in ONE gather, the next kDiveW levels are then expanded out of
// LDS alone -- a child continues when it improves on what the dive itself has
// seen of its node (a direct-mapped table over the window's relative
// coordinates) and its f stays in the batch's buckets -- and every child
// generated on the way is relaxed into the node table afterwards, all at
// once.  Only then is a continued node known to have been an improvement
// (its own relax says so): one that was not has been expanded for nothing,
// which costs work but never a wrong g (every g written is the cost of a
// real path).
// ---------------------------------------------------------------------------
#ifndef PASTAR_DIVE
#define PASTAR_DIVE 1
#endif
#ifndef PASTAR_SPLIT_COST
#define PASTAR_SPLIT_COST 1
#endif
#ifndef PASTAR_DIVE_W
#define PASTAR_DIVE_W 6
#endif
constexpr int kDiveW = PASTAR_DIVE_W;               // levels per dive; nodes up to kDiveW steps past the window's origin
static_assert(kDiveW <= 8, "4-bit window coordinates");
constexpr int kDiveWS = kDiveW + 1;
constexpr int kDiveCells = kDiveWS * kDiveWS;
constexpr int kDiveNodes = kDiveWS * kDiveWS * kDiveWS * kDiveWS;
#ifndef PASTAR_DIVE_SPREAD
#define PASTAR_DIVE_SPREAD (kDiveW - 2)
#endif
constexpr int kDiveMaxSpread = PASTAR_DIVE_SPREAD;  // start nodes at most this far apart
constexpr int kDiveFront = 4;           // nodes one dive level expands (the lane groups of one wave)
constexpr int kDiveRecs = 384;          // children one dive generates at most
struct DiveRec {
    uint64_t key;
    int g, h, info;  // info: parent mask | kDiveCont
};
constexpr int kDiveCont = 0x100;        // expanded inside the dive

// expand every entry of the batch (worker_inner's dequeue, closed check and
// getNeigh, PAStar.cpp:320-401) and relax its neighbours into the node table
// (PAStar::enqueue + conditional_enqueue, :219-237).
// SH = false: instantiated for the one-shard search, whose launches never
// route a child to another shard (the sharded protocol launches SH = true)
template <int N, int KW, bool SH = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(expand_waves_per_eu(N, KW)))) void expand_kernel(SearchArgs a)
{
    constexpr int SW = slot_words<KW>();
    // child-slot prefetch: fixed N (the rounds of 64 children are static)
    // and 1- or 2-word keys
    constexpr bool kPf = N > 0 && KW <= 2;
    // slots of the first probe line prefetched per child: the whole line
    // for 1-word keys at N <= 5 (a collision then costs no round trip; a
    // wave of 15-31 children almost always has one), one slot otherwise
    // (register budget)
    constexpr int kPfSlots = (KW == 1 && N > 0 && N <= 5) ? line_slots<KW>() : 1;
    Ctl *ctl = a.ctl;
    const DevProblem &Pg = *a.P;
    // the fields the level loop reads, in registers (KConst)
    const KConst<N, KW> P = load_kconst<N, KW>(Pg);
    const int n = N ? N : Pg.n;
    const int lpn = (1 << n) < 64 ? (1 << n) : 64;
    const int npw = 64 / lpn;
    const int per_block = kWaves * npw;
    const int status = ctl->status;
    const SelView view = load_view(ctl);
    if (status)
        return;
    const unsigned long long nb = view.n_batch;
    // blocks with work; with an empty batch block 0 still runs the tail
    // (the fused select of the first step)
    // a batch of at most one entry per block (N = 4): each block takes one
    // parent and starts its chain with the two-level pass below
    const bool single = N == 4 && KW == 1 && nb > 0 && nb <= gridDim.x && (!SH || P.n_shards == 1) && view.depth > 2;
    const unsigned long long eff_per_block = single ? 1 : per_block;
    const unsigned long long nact =
        nb ? ((nb + eff_per_block - 1) / eff_per_block < gridDim.x ? (nb + eff_per_block - 1) / eff_per_block
                                                                   : gridDim.x)
           : 1;
    if (blockIdx.x >= nact)
        return;  // blocks beyond the batch leave at once
    const bool timing = (view.timing & 1) && nb;
    if (timing && blockIdx.x < kArrive && threadIdx.x == 0)
        __hip_atomic_store(&a.stamps[blockIdx.x], device_clock(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int npairs = N ? N * (N - 1) / 2 : Pg.npairs;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int group = lane / lpn, glane = lane % lpn;
    const int leader_lane = group * lpn;
    // one child round (2^N <= 64): this lane's child mask is glane for the
    // whole launch, so its key increment is computed once
    constexpr bool kOneRound = N > 0 && (1 << N) <= 64;
    uint64_t kinc[KW];
    {
        const uint64_t zero[KW] = {};
        child_key<N, KW>(P, n, zero, kOneRound ? glane : 0, kinc);
    }
    // two continuation levels per pass for a one-parent level (N = 4: the
    // parent's 15 children and their 15 x 15 children on the block's 16
    // groups); the key increment of this group's child mask
    constexpr bool kTwoLevel = N == 4 && KW == 1;
    constexpr bool kDive = PASTAR_DIVE && N == 4 && KW == 1;  // (the two-level pass when built without)
    uint64_t kinc_grp[KW];
    {
        const uint64_t zero[KW] = {};
        child_key<N, KW>(P, n, zero, kTwoLevel ? wave * npw + group : 0, kinc_grp);
    }
    __shared__ int2 terms_all[kWaves][terms_per_wave(N)];
    // wide fan-outs with one parent per wave: a child's cost from split tables (device.hpp, SplitCost)
    constexpr bool kSplit = PASTAR_SPLIT_COST && N >= 7;
    __shared__ int2 split_all[kSplit ? kWaves : 1][kSplit ? SplitCost<N ? N : 8>::kEntries : 1];
    // batch offsets fit 32 bits (batch_nodes <= 2^30, checked on the host)
    __shared__ uint32_t prefix[kRanges + 1];
    __shared__ unsigned long long bstart[kRanges];
    __shared__ PairConst pc[kMaxPairs];
    int2 *terms = &terms_all[wave][group * 4 * npairs];
    // one round trip: the batch's ranges and the pair constants
    for (int r = threadIdx.x; r <= kRanges; r += blockDim.x) {
        prefix[r] = (uint32_t)ctl->b_prefix[r];
        if (r < kRanges)
            bstart[r] = ctl->b_start[r];
    }
    stage_pairs(Pg, pc);
    // block 0's phase timers (diagnostics, PASTAR_TIMING_MASK bit 2): built
    // only with -DPASTAR_PHASE_TIMERS, since their 64-bit clocks are held in
    // scalar registers through the whole level loop
#ifdef PASTAR_PHASE_TIMERS
    const bool bprof = (view.timing & 4) && timing && blockIdx.x == 0 && threadIdx.x == 0;
    unsigned long long bt0 = bprof ? device_clock() : 0, bt;
#define BPHASE(k)                                     \
    if (bprof) {                                      \
        bt = device_clock();                          \
        ctl->body_ticks[k] += bt - bt0;               \
        bt0 = bt;                                     \
    }
#else
    constexpr bool bprof = false;
#define BPHASE(k)
#endif
    StepStats *st = a.stats;
    const int w = view.band_log2, f0 = view.f0;
    const int goal_now = *(volatile int *)a.goal_g, prune_f = ctl->prune_f;
    const int bound = goal_now < prune_f ? goal_now : prune_f;
    // per-lane statistics of one launch (32-bit: at most a few million)
    unsigned expanded = 0, reopen = 0, generated = 0, claimed = 0, ovf = 0, stale = 0, part_q = 0, part_t = 0;
    const int masks = 1 << n;
    // upper edge of the batch's buckets: improved children below it continue
    // in this launch (block-local continuation)
    const int f_limit = f0 + (int)(((long long)view.batch_b + view.batch_nb) << w);
    // partial expansion (wide fan-outs: several child rounds per parent): a
    // child with f at or past `cutoff` is not generated now; its parent goes
    // back to the open list under the lowest such f and generates the rest
    // when it is taken again.  Most parents are expanded in the search's last
    // buckets, and their costlier children never come up before the search
    // ends: no probe, no table slot, no queue entry for them.  (A batch that
    // reaches the last bucket, which also holds everything above, expands in
    // full: the re-queued parent must land past its batch.)
    constexpr bool kPartial = N == 0 || N >= 7;
    const int partial_k = kPartial ? ctl->partial_k : -1;
    const int partial_ahead = kPartial ? ctl->partial_ahead : 0;
    const int partial_two = kPartial ? ctl->partial_two : 0;
    const int cutoff = (partial_k >= 0 && view.batch_b + view.batch_nb + partial_k < kBuckets - 1)
                           ? f_limit + (int)((long long)partial_k << w)
                           : kIntMax;
    __syncthreads();
    BPHASE(0)
    // expand one parent per lane group: entry -> staleness / closed check ->
    // pair terms in LDS -> one child mask per lane -> relax + route.  Every
    // thread of the block calls it (it holds a block barrier).
    // `local`: a continuation entry (parent fields carried in LDS); else a
    // batch entry {slot, f} whose parent is read from the table
    auto process = [&](bool ok, const Entry e, const PSlot<KW> &ps, const LEntry<KW> &le, bool local,
                       const LocalPush<KW> &lp) {
        Parent<N, KW> par_;
        par_.g = 0;
        par_.pmask = 0;
        par_.blocked = 0;
#pragma unroll
        for (int k = 0; k < KW; k++)
            par_.key[k] = 0;
        uint64_t lbest = 0, laux = 0;
        int resume = 0;            // partial expansion: children below this f were generated before
        int pend_f = kIntMax;      // lowest f among the children left for later
        int cut = cutoff;          // (a parent taken again generates all it has left: at most two passes)
        if (ok && local) {
#pragma unroll
            for (int k = 0; k < KW; k++)
                par_.key[k] = le.key[k];
            par_.g = le.g;
            par_.pmask = le.pmask;
            ok = le.g + le.h < bound;
            // current-ness and the closed mark are settled after the terms
            // are staged (these loads overlap the pair-table gathers)
            const uint64_t *s = a.table + (uint64_t)le.slot * SW;
            lbest = s[KW];
            laux = s[KW + 1];
        } else if (ok) {
            // the slot words were loaded by the caller, a chunk ahead
#pragma unroll
            for (int k = 0; k < KW; k++)
                par_.key[k] = ps.key[k];
            const uint64_t best = ps.best;
            const uint64_t aux = ps.aux;
            const int h = (int)(aux >> 32);
            par_.g = (int)(best >> 32);
            par_.pmask = (int)(uint32_t)best;
            const bool part = kPartial && e.f < 0;
            const int ef = entry_f(e);
            int verdict;
            if (part) {
                // the rest of a partially expanded parent, generated under
                // the node's best g as of now; not a new expansion.  Always
                // current: had the node improved since it was queued, the
                // improvement's own entry expands it from the start (and
                // queues its own rest), so this one only repeats part of
                // that; nothing tells the two apart cheaply, and nothing
                // needs to (relaxations are idempotent)
                verdict = ef < bound ? 1 : 0;
                resume = ef;
                if (partial_two == 1)
                    cut = kIntMax;
                else if (partial_two == 2 && cutoff != kIntMax) {
                    // each pass reaches as far past the batch as the last one
                    // left off past the parent's own f
                    const long long far = (long long)f_limit + (ef - (par_.g + h));
                    cut = far > cutoff ? (far < kIntMax ? (int)far : kIntMax) : cutoff;
                }
            } else {
                // an entry is current iff its f is the node's f under the
                // best g found so far; improvements are strict, so a current
                // entry is unique and the closed mark needs no atomic
                verdict = ((par_.g + h == ef) && ef < bound) ? 1 : 0;
                if (verdict && glane == 0) {
                    int *closed = (int *)(a.table + (uint64_t)e.slot * SW + KW + 1);
                    verdict = (int)(uint32_t)aux != kIntMax ? 2 : 1;
                    *closed = par_.g;
                }
            }
            verdict = group_verdict(verdict, leader_lane);
            ok = verdict != 0;
            if (glane == 0) {
                expanded += ok && !part;
                part_t += ok && part;
                reopen += verdict == 2;
                stale += !ok;
            }
        }
        BPHASE(1)
        // first-probe slot words of the first 64 children, read before the
        // pair terms are staged (one memory round trip less per level)
        SlotWords<KW, kPfSlots> pf{};
        bool has_pf = false;
        if (ok) {
            decode_key<N, KW>(P, n, par_.key, par_.pos);
#pragma unroll
            for (int i = 0; i < Parent<N, KW>::NMAX; i++)
                if ((N || i < n) && par_.pos[i] >= P.len[i])
                    par_.blocked |= 1 << i;
            // the slot prefetch is issued right after the gathers (before
            // their wait), so waiting for the gathers never waits for it
            auto prefetch = [&] {
                if constexpr (kPf) {
                    // issued by every lane (the slot index is masked into
                    // the table), so the wait counts do not depend on it
                    const int m = glane;
                    uint64_t ck[KW];
                    if constexpr (kOneRound) {
#pragma unroll
                        for (int k = 0; k < KW; k++)
                            ck[k] = par_.key[k] + kinc[k];
                    } else {
                        child_key<N, KW>(P, n, par_.key, m, ck);
                    }
                    pf = slot_prefetch<KW, kPfSlots>(a.table, a.cap_mask, ck);
                    has_pf = m >= 1 && m < masks && !(m & par_.blocked);
                }
            };
            if constexpr (N > 0) {
                stage_terms_fixed<N, KW>(P, pc, par_, terms, glane, prefetch);
            } else {
                prefetch();
                stage_terms<N, KW>(P, n, npairs, pc, par_, terms, glane, lpn);
            }
        }
        BPHASE(6)
        if (local) {  // uniform: a whole level is local or not
            // current iff nobody has improved the node since it was queued
            // (a larger or unset best is this block's own update, not yet
            // landed: the barriers here do not wait for global memory)
            bool cur = ok && (uint32_t)(lbest >> 32) >= (uint32_t)par_.g;
            int verdict = cur ? 1 : 0;
            if (cur && glane == 0) {
                int *closed = (int *)(a.table + (uint64_t)le.slot * SW + KW + 1);
                verdict = (int)(uint32_t)laux != kIntMax ? 2 : 1;
                *closed = par_.g;
            }
            verdict = group_verdict(verdict, leader_lane);
            if (glane == 0) {
                expanded += verdict != 0;
                reopen += verdict == 2;
                stale += ok && verdict == 0;
            }
            ok = verdict != 0;
        }
        // a wave reads only the terms it staged itself (terms_all[wave]):
        // its own LDS writes landing is enough, no block barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (kSplit) {
            // (one parent per wave: the wave's tables, built from its terms)
            if (__ballot(ok)) {  // uniform
                split_cost_build<N>(terms, split_all[wave], lane);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        BPHASE(2)
        // several rounds of 64 masks: the key of this lane's child is the
        // parent's plus the increments of the mask's low six bits, the lane's
        // and the same in every round, plus those of its high bits, the
        // round's and the same on every lane
        uint64_t klane[KW];
        if constexpr (!kOneRound && N > 0)
            child_key<N, KW>(P, n, par_.key, glane, klane);
        for (int r = 0; r * lpn < masks; r++) {
            const int m = r * lpn + glane;
            bool valid = ok && m >= 1 && m < masks && !(m & par_.blocked);
            int g = 0, h = 0, owner = P.shard;
            uint64_t ck[KW];
#pragma unroll
            for (int k = 0; k < KW; k++)
                ck[k] = 0;
            if (valid) {
                int2 dc;
                if constexpr (kSplit)
                    dc = split_cost<N>(split_all[wave], m);
                else
                    dc = child_cost<N>(Pg, npairs, terms, m);
                g = par_.g + dc.x;
                h = dc.y;
                const int f = g + h;
                if (kPartial && (f < resume || f >= cut)) {
                    valid = false;
                    if (f >= cut && f < bound)
                        pend_f = f < pend_f ? f : pend_f;
                } else {
                    generated++;
                    if (f >= bound)
                        valid = false;
                }
            }
            if (valid) {
                if constexpr (kOneRound) {
#pragma unroll
                    for (int k = 0; k < KW; k++)
                        ck[k] = par_.key[k] + kinc[k];
                } else if constexpr (N > 0) {
                    const uint64_t zero[KW] = {};
                    uint64_t rinc[KW];
                    child_key<N, KW>(P, n, zero, r * lpn, rinc);  // (uniform)
#pragma unroll
                    for (int k = 0; k < KW; k++)
                        ck[k] = klane[k] + rinc[k];
                } else {
                    child_key<N, KW>(P, n, par_.key, m, ck);
                }
                if (SH && P.n_shards > 1) {
                    int cp[Parent<N, KW>::NMAX];
#pragma unroll
                    for (int i = 0; i < Parent<N, KW>::NMAX; i++)
                        cp[i] = par_.pos[i] + ((m >> i) & 1);
                    owner = owner_dev<Parent<N, KW>::NMAX>(P, n, cp, P.n_shards);
                }
            }
            BPHASE(8)
            route_child<KW, kPfSlots, SH>(a, P, st, f0, w, valid, owner == P.shard, owner, ck, g, h, m, claimed, ovf, lp,
                                      false, has_pf && r == 0, pf);
            BPHASE(9)
        }
        if constexpr (kPartial) {
            if (partial_k >= 0) {  // uniform
                // the parent again, under the lowest f it has left
                // (one parent per wave wherever this is compiled in: a DPP reduction, no LDS round trips)
                pend_f = wave_min_i32(pend_f);
                // (queued `partial_ahead` buckets before its first child is
                // due, but past this batch: the children are then in their
                // buckets before those are cut, not after; the entry keeps
                // the f the parent resumes from)
                const bool again = ok && glane == 0 && pend_f != kIntMax;
                part_q += again;
                const Entry pe = {local ? le.slot : e.slot, pend_f | kPartialBit};
                int pb = bucket_of(pend_f, f0, w) - partial_ahead;
                pb = pb < view.batch_b + view.batch_nb ? view.batch_b + view.batch_nb : pb;
                open_append(a, lp, again, pb, pe, st, false);
            }
        }
        BPHASE(7)
    };

#ifdef PASTAR_PHASE_TIMERS
    const unsigned long long blk_t0 = device_clock();
    unsigned blk_levels = 1, blk_rounds = 0;
#define BLK_COUNT(lv, rd) \
    {                     \
        blk_levels += lv; \
        blk_rounds += rd; \
    }
#else
#define BLK_COUNT(lv, rd)
#endif
    // level 0: this block's share of the batch; levels 1..depth-1: the
    // children it queued in LDS (double-buffered)
    // continuation only while the batch leaves most of the chip idle (with
    // a full grid, deep chains in a few blocks would only stretch the
    // launch); a level may take R rounds of the block's width, R chosen so
    // that the blocks together run about kDeepBlocks block-rounds per level
    // (a round costs ceil(2^N / 64) child passes)
    const int passes = masks > 64 ? masks / 64 : 1;
    const unsigned long long rounds = (unsigned long long)ctl->deep_blocks / (nact * passes);
    const int depth = rounds >= (unsigned long long)ctl->deep_rounds ? view.depth : 1;
    __shared__ LEntry<KW> lq[2][kLocalCap];
    __shared__ int lq_count[2], out_n;
    __shared__ Entry outq[kOutCap];
    if (threadIdx.x < 2)
        lq_count[threadIdx.x] = 0;
    if (threadIdx.x == 0)
        out_n = 0;
    __syncthreads();
    // one level takes at most `rounds` rounds of the block's width, so a
    // block's chain never outgrows the work of its neighbours
    const int lq_cap = (unsigned long long)per_block * rounds < (unsigned long long)kLocalCap
                           ? per_block * (int)rounds : kLocalCap;
    LocalPush<KW> lp{depth > 1 ? lq[0] : nullptr, &lq_count[0], f_limit, lq_cap, outq, &out_n};
    const LEntry<KW> no_le{};
    // a block walks its chunks of the batch (grid-stride; the grid is about
    // one resident wave of blocks) as a software pipeline: a chunk's parent
    // slots and the next chunk's queue entries are loaded together, so a
    // chunk waits for one memory round trip before staging, not three
    // (entry: chunk table + pool, then the slot)
    const PSlot<KW> no_ps{};
    const uint32_t pf_lo = prefix[2 * lane], pf_hi = prefix[2 * lane + 1];
    if (single) {
        // the block's one batch entry, as a continuation entry of level 1
        // (its current-ness re-checked there; the closing and the counts
        // happen in the pass that expands it)
        if (wave == 0) {
            const unsigned long long node = blockIdx.x;
            const int r = batch_range(pf_lo, pf_hi, node, 1, 64);
            const Entry e = batch_entry_at(a, view, prefix, bstart, node, r);
            const PSlot<KW> ps = load_pslot<KW>(a.table, e.slot);
            if (lane == 0) {
                const int g = (int)(ps.best >> 32), h = (int)(ps.aux >> 32);
                if (g + h == e.f && e.f < bound) {
                    LEntry<KW> le;
#pragma unroll
                    for (int k = 0; k < KW; k++)
                        le.key[k] = ps.key[k];
                    le.slot = e.slot;
                    le.g = g;
                    le.h = h;
                    le.pmask = (int)(uint32_t)ps.best;
                    lq[0][0] = le;
                    lq_count[0] = 1;
                } else {
                    stale++;
                }
            }
        }
    }
    Entry e_nx{0, 0};
    if (!single) {
        const unsigned long long node = (unsigned long long)blockIdx.x * per_block + wave * npw + group;
        const int r = batch_range(pf_lo, pf_hi, node, npw, lpn);
        if (node < nb)
            e_nx = batch_entry_at(a, view, prefix, bstart, node, r);
    }
    for (unsigned long long chunk = blockIdx.x; !single && chunk * per_block < nb; chunk += gridDim.x) {
        const unsigned long long node = chunk * per_block + wave * npw + group;
        const bool ok = node < nb;
        const Entry e = e_nx;
        PSlot<KW> ps = no_ps;
        if (ok)
            ps = load_pslot<KW>(a.table, e.slot);
        const unsigned long long nn = node + (unsigned long long)gridDim.x * per_block;
        const int r = batch_range(pf_lo, pf_hi, nn, npw, lpn);
        if (nn < nb)
            e_nx = batch_entry_at(a, view, prefix, bstart, nn, r);
        process(ok, e, ps, no_le, false, lp);
        BLK_COUNT(0, 1)
    }
    // the continuation queue and the deferred entries are block-wide: one
    // barrier per level, after all of its chunks
    lds_barrier();
    BPHASE(3)
    int cur = 0;
    for (int lvl = 1; lvl < depth; lvl++) {
        const int cnt = lq_count[cur] < lq_cap ? lq_count[cur] : lq_cap;  // read after the level's barrier
        if (cnt == 0)
            break;
#ifdef PASTAR_PHASE_TIMERS
        if ((view.timing & 4) && timing && threadIdx.x == 0)
            atomicAdd(&ctl->blk_stats[cnt == 1 ? 6 : (cnt <= 4 ? 7 : (cnt <= 16 ? 8 : 9))], 1ull);
#endif
        const int nxt = cur ^ 1;
        if (threadIdx.x == 0)
            lq_count[nxt] = 0;
        lds_barrier();
        if constexpr (kDive) {
            // the level's nodes (at most kDiveFront), the window's origin (their
            // componentwise lowest position) and their spread: every wave
            // computes them for itself (no barrier).  Every start node needs a
            // level ahead of it in the window; a level whose nodes lie
            // further apart takes the one-level pass below.
            bool dive = cnt <= kDiveFront && lvl + kDiveW < depth && (!SH || P.n_shards == 1);
            int org[N];
            LEntry<KW> mine{};
            int mpos[N];
            if (dive) {  // uniform
                const int li = lane & (kDiveFront - 1);
                mine = lq[cur][li < cnt ? li : 0];
                const uint64_t mk[KW] = {mine.key[0]};
                decode_key<N, KW>(P, n, mk, mpos);
                int spread = 0;
#pragma unroll
                for (int i = 0; i < N; i++) {
                    int lo = mpos[i], hi = mpos[i];
                    if (cnt > 1) {  // uniform
#pragma unroll
                        for (int o = 1; o < kDiveFront; o <<= 1) {
                            const int yl = __shfl_xor(lo, o), yh = __shfl_xor(hi, o);
                            lo = yl < lo ? yl : lo;
                            hi = yh > hi ? yh : hi;
                        }
                    }
                    org[i] = __builtin_amdgcn_readfirstlane(lo);
                    const int sp = __builtin_amdgcn_readfirstlane(hi) - org[i];
                    spread = sp > spread ? sp : spread;
                }
                dive = spread <= kDiveMaxSpread;
            }
            if (dive) {
                constexpr int NP = N * (N - 1) / 2;
                __shared__ int2 cw[NP][kDiveCells];
                __shared__ int relbest[kDiveNodes];
                __shared__ DiveRec recs[kDiveRecs];
                __shared__ int rec_n, dive_done;
                auto rel_index = [](int rel) {
                    return (((rel & 15) * kDiveWS + ((rel >> 4) & 15)) * kDiveWS + ((rel >> 8) & 15)) * kDiveWS +
                           ((rel >> 12) & 15);
                };
                // ---- the window's pair cells (one gather), the start nodes' slot words
                constexpr int kCT = (NP * kDiveCells + kBlock - 1) / kBlock;
                int2 cell[kCT];
#pragma unroll
                for (int t = 0; t < kCT; t++) {
                    const int ct = threadIdx.x + t * kBlock;
                    cell[t] = make_int2(0, 0);
                    if (ct < NP * kDiveCells) {
                        const int p = ct / kDiveCells, r = ct % kDiveCells, i = r / kDiveWS, j = r % kDiveWS;
                        const PairConst k = pc[p];
                        int ox = 0, oy = 0;
#pragma unroll
                        for (int d = 0; d < N; d++) {
                            if (d == k.x)
                                ox = org[d];
                            if (d == k.y)
                                oy = org[d];
                        }
                        const int ix = ox + i, iy = oy + j;
                        if (ix <= k.lx && iy <= k.ly) {
                            const __attribute__((address_space(1))) int2 *cells =
                                (const __attribute__((address_space(1))) int2 *)(P.HC + k.off);
                            const int64_t at = (int64_t)ix * k.row + iy;
                            cell[t] = make_int2(cells[at].x, cells[at].y);
                        }
                    }
                }
                uint64_t sbest = 0, saux = 0;
                const bool starter = wave == 0 && lane < cnt;
                if (starter) {
                    const uint64_t *ps = a.table + (uint64_t)mine.slot * SW;
                    sbest = ps[KW];
                    saux = ps[KW + 1];
                }
                for (int k = threadIdx.x; k < kDiveNodes; k += kBlock)
                    relbest[k] = kIntMax;
#pragma unroll
                for (int t = 0; t < kCT; t++) {
                    const int ct = threadIdx.x + t * kBlock;
                    if (ct < NP * kDiveCells)
                        cw[ct / kDiveCells][ct % kDiveCells] = cell[t];
                }
                lds_barrier();
                BPHASE(12)
                // ---- wave 0 alone runs the levels, out of LDS and registers
                // (no block barrier inside): each of its lane groups holds
                // one node of the level, lane m of the group its child m
                if (wave == 0) {
                    bool okp = false;
                    int nrel = 0;
                    if (starter) {
                        // a start node, as a one-level continuation entry
                        const bool okb = mine.g + mine.h < bound;
                        okp = okb && (uint32_t)(sbest >> 32) >= (uint32_t)mine.g;
                        stale += okb && !okp;
                        if (okp) {
                            reopen += (int)(uint32_t)saux != kIntMax;
                            *(int *)(a.table + (uint64_t)mine.slot * SW + KW + 1) = mine.g;
                            expanded++;
#pragma unroll
                            for (int i = 0; i < N; i++)
                                nrel |= (mpos[i] - org[i]) << (4 * i);
                            atomicMin(&relbest[rel_index(nrel)], mine.g);
                        }
                    }
                    // this lane's child: its mask's constants
                    const int m = glane;
                    const int relinc = (m & 1) | ((m >> 1) & 1) << 4 | ((m >> 2) & 1) << 8 | ((m >> 3) & 1) << 12;
                    const int idxinc = rel_index(relinc);
                    // equal gap costs (the reference's): the gap part of the child's cost depends on the mask alone
                    const bool eqgap = P.gap_open == P.gap_ext;
                    int coff[NP], gapw[NP], dg_const = 0, both = 0;
                    {
                        int p = 0;
#pragma unroll
                        for (int x = 0; x < N - 1; x++) {
#pragma unroll
                            for (int y = x + 1; y < N; y++, p++) {
                                const int bx = (m >> x) & 1, by = (m >> y) & 1;
                                coff[p] = bx * kDiveWS + by;
                                gapw[p] = pc[p].w;
                                if (bx & by)
                                    both |= 1 << p;
                                else
                                    dg_const += ((bx | by) ? P.gap_open : P.gap_gap) * gapw[p];
                            }
                        }
                    }
                    // near the lattice's far border a coordinate may be at its end
                    bool edge = false;
#pragma unroll
                    for (int i = 0; i < N; i++)
                        edge |= org[i] + kDiveW >= P.len[i];
                    // the level's nodes: the first kDiveFront set lanes of `pick`, one per lane group
                    uint64_t nkey = mine.key[0], ckey = 0;
                    int ng = mine.g, npm = mine.pmask, nidx = rel_index(nrel);
                    bool nact = false;
                    uint64_t pick = __ballot(okp);
                    auto hand_over = [&](uint64_t key_v, int g_v, int pm_v, int rel_v, int idx_v, bool pm_is_lane) {
                        uint64_t k_o = 0;
                        int g_o = 0, pm_o = 0, rel_o = 0, idx_o = 0;
                        bool act_o = false;
#pragma unroll
                        for (int q = 0; q < kDiveFront; q++) {
                            const bool any = pick != 0;  // uniform
                            const int src = any ? __ffsll((long long)pick) - 1 : 0;
                            pick &= pick - 1;
                            const uint64_t kq = bcast_lane((unsigned long long)key_v, src);
                            const int gq = bcast_lane(g_v, src), relq = bcast_lane(rel_v, src), idxq = bcast_lane(idx_v, src);
                            const int pmq = pm_is_lane ? (src & (lpn - 1)) : bcast_lane(pm_v, src);
                            if (group == q) {
                                k_o = kq;
                                g_o = gq;
                                pm_o = pmq;
                                rel_o = relq;
                                idx_o = idxq;
                                act_o = any;
                            }
                        }
                        nkey = k_o;
                        ng = g_o;
                        npm = pm_o;
                        nrel = rel_o;
                        nidx = idx_o;
                        nact = act_o;
                    };
                    hand_over(nkey, ng, npm, nrel, nidx, false);
                    int rec_cnt = 0, done = 0;
                    for (int d = 0; d < kDiveW; d++) {
                        if (!__ballot(nact) || rec_cnt + kDiveFront * (masks - 1) > kDiveRecs)
                            break;  // uniform
                        done++;
                        int blocked = 0, dg = 0, hh = 0;
                        if (edge) {  // uniform
#pragma unroll
                            for (int i = 0; i < N; i++)
                                blocked |= (org[i] + ((nrel >> (4 * i)) & 15) >= P.len[i]) << i;
                        }
                        if (eqgap) {  // uniform
                            dg = dg_const;
                            int p = 0;
#pragma unroll
                            for (int x = 0; x < N - 1; x++) {
#pragma unroll
                                for (int y = x + 1; y < N; y++, p++) {
                                    const int base = ((nrel >> (4 * x)) & 15) * kDiveWS + ((nrel >> (4 * y)) & 15);
                                    const int2 ch = cw[p][base + coff[p]];
                                    const int2 c0 = cw[p][base];
                                    hh += ch.x;
                                    dg += ((both >> p) & 1) ? c0.y : 0;
                                }
                            }
                        } else {
                            int p = 0;
#pragma unroll
                            for (int x = 0; x < N - 1; x++) {
#pragma unroll
                                for (int y = x + 1; y < N; y++, p++) {
                                    const int bx = (m >> x) & 1, by = (m >> y) & 1;
                                    const int base = ((nrel >> (4 * x)) & 15) * kDiveWS + ((nrel >> (4 * y)) & 15);
                                    const int2 ch = cw[p][base + coff[p]];
                                    const int2 c0 = cw[p][base];
                                    hh += ch.x;
                                    // one moves, the other idles: gap open iff the idle one moved into the node
                                    const int idle = bx ? y : x;
                                    const int g0 =
                                        (bx | by) ? (((npm >> idle) & 1) ? P.gap_open : P.gap_ext) : P.gap_gap;
                                    dg += (bx & by) ? c0.y : g0 * gapw[p];
                                }
                            }
                        }
                        const int g = ng + dg, f = g + hh;
                        const bool valid = nact && m >= 1 && !(m & blocked);
                        generated += valid;
                        const bool keep = valid && f < bound;
                        const int relc = nrel + relinc, cidx = nidx + idxinc;
                        // (a coordinate at kDiveW has no cells ahead of it in the window: not expanded
                        // here; coordinates are at most kDiveW <= 8, so adding 8 - kDiveW sets a
                        // field's top bit exactly there)
                        const bool inside = ((relc + (8 - kDiveW) * 0x1111) & 0x8888) == 0;
                        bool cont = false;
                        if (keep) {
                            const int old = atomicMin(&relbest[cidx], g);
                            cont = old > g && f < f_limit && inside && d + 1 < kDiveW;
                        }
                        const uint64_t km = __ballot(keep);
                        const int ri = rec_cnt + __popcll(km & ((1ull << lane) - 1ull));
                        rec_cnt += __popcll(km);
                        // the first kDiveFront continuing children are the next level
                        pick = __ballot(cont);
                        {
                            uint64_t rest = pick;
#pragma unroll
                            for (int q = 0; q < kDiveFront; q++)
                                rest &= rest - 1;
                            cont = cont && !((rest >> lane) & 1ull);
                        }
                        ckey = nkey + kinc[0];
                        if (keep)
                            recs[ri] = DiveRec{ckey, g, hh, m | (cont ? kDiveCont : 0)};
                        hand_over(ckey, g, 0, relc, cidx, true);
                    }
                    if (lane == 0) {
                        rec_n = rec_cnt;
                        dive_done = done;
                    }
                }
                lds_barrier();
                BPHASE(13)
                // ---- every generated child into the node table, at once, by the whole block
                const int nrec = rec_n, done = dive_done;
                const LocalPush<KW> lq_dive{lvl + done < depth ? lq[nxt] : nullptr, &lq_count[nxt], f_limit, lq_cap,
                                            outq, &out_n};
                for (int base = 0; base < nrec; base += kBlock) {
                    const int r = base + threadIdx.x;
                    const bool has = r < nrec;
                    const DiveRec rc = recs[has ? r : 0];
                    const uint64_t ck[KW] = {rc.key};
                    bool imp = false, cl = false;
                    int64_t slot = 0;
                    if (has) {
                        slot = relax<KW, kPfSlots>(a.table, a.cap_mask, ck, rc.g, rc.info & 15, rc.h, imp, cl, false,
                                                   SlotWords<KW, kPfSlots>{});
                        if (slot < 0) {
                            ovf++;
                            imp = false;
                            slot = 0;
                        }
                        claimed += cl;
                        if (imp && rc.key == P.goal_key[0])
                            atomicMin(a.goal_g, rc.g);
                    }
                    const bool was_cont = has && (rc.info & kDiveCont);
                    if (was_cont && imp) {
                        // an expansion that counted: close the node.  A slot claimed just now was
                        // never closed (a plain store); else a min, whose old value tells a reopening
                        int *closed = (int *)(a.table + (uint64_t)slot * SW + KW + 1);
                        if (cl) {
                            *closed = rc.g;
                        } else {
                            const int old = atomicMin(closed, rc.g);
                            reopen += old != kIntMax;
                        }
                        expanded++;
                    }
                    queue_improved<KW>(a, st, f0, w, has && imp && !was_cont, slot, ck, rc.g, rc.h, rc.info & 15, lq_dive);
                }
                BLK_COUNT(done, 1)
                BPHASE(14)
#ifdef PASTAR_PHASE_TIMERS
                if ((view.timing & 4) && timing && threadIdx.x == 0) {
                    atomicAdd(&ctl->body_ticks[10], 1ull);                       // dives
                    atomicAdd(&ctl->body_ticks[11], (unsigned long long)done);   // their levels
                    atomicAdd(&ctl->phase_ticks[4 + (done < 3 ? done : 3)], 1ull);  // dives of 0, 1, 2, 3+ levels
                    atomicAdd(&ctl->phase_ticks[cnt == 1 ? 0 : 1], 1ull);        // one start node / several
                    atomicAdd(&ctl->phase_ticks[2], (unsigned long long)nrec);   // children generated
                }
#endif
                lds_barrier();
                BPHASE(3)
                cur = nxt;
                lvl += done > 0 ? done - 1 : 0;
                continue;
            }
        }
        if constexpr (kTwoLevel && !kDive) {
            if (cnt == 1 && lvl + 1 < depth && (!SH || P.n_shards == 1)) {
                // one parent: this level and the next in one pass.  The next
                // level of the one-level pass would expand exactly this
                // parent's improved children below f_limit (its whole queue);
                // here group c expands child c right after group 0 relaxed it
                // (without the one-level pass's re-read of the child's best:
                // a child another block improved meanwhile is expanded at its
                // older g, which only adds work the improvement then redoes)
                __shared__ int kid_slot[16], kid_g[16];
                __shared__ unsigned kid_exp;
                const LEntry<KW> le = lq[cur][0];
                const int c = wave * npw + group;  // 0: the parent, else its child c
                const uint64_t *pslot = a.table + (uint64_t)le.slot * SW;
                const uint64_t lbest = pslot[KW], laux = pslot[KW + 1];
                Parent<N, KW> me;
                int posX[N], blockedX = 0;
                {
                    const uint64_t pk[KW] = {le.key[0]};
                    decode_key<N, KW>(P, n, pk, posX);
                }
#pragma unroll
                for (int i = 0; i < N; i++)
                    blockedX |= (posX[i] >= P.len[i]) << i;
                me.key[0] = le.key[0] + kinc_grp[0];
                me.blocked = 0;
#pragma unroll
                for (int i = 0; i < N; i++) {
                    me.pos[i] = posX[i] + ((c >> i) & 1);
                    me.blocked |= (me.pos[i] >= P.len[i]) << i;
                }
                me.pmask = c == 0 ? le.pmask : c;
                me.g = le.g;
                // this lane's target: group 0 lane m the parent's child m,
                // group c lane m child c's child m
                uint64_t tk[KW] = {me.key[0] + kinc[0]};
                SlotWords<KW, kPfSlots> pf{};
                auto prefetch = [&] { pf = slot_prefetch<KW, kPfSlots>(a.table, a.cap_mask, tk); };
                stage_terms_fixed<N, KW>(P, pc, me, terms, glane, prefetch);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                // the parent, as a one-level continuation entry
                const bool okb = le.g + le.h < bound;
                const bool okp = okb && (uint32_t)(lbest >> 32) >= (uint32_t)le.g;
                if (threadIdx.x == 0) {
                    if (okp) {
                        reopen += (int)(uint32_t)laux != kIntMax;
                        *(int *)(a.table + (uint64_t)le.slot * SW + KW + 1) = le.g;
                        expanded++;
                    }
                    stale += okb && !okp;
                }
                // level L: the parent's children on group 0
                const int m = glane;
                const int2 d1 = child_cost<N>(Pg, npairs, terms, m);
                const bool v1 = okp && c == 0 && m >= 1 && !(m & blockedX);
                const int g1 = le.g + d1.x, h1 = d1.y, f1 = g1 + h1;
                generated += v1;
                bool imp1 = false, cl1 = false;
                int64_t slot1 = 0;
                if (v1 && f1 < bound) {
                    slot1 = relax<KW, kPfSlots>(a.table, a.cap_mask, tk, g1, m, h1, imp1, cl1, true, pf);
                    if (slot1 < 0) {
                        ovf++;
                        imp1 = false;
                    }
                    claimed += cl1;
                    if (imp1 && tk[0] == P.goal_key[0])
                        atomicMin(a.goal_g, g1);
                }
                const bool exp1 = imp1 && f1 < f_limit;
                // improved children past the batch: the block's deferred
                // open-list entries (route_child's out path)
                {
                    bool global = imp1 && !exp1;
                    const Entry e1 = {(uint32_t)(slot1 < 0 ? 0 : slot1), f1};
                    const uint64_t gm = __ballot(global);
                    if (gm) {
                        const int leader = __ffsll((long long)gm) - 1;
                        int b0 = 0;
                        if (lane == leader)
                            b0 = atomicAdd(&out_n, __popcll(gm));
                        b0 = bcast_lane(b0, leader);
                        if (global) {
                            const int pos = b0 + __popcll(gm & ((1ull << lane) - 1ull));
                            if (pos < kOutCap) {
                                outq[pos] = e1;
                                global = false;
                            }
                        }
                    }
                    queue_append(a, global, bucket_of(f1, f0, w), e1, st, false);
                }
                if (c == 0) {
                    kid_slot[m] = (int)slot1;
                    kid_g[m] = g1;
                }
                const uint64_t eb = __ballot(c == 0 && exp1);
                if (threadIdx.x == 0)
                    kid_exp = (unsigned)eb;  // group 0 is lanes 0..15 of wave 0
                lds_barrier();
                // level L + 1: group c expands child c
                const bool expc = c >= 1 && ((kid_exp >> c) & 1u);
                const int gc = kid_g[c], slotc = kid_slot[c];
                if (expc && glane == 0) {
                    // the closing of the child (the one-level pass's store), as
                    // a min: its old value tells a reopening
                    const int old = atomicMin((int *)(a.table + (uint64_t)slotc * SW + KW + 1), gc);
                    reopen += old != kIntMax;
                    expanded++;
                }
                const int2 d2 = child_cost<N>(Pg, npairs, terms, m);
                bool v2 = expc && m >= 1 && !(m & me.blocked);
                const int g2 = gc + d2.x, h2 = d2.y;
                if (v2) {
                    generated++;
                    if (g2 + h2 >= bound)
                        v2 = false;
                }
                const LocalPush<KW> lq_next2{lvl + 2 < depth ? lq[nxt] : nullptr, &lq_count[nxt], f_limit, lq_cap,
                                             outq, &out_n};
                route_child<KW, kPfSlots, SH>(a, P, st, f0, w, v2, true, P.shard, tk, g2, h2, m, claimed, ovf, lq_next2,
                                          false, v2, pf);
                BLK_COUNT(2, 1)
                lds_barrier();
                BPHASE(3)
                cur = nxt;
                lvl++;  // two levels
                continue;
            }
        }
        const LocalPush<KW> lq_next{lvl + 1 < depth ? lq[nxt] : nullptr, &lq_count[nxt], f_limit, lq_cap, outq,
                                    &out_n};
        for (int base = 0; base < cnt; base += per_block) {
            const int idx = base + wave * npw + group;
            const bool ok = idx < cnt;
            process(ok, Entry{0, 0}, no_ps, ok ? lq[cur][idx] : no_le, true, lq_next);
            BLK_COUNT(0, 1)
        }
        BLK_COUNT(1, 0)
        lds_barrier();
        BPHASE(3)
        cur = nxt;
    }
    // the deferred open-list entries: ranked per bucket in LDS, then one
    // cursor atomic per bucket for the whole block, all buckets at once (a
    // wave-serial loop over buckets costs one dependent round trip each)
    {
        constexpr int kPer = kOutCap / kBlock;
        constexpr int kWin = 64;  // buckets above the block's lowest one ranked in LDS
        __shared__ int fb_min;
        __shared__ unsigned fb_cnt[kWin];
        __shared__ unsigned long long fb_base[kWin];
        const int no = out_n < kOutCap ? out_n : kOutCap;  // read after the last process barrier
        if (no > 0) {  // uniform
            if (threadIdx.x == 0)
                fb_min = kBuckets;
            if (threadIdx.x < kWin)
                fb_cnt[threadIdx.x] = 0;
            Entry e[kPer];
            int bk[kPer], rk[kPer];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                const int i = k * kBlock + threadIdx.x;
                e[k] = i < no ? outq[i] : Entry{0, 0};
                bk[k] = i < no ? bucket_of(entry_f(e[k]), f0, w) : kBuckets;
                if (kPartial && i < no && e[k].f < 0) {  // a parent with children left: queued ahead of them
                    const int pb = bk[k] - partial_ahead, be = view.batch_b + view.batch_nb;
                    bk[k] = pb < be ? be : pb;
                }
                if (i < no)
                    atomicMin(&fb_min, bk[k]);
            }
            __syncthreads();
            const int bmin = fb_min;
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                rk[k] = -1;
                if (k * kBlock + (int)threadIdx.x < no && bk[k] - bmin < kWin)
                    rk[k] = (int)atomicAdd(&fb_cnt[bk[k] - bmin], 1u);
            }
            __syncthreads();
            const int sq = blockIdx.x % kSub;
            // (each reserving lane also opens the chunks that start in its
            // range, before any store of the block: queue_reserve)
            if (threadIdx.x < kWin && fb_cnt[threadIdx.x])
                fb_base[threadIdx.x] = queue_reserve(a, bmin + threadIdx.x, sq, fb_cnt[threadIdx.x]);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                if (rk[k] >= 0)
                    queue_store(a, bk[k], sq, fb_base[bk[k] - bmin] + (unsigned long long)rk[k], e[k], st);
                // beyond the window: the wave-aggregated path
                const int i = k * kBlock + threadIdx.x;
                queue_append(a, i < no && rk[k] < 0, bk[k], e[k], st, false);
            }
        }
    }
    expanded = wave_sum(expanded);
    reopen = wave_sum(reopen);
    generated = wave_sum(generated);
    claimed = wave_sum(claimed);
    ovf = wave_sum(ovf);
    stale = wave_sum(stale);
    if constexpr (kPartial) {
        part_q = wave_sum(part_q);
        part_t = wave_sum(part_t);
    }
    if (lane == 0) {
        unsigned long long *row = stat_row(st, blockIdx.x * kWaves + wave);
        if (expanded)
            atomicAdd(&row[kStExpanded], (unsigned long long)expanded);
        if (reopen)
            atomicAdd(&row[kStReopen], (unsigned long long)reopen);
        if (generated)
            atomicAdd(&row[kStGenerated], (unsigned long long)generated);
        if (claimed)
            atomicAdd(&row[kStClaimed], (unsigned long long)claimed);
        if (ovf)
            atomicAdd(&row[kStOvfTable], (unsigned long long)ovf);
        if (stale)
            atomicAdd(&row[kStDropped], (unsigned long long)stale);
        if constexpr (kPartial) {
            if (part_q)
                atomicAdd(&row[kStPartQueued], (unsigned long long)part_q);
            if (part_t)
                atomicAdd(&row[kStPartTaken], (unsigned long long)part_t);
        }
    }
#ifdef PASTAR_PHASE_TIMERS
    if ((view.timing & 4) && timing && threadIdx.x == 0) {
        const unsigned long long dt = device_clock() - blk_t0;
        atomicAdd(&ctl->blk_stats[0], 1ull);
        atomicAdd(&ctl->blk_stats[1], (unsigned long long)blk_levels);
        atomicMax(&ctl->blk_stats[2], (unsigned long long)blk_levels);
        atomicAdd(&ctl->blk_stats[3], (unsigned long long)blk_rounds);
        atomicMax(&ctl->blk_stats[4], (unsigned long long)blk_rounds);
        atomicMax(&ctl->blk_stats[5], dt);
    }
#endif
#undef BLK_COUNT
    const bool fuse = ctl->fuse;
    const bool xsnap = SH && a.x != nullptr;  // sharded: the last block publishes the step's hand-over values
    if (!fuse && !timing && !xsnap)
        return;
    // the last block to finish: two-level arrival (blockIdx % kArrive, then
    // the groups) so that no counter takes more than ~64 arrivals
    // Everything select reads from this launch is an atomic result (the
    // step statistics, queue W cursors, goal, cur_b), executed at the memory
    // side; each wave waits for its own atomics to complete before the
    // block arrives, and select reads them with coherent (sc1) loads.  No
    // agent-scope fence: on gfx950 it writes back the whole L2 (buffer_wbl2),
    // which costs far more than the arrival itself.
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    BPHASE(4)
    if (threadIdx.x == 0) {
        const unsigned na = (unsigned)nact;
        const unsigned sub = blockIdx.x % kArrive;
        const unsigned nsub = (na - sub + kArrive - 1) / kArrive;
        const unsigned ngrp = na < (unsigned)kArrive ? na : (unsigned)kArrive;
        int l = 0;
        if (na <= (unsigned)kArrive)  // few blocks: one level
            l = __hip_atomic_fetch_add(&ctl->arrive_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == na - 1;
        else if (__hip_atomic_fetch_add(&ctl->arrive[sub], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 nsub - 1)
            l = __hip_atomic_fetch_add(&ctl->arrive_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                ngrp - 1;
        last = l;
    }
    __syncthreads();
    BPHASE(5)
    if (bprof)
        ctl->body_launches++;
#undef BPHASE
    if (!last)
        return;
    if (threadIdx.x < kArrive)
        st_agent(&ctl->arrive[threadIdx.x], 0u);
    if (threadIdx.x == 0)
        st_agent(&ctl->arrive_top, 0u);
    if (xsnap) {
        // every block's ring appends are complete (each wave waited for its
        // own before arriving): the positions reserved so far are what the
        // pack kernel of this step may take
        const int slot = a.step & (kXSlots - 1);
        if (threadIdx.x < kMaxShards)
            st_agent(&a.x->w_snap[slot][threadIdx.x], ld_agent(&a.x->w[threadIdx.x]));
    }
    unsigned long long t0 = 0;
    if (timing) {
        __shared__ unsigned long long t_lo;
        if (threadIdx.x == 0)
            t_lo = ~0ull;
        __syncthreads();
        if (threadIdx.x < kArrive && threadIdx.x < nact)
            atomicMin(&t_lo, ld_agent(&a.stamps[threadIdx.x]));
        __syncthreads();
        t0 = t_lo;
    }
    const unsigned long long ts = timing ? device_clock() : 0;
    if (fuse)
        select_block<false>(a, view);  // (the sharded search selects in its own launch)
    if (timing && threadIdx.x == 0) {
        const unsigned long long t1 = device_clock();
        if (t1 > t0) {
            ctl->expand_ticks += t1 - t0;
            ctl->select_ticks += t1 - ts;
            ctl->timed_launches++;
            if (ctl->prev_end && t0 > ctl->prev_end)
                ctl->gap_ticks += t0 - ctl->prev_end;
            ctl->prev_end = t1;
        }
    }
}

// Relax nodes received from other shards (the owner side of the RCCL
// exchange; replaces PAStarMessageProcesser -> enqueue, PAStar.cpp:241-250).
template <int KW>
__global__ __launch_bounds__(kBlock) void insert_remote_kernel(SearchArgs a, const Remote<KW> *__restrict__ recs,
                                                               unsigned long long count)
{
    const DevProblem &P = *a.P;
    Ctl *ctl = a.ctl;
    StepStats *st = a.stats;
    const int w = ctl->band_log2, f0 = ctl->f0;
    const int bound = *(volatile int *)a.goal_g;
    unsigned claimed = 0, ovf = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long iters = (count + stride - 1) / stride;
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x + it * stride;
        bool valid = i < count;
        uint64_t ck[KW];
        int g = 0, h = 0, m = 0;
#pragma unroll
        for (int k = 0; k < KW; k++)
            ck[k] = 0;
        if (valid) {
            const Remote<KW> r = recs[i];
#pragma unroll
            for (int k = 0; k < KW; k++)
                ck[k] = r.key[k];
            g = r.g;
            h = r.h;
            m = r.pmask;
            valid = g + h < bound;
        }
        route_child<KW, 1, false>(a, P, st, f0, w, valid, true, P.shard, ck, g, h, m, claimed, ovf,
                                  LocalPush<KW>{nullptr, nullptr, 0, 0, nullptr, nullptr}, true);
    }
    claimed = wave_sum(claimed);
    ovf = wave_sum(ovf);
    if (lane_id() == 0) {
        unsigned long long *row = stat_row(st, (blockIdx.x * blockDim.x + threadIdx.x) / 64);
        if (claimed)
            atomicAdd(&row[kStClaimed], (unsigned long long)claimed);
        if (ovf)
            atomicAdd(&row[kStOvfTable], (unsigned long long)ovf);
    }
}

// The staged open-list entries of an insert that ran beside a select
// (xchg_lag = 1), appended on the select's own stream: every entry is written
// before the next select can cut it.  The count is cleared by the launch's
// last block for the insert that uses the staging array next.
__global__ __launch_bounds__(kBlock) void xdrain_kernel(SearchArgs a, const Entry *__restrict__ stage,
                                                        unsigned long long *stage_n, unsigned long long stage_cap,
                                                        unsigned *arrive)
{
    const Ctl *ctl = a.ctl;
    if (ld_agent(&ctl->status))
        return;
    const int w = ctl->band_log2, f0 = ctl->f0;
    unsigned long long n = ld_agent(stage_n);
    n = n < stage_cap ? n : stage_cap;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long iters = (n + stride - 1) / stride;
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x + it * stride;
        const bool has = i < n;
        const Entry e = has ? stage[i] : Entry{0, 0};
        queue_append(a, has, bucket_of(e.f, f0, w), e, a.stats, true);
    }
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {
        st_agent(stage_n, 0ull);
        st_agent(arrive, 0u);
    }
}

// ---------------------------------------------------------------------------
// Shard exchange kernels (side stream).  One step:
//   xpack    ring -> fixed-size blocks, one per destination shard, each with
//            a header {records, backlog, had work, failed, goal}
//   (all-to-all of the blocks: RCCL send/recv, or xcopy in a shard group)
//   xinsert  relax the received records on their owner; fold the headers:
//            the best goal, failures, and the termination count
// They replace the reference's sender / receiver / message processor threads
// (PAStarSender.cpp:10-131, PAStarReceiver.cpp:11-120,
// PAStarMessageProcesser.cpp:12-78) and check_stop's allreduces
// (PAStar.cpp:502-519).
// ---------------------------------------------------------------------------
struct XArgs {
    XState *x;
    Ctl *ctl;
    StepStats *stats_b;  // the insert kernel's own step statistics
    const int *goal_g;
    void *outbox;        // Remote<KW>[n_shards][outbox_cap] rings
    unsigned long long outbox_cap;
    unsigned char *send;  // [n_shards] blocks of block_bytes
    unsigned char *recv;  // [n_shards] blocks of block_bytes
    unsigned long long block_bytes, block_recs;
    int n_shards, shard, step, lag;
    // lag 1: the open-list entries of this step's received records (see LocalPush::stage)
    Entry *stage;
    unsigned long long *stage_n;
    unsigned long long stage_cap;
};

__device__ __forceinline__ XHdr *xblock_hdr(unsigned char *blocks, unsigned long long block_bytes, int d)
{
    return reinterpret_cast<XHdr *>(blocks + (size_t)d * block_bytes);
}

// grid (n_shards, blocks per destination)
template <int KW>
__global__ __launch_bounds__(kBlock) void xpack_kernel(XArgs t)
{
    XState *x = t.x;
    const int d = blockIdx.x, par = t.step & 1, slot = t.step & (kXSlots - 1);
    // fold the insert kernel's statistics of the step before (stream order:
    // that launch is complete, the next one not started)
    if (blockIdx.x == 0 && blockIdx.y == 0) {
        StepStats *sb = t.stats_b;
        if (threadIdx.x < kStatRows) {
            unsigned long long cl = sb->row[threadIdx.x][kStClaimed], ov = sb->row[threadIdx.x][kStOvfTable];
            sb->row[threadIdx.x][kStClaimed] = 0;
            sb->row[threadIdx.x][kStOvfTable] = 0;
            cl = wave_sum(cl);
            ov = wave_sum(ov);
            if (threadIdx.x == 0) {
                x->claimed_b += cl;
                const int fm = fail_bits(sb->ovf_near, sb->ovf_far, ov, sb->ovf_out);
                sb->ovf_near = sb->ovf_far = sb->ovf_out = 0;
                if (fm)
                    atomicOr(&x->fail_b, fm);  // read by the next select (StepInfo::fail)
            }
        }
    }
    __syncthreads();
    // this step's share of every destination's ring, from values that are
    // fixed by now: the ring positions the expand kernel's last block
    // published (a launch that left early publishes nothing: the slot then
    // holds an older, lower position, which only sends less), the positions
    // the last pack consumed, and the select kernel's StepInfo
    const XState::StepInfo si = x->info[slot];
    const bool stopped = si.fail != 0;
    unsigned long long r0 = 0, n = 0, sent_all = 0, backlog_all = 0, pair_max = 0;
    for (int k = 0; k < t.n_shards; k++) {
        const unsigned long long rk = x->r[par][k], wk = ld_agent(&x->w_snap[slot][k]);
        const unsigned long long avail = (k == t.shard || stopped || wk < rk) ? 0 : wk - rk;
        const unsigned long long nk = avail < t.block_recs ? avail : t.block_recs;
        sent_all += nk;
        backlog_all += avail - nk;
        pair_max = avail > pair_max ? avail : pair_max;
        if (k == d) {
            r0 = rk;
            n = nk;
        }
    }
    const Remote<KW> *ring = reinterpret_cast<const Remote<KW> *>(t.outbox) + (size_t)d * t.outbox_cap;
    Remote<KW> *dst = reinterpret_cast<Remote<KW> *>(t.send + (size_t)d * t.block_bytes + sizeof(XHdr));
    for (unsigned long long k = (unsigned long long)blockIdx.y * blockDim.x + threadIdx.x; k < n;
         k += (unsigned long long)gridDim.y * blockDim.x)
        dst[k] = ring[(r0 + k) & (t.outbox_cap - 1)];
    if (blockIdx.y == 0 && threadIdx.x == 0) {
        // (the consumed position becomes visible to the expand kernel, which may
        // run beside this launch and reuses ring places up to it, only once every
        // block of this launch has copied its records out: the insert kernel that
        // follows on this stream publishes it)
        x->r[par ^ 1][d] = r0 + n;
        XHdr h{};
        h.n = n;
        h.sent_all = sent_all;
        h.backlog_all = backlog_all;
        h.has_work = si.has_work != 0;
        h.low_b = (unsigned long long)(unsigned)si.low_b | (pair_max << 32);
        h.fail = (unsigned long long)si.fail;
        h.goal = si.goal;
        h.step = (unsigned long long)t.step;
        *xblock_hdr(t.send, t.block_bytes, d) = h;
        if (d == t.shard) {  // this shard's own header needs no transport
            *xblock_hdr(t.recv, t.block_bytes, d) = h;
            x->sent += sent_all;
            if (backlog_all) {
                x->backlog_steps++;
                if (backlog_all > x->backlog_max)
                    x->backlog_max = backlog_all;
            }
        }
    }
}

// In-process shard group: block s of this shard's inbox is read from shard
// s's send area (src[s] points at the block shard s packed for this shard).
// grid (n_shards, blocks per source)
struct XPeers {
    const unsigned char *src[kMaxShards];
};

__global__ __launch_bounds__(kBlock) void xcopy_kernel(XPeers p, unsigned char *recv, unsigned long long block_bytes,
                                                       unsigned long long rec_bytes, int shard)
{
    const int s = blockIdx.x;
    if (s == shard)
        return;
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 *src = reinterpret_cast<const u64x2 *>(p.src[s]);
    u64x2 *dst = reinterpret_cast<u64x2 *>(recv + (size_t)s * block_bytes);
    unsigned long long n = reinterpret_cast<const XHdr *>(src)->n;
    const unsigned long long fit = (block_bytes - sizeof(XHdr)) / rec_bytes;
    n = n < fit ? n : fit;  // (never past the block, whatever the header says)
    const unsigned long long vecs = (sizeof(XHdr) + n * rec_bytes + 15) / 16;
    for (unsigned long long k = (unsigned long long)blockIdx.y * blockDim.x + threadIdx.x; k < vecs;
         k += (unsigned long long)gridDim.y * blockDim.x)
        dst[k] = src[k];
}

// Relax the records received from the other shards (the owner side of the
// exchange; replaces PAStarMessageProcesser -> enqueue, PAStar.cpp:241-250),
// and fold every shard's header: the best goal, failures, and termination
// (check_stop, PAStar.cpp:480-547): the search ends when, for lag + 1 steps
// in a row, no shard had a batch, sent a record or kept a backlog; every
// shard sees the same headers and so decides the same at the same step.
template <int KW>
__global__ __launch_bounds__(kBlock) void xinsert_kernel(SearchArgs a, XArgs t)
{
    const DevProblem &P = *a.P;
    Ctl *ctl = a.ctl;
    StepStats *st = a.stats;  // the side stream's own statistics (XArgs::stats_b)
    const int G = t.n_shards;
    __shared__ unsigned long long pre[kMaxShards + 1];
    __shared__ int goal_s;
    if (threadIdx.x == 0) {
        unsigned long long tot = 0, backlog = 0, demand = 0;
        int work = 0, fl = 0, gmin = kBuckets;
        long long goal = kIntMax;
        for (int s = 0; s < G; s++) {
            const XHdr *h = xblock_hdr(t.recv, t.block_bytes, s);
            pre[s] = tot;
            const unsigned long long n = s == t.shard ? 0 : (h->n <= t.block_recs ? h->n : t.block_recs);
            tot += n;
            // (only fields that are the same in every block of sender s)
            backlog += h->backlog_all;
            work |= h->has_work != 0 || h->sent_all != 0;
            // the most one shard had for one destination in a step (sent and
            // left over): sizes the next round's blocks, the same on every shard
            if ((h->low_b >> 32) > demand)
                demand = h->low_b >> 32;
            if ((int)(unsigned)h->low_b < gmin)
                gmin = (int)(unsigned)h->low_b;
            fl |= (int)h->fail;
            if (h->goal < goal)
                goal = h->goal;
        }
        pre[G] = tot;
        goal_s = (int)goal;
        if (blockIdx.x == 0) {
            XState *x = t.x;
            // the ring places this step's pack kernel has copied out are free now
            for (int d = 0; d < G; d++)
                st_agent(&x->r_pub[d], x->r[(t.step & 1) ^ 1][d]);
            x->received += tot;
            if (demand > x->demand_max)
                x->demand_max = demand;
            st_agent(&x->gmin_b, gmin);
            if (goal < ld_agent(a.goal_g))
                atomicMin(a.goal_g, (int)goal);
            const int status = ld_agent(&ctl->status);
            if (fl && status < 2) {
                // a shard failed: every shard stops at this step (each
                // reports its own fail bits; 0x200: a device wait ran out)
                if (fl & 0x200) {
                    ctl->fault_sites = ld_agent(&ctl->fault);
                    ctl->status = 4;
                } else if (fl & 0x100) {
                    ctl->status = 3;
                } else {
                    atomicOr(&ctl->fail_mask, x->fail_b | 0x1000);  // 0x1000: some shard ran out of capacity
                    ctl->status = 2;
                }
            } else if (status == 0) {
                const bool quiet = !work && backlog == 0;
                const int run = quiet ? x->quiet_run + 1 : 0;
                x->quiet_run = run;
                if (run > t.lag) {
                    // (the step count every shard agrees on: the main
                    // stream's own counter may be a select ahead)
                    x->steps_done = (unsigned long long)t.step + 1;
                    ctl->status = 1;
                }
            }
        }
    }
    __syncthreads();
    const unsigned long long count = pre[G];
    if (count == 0)
        return;
    const int w = ctl->band_log2, f0 = ctl->f0;
    int bound = *(volatile int *)a.goal_g;
    if (goal_s < bound)
        bound = goal_s;
    unsigned claimed = 0, ovf = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long iters = (count + stride - 1) / stride;
    for (unsigned long long it = 0; it < iters; it++) {
        const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x + it * stride;
        bool valid = i < count;
        uint64_t ck[KW];
        int g = 0, h = 0, m = 0;
#pragma unroll
        for (int k = 0; k < KW; k++)
            ck[k] = 0;
        if (valid) {
            int s = 0;
            while (pre[s + 1] <= i)
                s++;
            const Remote<KW> *recs =
                reinterpret_cast<const Remote<KW> *>(t.recv + (size_t)s * t.block_bytes + sizeof(XHdr));
            const Remote<KW> r = recs[i - pre[s]];
#pragma unroll
            for (int k = 0; k < KW; k++)
                ck[k] = r.key[k];
            g = r.g;
            h = r.h;
            m = r.pmask;
            valid = g + h < bound;
        }
        route_child<KW, 1, false>(a, P, st, f0, w, valid, true, P.shard, ck, g, h, m, claimed, ovf,
                                  LocalPush<KW>{nullptr, nullptr, 0, 0, nullptr, nullptr, t.stage, t.stage_n, t.stage_cap},
                                  true);
    }
    claimed = wave_sum(claimed);
    ovf = wave_sum(ovf);
    if (lane_id() == 0) {
        unsigned long long *row = stat_row(st, (blockIdx.x * blockDim.x + threadIdx.x) / 64);
        if (claimed)
            atomicAdd(&row[kStClaimed], (unsigned long long)claimed);
        if (ovf)
            atomicAdd(&row[kStOvfTable], (unsigned long long)ovf);
    }
}

// Reset the open list between searches: zero the chunk-table entries the
// last search used (its W cursors say how many chunks each sub-queue took)
// and then the cursors.  One thread per (bucket, sub-queue); replaces a
// memset of the whole chunk table (64 MB at the default capacity).
__global__ void queue_reset_kernel(Queues *__restrict__ q, uint32_t *__restrict__ chunk_tab,
                                   unsigned long long maxch)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= kBuckets * kSub)
        return;
    const int b = k % kBuckets, sq = k / kBuckets;  // sub-queue-major like the cursors
    const unsigned long long w = q->W[b][sq];
    unsigned long long used = (w + kChunk - 1) >> kChunkLog2;
    if (used > maxch)
        used = maxch;
    uint32_t *row = chunk_tab + ((size_t)b * kSub + sq) * maxch;
    for (unsigned long long c = 0; c < used; c++)
        row[c] = 0;
    q->W[b][sq] = 0;
    q->R[b][sq] = 0;
}

// A search's device setup in one launch (in place of a table fill, a queue
// reset and five small memsets): the node table cleared (init_table_kernel),
// the queues reset (queue_reset_kernel's rule, when they are known
// consistent), the step statistics, the arrival stamps, the goal and the
// open-list census zeroed by block 0, which also copies the search's control
// block and origin record from pinned host memory (`stage`, written by the
// host before the launch; in place of a host-to-device copy).
template <int SW>
__global__ __launch_bounds__(kBlock) void search_init_kernel(uint64_t *__restrict__ table, uint64_t nslots, int kw,
                                                            Queues *__restrict__ q, uint32_t *__restrict__ chunk_tab,
                                                            unsigned long long maxch, int reset_queues,
                                                            StepStats *__restrict__ stats,
                                                            unsigned long long *__restrict__ stamps,
                                                            int *__restrict__ goal,
                                                            unsigned long long *__restrict__ census,
                                                            const uint32_t *__restrict__ stage,
                                                            uint32_t *__restrict__ ctl_dst, int stage_words,
                                                            int seed_taken)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = tid; i < nslots; i += stride) {
        uint64_t *s = table + i * SW;
#pragma unroll
        for (int w = 0; w < SW; w++)
            s[w] = w == kw ? ~0ull : (w == kw + 1 ? (uint64_t)kIntMax : 0ull);
    }
    if (reset_queues) {
        for (uint64_t k = tid; k < (uint64_t)kBuckets * kSub; k += stride) {
            const int b = (int)(k % kBuckets), sq = (int)(k / kBuckets);
            const unsigned long long w = q->W[b][sq];
            unsigned long long used = (w + kChunk - 1) >> kChunkLog2;
            if (used > maxch)
                used = maxch;
            uint32_t *row = chunk_tab + ((size_t)b * kSub + sq) * maxch;
            for (unsigned long long c = 0; c < used; c++)
                row[c] = 0;
            q->W[b][sq] = 0;
            // seed_taken: the origin, appended next at (bucket 0, sub-queue
            // 0), is already the first batch the staged control block holds
            q->R[b][sq] = seed_taken && b == 0 && sq == 0 ? 1 : 0;
        }
    }
    if (blockIdx.x == 0) {
        if (seed_taken && !reset_queues && threadIdx.x == 0)
            q->R[0][0] = 1;  // (the queues were cleared by a memset)
        for (int k = threadIdx.x; k < stage_words; k += blockDim.x)
            if (k != (int)(offsetof(Ctl, fault) / 4))  // (sticky: see Ctl::fault)
                ctl_dst[k] = stage[k];
        unsigned long long *sw = reinterpret_cast<unsigned long long *>(stats);
        for (int k = threadIdx.x; k < (int)(sizeof(StepStats) / 8); k += blockDim.x)
            sw[k] = 0;
        for (int k = threadIdx.x; k < kArrive; k += blockDim.x)
            stamps[k] = 0;
        if (threadIdx.x == 0) {
            *goal = kIntMax;
            census[0] = census[1] = census[2] = 0;
            census[3] = census[4] = ~0ull;
        }
    }
}

// Open entries left in the queues (current or superseded), for the
// statistics: one read of every cursor pair.
// gate (may be null): run only when the search ended with the goal found
// (*gate == 1, Ctl::status), so the host may enqueue it behind a graph
// replay before knowing whether that replay finished the search
__global__ void queue_census_kernel(const Queues *__restrict__ q, unsigned long long *__restrict__ out,
                                    const int *__restrict__ gate)
{
    if (gate && *(volatile const int *)gate != 1)
        return;
    unsigned long long s = 0;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < kBuckets * kSub; k += gridDim.x * blockDim.x)
        s += q->W[k / kSub][k % kSub] - q->R[k / kSub][k % kSub];
    s = wave_sum(s);
    if (lane_id() == 0 && s)
        atomicAdd(out, s);
}

// Debug check (PASTAR_DEBUG): open nodes left in the queues: entries that are still current (f equal to
// the node's best g + h; stale ones are superseded), out[0]; out[1] counts
// those with f below `goal` (none may remain when the search terminates).
template <int KW>
__global__ __launch_bounds__(kBlock) void open_census_kernel(SearchArgs a, int goal, unsigned long long *__restrict__ out)
{
    constexpr int SW = slot_words<KW>();
    const unsigned long long maxch = a.ctl->maxch;
    unsigned long long live = 0, below = 0;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < kBuckets * kSub; k += gridDim.x * blockDim.x) {
        const int b = k / kSub, sq = k % kSub;
        const unsigned long long w = a.q->W[b][sq];
        for (unsigned long long p = a.q->R[b][sq]; p < w; p++) {
            if ((p >> kChunkLog2) >= maxch)
                break;
            const uint32_t c = a.chunk_tab[((size_t)b * kSub + sq) * maxch + (p >> kChunkLog2)];
            if (c == 0 || c == kNoChunk)
                break;
            const Entry e = a.pool[(size_t)(c - 1) * kChunk + (p & (kChunk - 1))];
            const uint64_t *slot = a.table + (uint64_t)e.slot * SW;
            const int g = (int)(slot[KW] >> 32), h = (int)(slot[KW + 1] >> 32);
            if (g + h == e.f) {
                live++;
                below += e.f < goal;
                if (e.f < goal) {
                    atomicMin(&out[2], (unsigned long long)e.f);
                    atomicMin(&out[3], (unsigned long long)b);
                }
            }
        }
    }
    live = wave_sum(live);
    below = wave_sum(below);
    if (lane_id() == 0) {
        if (live)
            atomicAdd(&out[0], live);
        if (below)
            atomicAdd(&out[1], below);
    }
}

// Backtrace walk (backtrace.cpp:47-69): from `start`, follow parent masks,
// writing them to `masks`, until the origin, `max` steps, or (local_only) a
// parent owned by another shard.  Single lane.  info = {steps, status}.
template <int N, int KW>
__device__ __forceinline__ void walk_chain(const DevProblem *__restrict__ Pp, const uint64_t *__restrict__ table,
                                           uint64_t cap_mask, const uint64_t *__restrict__ start, int max,
                                           int local_only, int32_t *__restrict__ masks,
                                           uint64_t *__restrict__ last_key, int *__restrict__ info)
{
    const DevProblem &Pg = *Pp;
    const int n = N ? N : Pg.n;
    constexpr int SW = slot_words<KW>();
    // one dependent chain: the constants in registers up front, and each
    // step's probe reads a slot's key words and best in one go
    const KConst<N, KW> P = load_kconst<N, KW>(Pg);
    uint64_t origin[KW], key[KW];
#pragma unroll
    for (int w = 0; w < KW; w++) {
        origin[w] = Pg.origin_key[w];
        key[w] = start[w];
    }
    int steps = 0, status = 0;
    for (;;) {
        bool at_origin = true;
#pragma unroll
        for (int w = 0; w < KW; w++)
            at_origin &= key[w] == origin[w];
        if (at_origin) {
            status = 1;
            break;
        }
        if (steps >= max) {
            status = 2;
            break;
        }
        // lookup (backtrace.cpp:47-69 ClosedList find), slot words
        // [0, KW] = key + best in one read
        uint64_t idx = probe_start<KW>(key, cap_mask);
        int m = -1;
        for (int probe = 0; probe < kMaxProbe; probe++) {
            // the slot's key words and best in one round trip (plain loads
            // get best sunk behind the key compare, a second trip per step)
            const uint64_t *sl = table + idx * SW;
            uint64_t wv[KW + 1];
            if constexpr (KW <= 2) {
                typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                u64x2 a0, a1;
                asm volatile("global_load_dwordx4 %0, %2, off\n\t"
                             "global_load_dwordx4 %1, %2, off offset:16\n\t"
                             "s_waitcnt vmcnt(0)"
                             : "=&v"(a0), "=&v"(a1)
                             : "v"(sl)
                             : "memory");
                wv[0] = a0.x;
                wv[1] = a0.y;
                if constexpr (KW == 2)
                    wv[2] = a1.x;
            } else {
#pragma unroll
                for (int w = 0; w <= KW; w++)
                    wv[w] = sl[w];
            }
            if (wv[0] == 0)
                break;
            bool same = true;
#pragma unroll
            for (int w = 0; w < KW; w++)
                same &= wv[w] == key[w];
            if (same) {
                m = (int)(uint32_t)wv[KW];
                break;
            }
            idx = (idx + 1) & cap_mask;
        }
        if (m < 0) {
            status = -1;
            break;
        }
        masks[steps++] = m;
        int pos[Parent<N, KW>::NMAX];
        decode_key<N, KW>(P, n, key, pos);
#pragma unroll
        for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
            if ((N == 0 && i >= n) || !((m >> i) & 1))
                continue;
            pos[i] -= 1;
            const uint64_t dec = 1ull << P.kshift[i];
            const int w = KW == 1 ? 0 : P.kword[i];
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

template <int N, int KW>
__global__ void walk_kernel(const DevProblem *__restrict__ Pp, const uint64_t *__restrict__ table, uint64_t cap_mask,
                            const uint64_t *__restrict__ start, int max, int local_only,
                            int32_t *__restrict__ masks, uint64_t *__restrict__ last_key, int *__restrict__ info,
                            const int *__restrict__ gate)
{
    if (gate && *(volatile const int *)gate != 1)  // see queue_census_kernel
        return;
    walk_chain<N, KW>(Pp, table, cap_mask, start, max, local_only, masks, last_key, info);
}

// The backtrace walk many steps per memory round trip (one shard; 1-word
// keys of 2..6 sequences, 2-word keys of 7 or 8; same result as walk_kernel
// with local_only = 0).  Most columns of an alignment hold no gap: their
// parent mask steps back in every sequence at once.  One wave: lane j fetches the first probe line of the node
// j such steps behind the current one (lane 0: the node itself).  The records
// that came back tell in one ballot how far the path keeps to that diagonal;
// the first record with another mask, if it is at hand, is the round's last
// step, and the next round starts from where it leads.  Nothing in a round
// is serial but the one memory latency (~0.5 us): no step-by-step chain (a
// store and a dependent broadcast per step cost 160 ns each), and every
// lane's mask goes out in one store.  A node missing from its first line (a
// displaced key, rare at the table's load) is looked up along its probe
// chain when it is the round's first, and ends the round before it otherwise.
// (fixed N: 1-word keys of 2..6 sequences, 2-word keys of 7 or 8)
__host__ __device__ constexpr bool walk_ahead_ok(int n, int kw)
{
    return (kw == 1 && n >= 2 && n <= 6) || (kw == 2 && n >= 7 && n <= 8);
}

template <int N, int KW>
__device__ __forceinline__ void walk2_chain(const DevProblem *__restrict__ Pp, const uint64_t *__restrict__ table,
                                            uint64_t cap_mask, const uint64_t *__restrict__ start, int max,
                                            int32_t *__restrict__ masks, uint64_t *__restrict__ last_key,
                                            int *__restrict__ info, unsigned long long *dbg = nullptr)
{
    static_assert(N >= 2 && KW >= 1 && KW <= 2, "fixed N; 1-word keys by the line, 2-word keys by the slot");
#ifdef PASTAR_PHASE_TIMERS
    const unsigned long long w_t0 = device_clock();
    unsigned long long w_t1 = 0, w_t2 = 0, w_rounds = 0, w_fetch = 0;
#endif
    constexpr int SW = slot_words<KW>();
    constexpr int LS = KW == 1 ? line_slots<1>() : 1;  // slots compared: a 1-word key's probe line, a 2-word key's first slot
    constexpr uint32_t kFull = (1u << N) - 1;  // the mask of a step back in every sequence at once
    const DevProblem &Pg = *Pp;
    const KConst<N, KW> P = load_kconst<N, KW>(Pg);
    const int lane = lane_id();
    // one step back in every sequence, and this lane's `lane` of them
    // (a sequence's position is a field of one key word: no borrow crosses words)
    uint64_t diag[KW], dec[KW], origin[KW], key[KW];
#pragma unroll
    for (int k = 0; k < KW; k++) {
        diag[k] = 0;
#pragma unroll
        for (int i = 0; i < N; i++)
            if (KW == 1 || P.kword[i] == k)
                diag[k] += 1ull << P.kshift[i];
        dec[k] = diag[k] * (uint64_t)lane;
        origin[k] = Pg.origin_key[k];
        key[k] = start[k];  // uniform
    }
    auto same = [](const uint64_t (&x)[KW], const uint64_t (&y)[KW]) {
        bool eq = true;
#pragma unroll
        for (int k = 0; k < KW; k++)
            eq &= x[k] == y[k];
        return eq;
    };
    int steps = 0, status = 0;
    while (status == 0) {
#ifdef PASTAR_PHASE_TIMERS
        if (w_rounds == 0)
            w_t1 = device_clock();
        if (w_rounds == 1)
            w_t2 = device_clock();
        w_rounds++;
        const unsigned long long w_r0 = device_clock();
#endif
        if (same(key, origin)) {
            status = 1;
            break;
        }
        if (steps >= max) {
            status = 2;
            break;
        }
        int pos[N];
        decode_key<N, KW>(P, N, key, pos);
        bool valid = true;  // the node `lane` steps down the diagonal exists
#pragma unroll
        for (int i = 0; i < N; i++)
            if (pos[i] < lane)
                valid = false;
        uint64_t ck[KW];  // lane 0: the node itself
#pragma unroll
        for (int k = 0; k < KW; k++)
            ck[k] = key[k] - dec[k];
        uint64_t best = ~0ull;
        bool found = false;
        if (valid) {
            const uint64_t *line = table + probe_start<KW>(ck, cap_mask) * SW;
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            if constexpr (KW == 1) {
                u64x2 v[LS];
#pragma unroll
                for (int t = 0; t < LS; t++)
                    v[t] = *reinterpret_cast<const u64x2 *>(line + t * SW);  // key, best
#pragma unroll
                for (int t = 0; t < LS; t++)
                    if (!found && v[t].x == ck[0]) {
                        best = v[t].y;
                        found = true;
                    }
            } else {
                const u64x2 kv = *reinterpret_cast<const u64x2 *>(line);  // key words
                const uint64_t bv = line[KW];
                if (kv.x == ck[0] && kv.y == ck[KW - 1]) {
                    best = bv;
                    found = true;
                }
            }
        }
        if (!(__ballot(found) & 1ull)) {  // (uniform; the rare path for 1-word keys, one node in a few for 2-word keys)
            const int64_t s = lookup<KW>(table, cap_mask, key);
            if (s < 0) {
                status = -1;
                break;
            }
            if (lane == 0) {
                best = table[(uint64_t)s * SW + KW];
                found = true;
            }
        }
#ifdef PASTAR_PHASE_TIMERS
        if (w_rounds > 1)
            w_fetch += device_clock() - w_r0;
#endif
        const uint32_t m = (uint32_t)best;  // the parent mask of this lane's node
        const uint64_t hit = __ballot(found);
        // (the origin's record carries the full mask too: it has no parent)
        const uint64_t full = __ballot(found && m == kFull && !same(ck, origin));
        // (uniform from here) the run of full steps from the node on; it ends
        // at the origin at the latest
        const int run = full == ~0ull ? 64 : __builtin_ctzll(~full);
        int count = run;
        uint64_t next[KW];
#pragma unroll
        for (int k = 0; k < KW; k++)
            next[k] = key[k] - diag[k] * (uint64_t)run;
        if (!same(next, origin) && run < 64 && ((hit >> run) & 1ull)) {
            // the record that ends the run is at hand: the round's last step
            const uint32_t ml = (uint32_t)bcast_lane((int)m, run);
            if (ml == 0 || ml > kFull) {
                status = -1;  // no such parent
                break;
            }
            count++;
#pragma unroll
            for (int i = 0; i < N; i++)
                if ((ml >> i) & 1) {
#pragma unroll
                    for (int k = 0; k < KW; k++)
                        if (KW == 1 || P.kword[i] == k)
                            next[k] -= 1ull << P.kshift[i];
                }
        }
        if (steps + count > max) {
            status = 2;
            break;
        }
        if (lane < count)
            masks[steps + lane] = (int32_t)m;
        steps += count;
#pragma unroll
        for (int k = 0; k < KW; k++)
            key[k] = next[k];
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < KW; k++)
            last_key[k] = key[k];
        info[0] = steps;
        info[1] = status;
#ifdef PASTAR_PHASE_TIMERS
        if (dbg) {  // diagnostics: set-up, the first round trip, the rest (device clock ticks), round trips
            dbg[0] = w_t1 - w_t0;
            dbg[1] = w_t2 - w_t1;
            dbg[2] = device_clock() - w_t2;
            dbg[10] = w_rounds;
            dbg[12] = w_fetch;  // of the rest: a round's start to its records' arrival
        }
#endif
    }
}

template <int N, int KW>
__global__ __launch_bounds__(64) void walk2_kernel(const DevProblem *__restrict__ Pp, const uint64_t *__restrict__ table,
                                                   uint64_t cap_mask, const uint64_t *__restrict__ start, int max,
                                                   int32_t *__restrict__ masks, uint64_t *__restrict__ last_key,
                                                   int *__restrict__ info, const int *__restrict__ gate)
{
    if (gate && *(volatile const int *)gate != 1)  // see queue_census_kernel
        return;
    walk2_chain<N, KW>(Pp, table, cap_mask, start, max, masks, last_key, info);
}

// The end of a one-shard graph replay in one launch (in place of the census,
// the walk and a pack of the results; each small launch costs ~4.5 us of
// stream time even when it has nothing to do).  Not finished (status != 1):
// block 0 writes the control block and the goal to pinned host memory.
// Finished: blocks 1.. count the open list's queue entries
// (queue_census_kernel), block 0's first wave walks the goal's parent chain
// (walk2_chain, or walk_chain on one lane), and the last block to arrive
// writes the control block, the goal, the census and the walk's {steps,
// status} and masks to pinned host memory.
struct TailArgs {
    const DevProblem *P;
    const uint64_t *table;
    uint64_t cap_mask;
    const uint64_t *goal_key;
    int max;
    int32_t *masks;
    uint64_t *last_key;
    int *info;
    const Queues *q;
    unsigned long long *census;
    const Ctl *ctl;
    const int *goal;
    unsigned *arrive;  // [0] zero between launches; [1] tail launches so far (the completion word's value)
    Ctl *h_ctl;
    int *h_goal;
    unsigned long long *h_census;
    int *h_info;
    int32_t *h_masks;
    uint32_t *h_done;  // set to the launch's number after everything above is in host memory
};

__device__ __forceinline__ void tail_done(const TailArgs &t)
{
    __syncthreads();  // the block's host writes issued
    if (threadIdx.x == 0) {
        // (one thread per launch comes here, launches run in stream order)
        const unsigned ticket = t.arrive[1] + 1;
        t.arrive[1] = ticket;
        __threadfence_system();
        __hip_atomic_store(t.h_done, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ void tail_copy_ctl(const TailArgs &t)
{
    const uint32_t *src = reinterpret_cast<const uint32_t *>(t.ctl);
    uint32_t *dst = reinterpret_cast<uint32_t *>(t.h_ctl);
    for (int k = threadIdx.x; k < (int)(sizeof(Ctl) / 4); k += blockDim.x)
        dst[k] = ld_agent(&src[k]);
    if (threadIdx.x == 0)
        *t.h_goal = ld_agent(t.goal);
}

template <int N, int KW>
__global__ __launch_bounds__(kBlock) void tail_kernel(TailArgs t)
{
    if (ld_agent(&t.ctl->status) != 1) {
        if (blockIdx.x == 0) {
            tail_copy_ctl(t);
            tail_done(t);
        }
        return;
    }
#ifdef PASTAR_PHASE_TIMERS
    const unsigned long long tail_t0 = device_clock();
#endif
    if (blockIdx.x == 0) {
        if (threadIdx.x < 64) {
            constexpr bool kTwo = walk_ahead_ok(N, KW);
            if constexpr (kTwo)
#ifdef PASTAR_PHASE_TIMERS
                walk2_chain<kTwo ? N : 2, kTwo ? KW : 1>(t.P, t.table, t.cap_mask, t.goal_key, t.max, t.masks, t.last_key,
                                                         t.info, t.h_census + 5);
#else
                walk2_chain<kTwo ? N : 2, kTwo ? KW : 1>(t.P, t.table, t.cap_mask, t.goal_key, t.max, t.masks, t.last_key,
                                                         t.info);
#endif
            else if (threadIdx.x == 0)
                walk_chain<N, KW>(t.P, t.table, t.cap_mask, t.goal_key, t.max, 0, t.masks, t.last_key, t.info);
        }
    } else {
        unsigned long long s = 0;
        const int stride = (gridDim.x - 1) * blockDim.x;
        for (int k = (blockIdx.x - 1) * blockDim.x + threadIdx.x; k < kBuckets * kSub; k += stride)
            s += t.q->W[k / kSub][k % kSub] - t.q->R[k / kSub][k % kSub];
        s = wave_sum(s);
        if (lane_id() == 0 && s)
            atomicAdd(t.census, s);
    }
    __shared__ int last;
    __syncthreads();
#ifdef PASTAR_PHASE_TIMERS
    const unsigned long long tail_t1 = device_clock();
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // diagnostics: the walk's start and end
        t.h_census[13] = tail_t0;
        t.h_census[14] = tail_t1;
    }
#endif
    if (threadIdx.x == 0) {
        __threadfence();  // the walk's masks and info, the census adds: visible to the last block
        last = atomicAdd(t.arrive, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last)
        return;
    __threadfence();
#ifdef PASTAR_PHASE_TIMERS
    // diagnostics: the last block's start, its work done, the fences passed, the copies issued (device clock ticks)
    if (threadIdx.x == 0) {
        t.h_census[8] = tail_t0;
        t.h_census[9] = tail_t1;
        t.h_census[10] = device_clock();
        t.h_census[12] = blockIdx.x;
    }
#endif
    tail_copy_ctl(t);
    if (threadIdx.x < 5)
        t.h_census[threadIdx.x] = ld_agent(&t.census[threadIdx.x]);
    const int steps = ld_agent(&t.info[0]);
    if (threadIdx.x < 2)
        t.h_info[threadIdx.x] = ld_agent(&t.info[threadIdx.x]);
    const int n = steps < t.max ? steps : t.max;
    for (int k = threadIdx.x; k < n; k += blockDim.x)
        t.h_masks[k] = ld_agent(&t.masks[k]);
    if (threadIdx.x == 0)
        *t.arrive = 0;
#ifdef PASTAR_PHASE_TIMERS
    if (threadIdx.x == 0)
        t.h_census[11] = device_clock();
#endif
    tail_done(t);
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

}  // namespace dev
}  // namespace pastar
