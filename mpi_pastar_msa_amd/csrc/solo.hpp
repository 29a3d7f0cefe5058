// solo.hpp -- LDS-resident search of a small problem (DESIGN.md §4 "Solo
// path").
//
// When the search form of the pair tables (HC) and a node table of a few
// thousand slots fit in one CU's 160 KB of LDS (PF08184: 3 x 60 x 60 cells,
// 86 KB), one workgroup runs the whole search in a single launch, with no
// global atomics and no grid-wide step boundary:
//   1. PairAlign::Align (PairAlign.cpp:107-171) of every pair, one wave per
//      pair, written straight into LDS: the band sweep of
//      pairalign_wave_kernel (DPP lane shifts, bands of 64 rows) in weighted
//      units (w * H; min and + commute with w >= 0, so the cells equal the
//      batched engine's H * w bit for bit)
//   2. the A* (worker_inner, PAStar.cpp:320-401) on wave 0 alone: each level
//      expands every open entry of the lowest live f bucket, as the batched
//      engine's select does (kernels.hpp select_block), with the same
//      relaxation (g << 32 | parent mask, atomicMin: ties keep the smaller
//      mask), staleness and closed rules; the search ends when no entry is
//      left at or below the goal's bucket (check_stop, PAStar.cpp:480-547)
//   3. the backtrace (backtrace.cpp:47-69), masks to pinned host memory, then
//      the result record and the completion word the host watches
//   4. the node table dumped to HBM in the batched engine's slot layout (KW =
//      1 keys; the solo probe rule, solo_lookup_kernel), for
//      pastar_gpu_closed_lookup, after the result is published
// Only the reference's equal gap costs (Cost.h:13) and coordinates that pack
// into 31 bits take this path (keys and their hash are then 32-bit
// arithmetic: the level loop is instruction-bound); the host falls back to
// the batched engine on a capacity overflow.
#pragma once

#include "kernels.hpp"

namespace pastar {
namespace dev {

constexpr int kSoloThreads = 256;   // 4 waves: PairAlign one pair per wave, the search on wave 0
constexpr int kSoloLds = 160 * 1024;
constexpr int kSoloMaxCapLog2 = 12;  // node table slots (LDS), at most
constexpr int kSoloMinCapLog2 = 8;
// per node-table slot: key (4 B), best (8), {h, closed g} (8), a pile entry
// (8), and 2 x 1/4 of a 16-B batch entry (the current and the next level)
constexpr int kSoloSlotBytes = 36;
constexpr int kSoloKeyBits = 31;  // packed coordinate bits; bit 31 marks a used slot

struct SoloOut {
    int status;       // 1 optimum, 2 capacity exceeded, 3 open list exhausted, 4 level limit
    int score;
    int levels;
    int path_len;     // backtrace masks written (from the goal backwards)
    int path_status;  // 1 origin reached, 2 broken
    int band_log2;
    int h0;
    int cap;
    unsigned long long expanded, reopen, generated, claimed, dropped, open_left;
    unsigned long long t_start, t_end;  // device clock (100 MHz)
    unsigned long long t_tables, t_search;  // PairAlign done, search done
    unsigned long long pile_cuts;           // levels that had to cut their batch from the pile
    unsigned long long phase[4];            // diagnostics (-DPASTAR_SOLO_PHASES): core clocks per level phase
};

struct SoloArgs {
    const DevProblem *P;
    SoloOut *out;
    int32_t *masks;   // [max_path] backtrace masks, goal first
    uint64_t *dump;   // [cap] 4-word slots (kernels.hpp table layout, KW = 1)
    const uint8_t *codes;  // DevProblem::codes / sub / alpha * alpha (no dependent load)
    const int32_t *sub;
    long long max_levels;
    int cap_log2, max_path, hc_cells, codes_len, alpha2;
    int off_prob, off_sub, off_codes, off_keys, off_best, off_hcl, off_open, off_batch, off_subw;  // LDS bytes
    int band_log2;  // < 0: the engine's automatic band (pastar_gpu.hip estimate_band_log2)
    uint32_t *done;  // pinned host word: set to `ticket` after every result is written
    uint32_t ticket;
};

// LDS pointers carry their address space, so every access is a ds_*
// instruction (a generic pointer turns into flat loads that wait on both the
// vector-memory and the LDS counters)
#define SOLO_LDS __attribute__((address_space(3)))

// LDS element types are clang vectors (HIP's int2 / int4 structs cannot be
// assigned through an address-space-qualified pointer)
typedef int solo_v2 __attribute__((ext_vector_type(2)));
typedef int solo_v4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ SOLO_LDS T *lds_at(unsigned char *smem, int off)
{
    return (SOLO_LDS T *)(smem + off);
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// PairAlign of pair p by one wave into the LDS table T (search form HC: {w *
// H, w * cost}), equal gap costs: the EQ_GAPS sweep of pairalign_wave_kernel
// in weighted units.  Bands of 64 rows run one after the other on the same
// wave; lane 63 of band k reads the row below from band k - 1's top row in T.
__device__ __forceinline__ void solo_pairalign(const SOLO_LDS DevProblem &P, int p, SOLO_LDS solo_v2 *HCl,
                                               const SOLO_LDS int *sub, const SOLO_LDS uint8_t *codes,
                                               SOLO_LDS int *subw, SOLO_LDS solo_v2 *sink)
{
    const int lane = lane_id();
    const int x = P.pair_x[p], y = P.pair_y[p], wgt = P.weight[p];
    const int L1 = P.len[x], L2 = P.len[y], W = L2 + 1, alpha = P.alpha;
    const int GO = P.gap_open * wgt;
    // the wave's copy of the distance table, pre-weighted: no multiply in
    // the sweep
    for (int k = lane; k < alpha * alpha; k += 64)
        subw[k] = sub[k] * wgt;
    lds_fence();
    const SOLO_LDS uint8_t *s1 = codes + P.seq_off[x];
    const SOLO_LDS uint8_t *s2 = codes + P.seq_off[y];
    SOLO_LDS solo_v2 *T = HCl + P.h_off[p];
    const int nbands = L1 / 64 + 1;
    for (int band = 0; band < nbands; band++) {
        const int bottom = L1 - 64 * band;
        const int i = bottom - (63 - lane);
        const bool row_ok = i >= 0;
        const int cx = row_ok ? (int)s1[i] : 0;  // code 0 at i == L1 (string end)
        const SOLO_LDS int *crow = subw + cx * alpha;
        const bool last_row = i == L1;
        const SOLO_LDS solo_v2 *below = T + (bottom + 1) * W;  // band - 1's top row (band > 0)
        SOLO_LDS solo_v2 *Trow = T + (row_ok ? i : 0) * W;
        int m = kPaInf, down = kPaInf, diag = 0;
        int j = L2 + 63 - lane;
        int cost = (j >= 0 && j <= L2) ? crow[s2[j]] : 0;
        // the band's top row (lane 63 - min(63, bottom)) lags lane 63 by
        // min(63, bottom) steps: a band of few rows sweeps only that much
        // past the last column
        const int nsteps = L2 + 1 + (bottom < 63 ? bottom : 63);
        // a chunk's costs are read one chunk ahead and its codes two ahead,
        // so the sweep does not wait on the two dependent LDS reads; reads
        // past the table only feed cells outside it (unclamped, as in
        // pairalign_wave_kernel)
        int nc[kPaChunk], code[kPaChunk];
#pragma unroll
        for (int u = 0; u < kPaChunk; u++)
            nc[u] = crow[s2[j - u - 1]];
#pragma unroll
        for (int u = 0; u < kPaChunk; u++)
            code[u] = s2[j - kPaChunk - u - 1];
        for (int t0 = 0; t0 < nsteps; t0 += kPaChunk) {
            const int j0 = j;
            // lb is lane 63's row below (+inf under the table), the old value
            // of the DPP shift
            int lb[kPaChunk], ncn[kPaChunk];
#pragma unroll
            for (int u = 0; u < kPaChunk; u++) {
                lb[u] = band > 0 ? below[j0 - u].x : kPaInf;
                ncn[u] = crow[code[u]];
                code[u] = s2[j0 - 2 * kPaChunk - u - 1];
            }
            solo_v2 cb[kPaChunk];
#pragma unroll
            for (int u = 0; u < kPaChunk; u++, j--) {
                const int cost_here = cost;
                cost = nc[u];
                diag = down;
                down = __builtin_amdgcn_update_dpp(lb[u], m, 0x130, 0xf, 0xf, false);
                int mm = (down < m ? down : m) + GO;
                const int c2 = diag + cost_here;
                mm = c2 < mm ? c2 : mm;
                mm = (last_row && t0 + u == 0) ? 0 : mm;  // the corner (L1, L2)
                cb[u] = solo_v2{mm, cost_here};
                m = j <= L2 ? mm : m;  // only the columns right of the table stay +inf
            }
            // cells outside the table go to this lane's sink word: every
            // store is unconditional (no exec-mask branches)
#pragma unroll
            for (int u = 0; u < kPaChunk; u++) {
                const int jj = j0 - u;
                SOLO_LDS solo_v2 *dst = row_ok && (unsigned)jj <= (unsigned)L2 ? Trow + jj : sink + lane;
                *dst = cb[u];
            }
#pragma unroll
            for (int u = 0; u < kPaChunk; u++)
                nc[u] = ncn[u];
        }
        lds_fence();  // band k's top row lands before band k + 1 reads it
    }
}

// A node's best = g << 32 | parent mask << 16 | parent slot.  The minimum
// over relaxations orders by (g, mask) exactly as the batched engine's g << 32
// | mask (a (g, mask) pair fixes the parent's coordinate, hence its slot), and
// the backtrace follows parent slots without hashing.
__device__ __forceinline__ uint64_t solo_best(int g, int mask, int pslot)
{
    return ((uint64_t)(uint32_t)g << 32) | ((uint64_t)(uint32_t)mask << 16) | (uint32_t)pslot;
}

// Multiplicative hash of a 32-bit key (Fibonacci hashing: the top cap_log2
// bits of key * 2^32 / phi), linear probing.  solo_lookup_kernel uses the same.
__host__ __device__ __forceinline__ uint32_t solo_hash(uint32_t key, int cap_log2)
{
    return (key * 0x9E3779B1u) >> (32 - cap_log2);
}

// Relax (key, g, parent mask, parent slot) into the LDS node table: the
// batched engine's rule (device.hpp relax) on one wave, in one LDS round trip
// when the first probe settles it: a CAS claims the key's slot (and doubles
// as the probe read), the slot's best is read right behind it, and the new
// best goes in by a non-returning atomic min.  improved: g strictly below the
// best read.  Two lanes of one wave relaxing the same key in the same round
// may then both see the older best; the one with the larger g leaves a stale
// entry (dropped when popped), equal g's an entry expanded twice (counted as
// a reopening) -- the node's final best is the exact minimum either way.
__device__ __forceinline__ int solo_relax(SOLO_LDS uint32_t *keys, SOLO_LDS uint64_t *best, SOLO_LDS solo_v2 *hcl,
                                          int cap_log2, uint32_t key, int g, int mask, int pslot, int h,
                                          bool &improved, bool &claimed)
{
    const uint32_t cmask = (1u << cap_log2) - 1u;
    uint32_t idx = solo_hash(key, cap_log2);
    // the first probe straight-line (the table stays at most 3/4 full, most
    // relaxes settle here); only a wave with a lane on an occupied slot
    // enters the probing loop, so the common path carries no loop-exit mask
    // bookkeeping
    uint32_t prev = 0;
    __hip_atomic_compare_exchange_strong(&keys[idx], &prev, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    uint64_t seen = best[idx];  // after this instruction's claims (in-order LDS)
    bool hit = prev == 0 || prev == key;
    if (__builtin_expect(__ballot(!hit) != 0ull, 0)) {
        for (uint32_t probe = 1; !hit && probe <= cmask; probe++) {
            idx = (idx + 1) & cmask;
            prev = 0;
            __hip_atomic_compare_exchange_strong(&keys[idx], &prev, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            seen = best[idx];
            hit = prev == 0 || prev == key;
        }
        if (!hit) {
            improved = claimed = false;
            return -1;
        }
    }
    // unconditional stores (no exec-mask branches): h is the key's own, so
    // rewriting it is harmless, and a min that does not lower is a no-op
    claimed = prev == 0;
    hcl[idx].x = h;
    const uint64_t nb = solo_best(g, mask, pslot);
    improved = nb < seen && (uint32_t)(seen >> 32) > (uint32_t)g;
    __hip_atomic_fetch_min(&best[idx], nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (int)idx;
}

__device__ __forceinline__ int solo_lookup(const SOLO_LDS uint32_t *keys, int cap_log2, uint32_t key)
{
    const uint32_t cmask = (1u << cap_log2) - 1u;
    uint32_t idx = solo_hash(key, cap_log2);
    for (uint32_t probe = 0; probe <= cmask; probe++) {
        const uint32_t k = keys[idx];
        if (k == key)
            return (int)idx;
        if (k == 0)
            return -1;
        idx = (idx + 1) & cmask;
    }
    return -1;
}

// The backtrace by pointer jumping (backtrace.cpp:47-69 follows the parent
// chain one node at a time): level j of `anc` holds every slot's 2^j-th
// ancestor, built by all four waves from the parent slots in the best words
// (the origin, empty slots and broken links point to themselves).  Eight
// levels of C 16-bit slots take the pile and batch areas (16 B per slot),
// free once the search is over.  Every wave of the block must call it.
constexpr int kLiftLevels = 8;

__device__ __forceinline__ void solo_lift_levels(const SOLO_LDS uint32_t *keys, const SOLO_LDS uint64_t *best,
                                                 SOLO_LDS uint16_t *anc, int C, int origin_slot)
{
    for (int s = threadIdx.x; s < C; s += kSoloThreads) {
        const int p = (int)(best[s] & 0xffff);
        anc[s] = (uint16_t)(keys[s] == 0 || s == origin_slot || p >= C ? s : p);
    }
    __syncthreads();
    for (int j = 1; j < kLiftLevels; j++) {
        const SOLO_LDS uint16_t *prev = anc + (j - 1) * C;
        SOLO_LDS uint16_t *cur = anc + j * C;
        for (int s = threadIdx.x; s < C; s += kSoloThreads)
            cur[s] = prev[prev[s]];
        __syncthreads();
    }
}

// The node table to HBM (kernels.hpp slot layout: key word with bit 63 set,
// g << 32 | mask, closed | h << 32; the solo probe order), by threads
// first, first + stride, ...
__device__ __forceinline__ void solo_dump(const SOLO_LDS uint32_t *keys, const SOLO_LDS uint64_t *best,
                                          const SOLO_LDS solo_v2 *hcl, int C, uint64_t *dump, int first, int stride)
{
    ulonglong2 *d = reinterpret_cast<ulonglong2 *>(dump);
    for (int k = first; k < C; k += stride) {
        const uint32_t key = keys[k];
        const uint64_t b = best[k];
        const solo_v2 v = hcl[k];
        const uint64_t k64 = key ? (kMark | (key & 0x7fffffffu)) : 0;
        const uint64_t bm = b == ~0ull ? b : ((b & 0xffffffff00000000ull) | ((b >> 16) & 0xffff));
        d[2 * k] = make_ulonglong2(k64, bm);
        d[2 * k + 1] = make_ulonglong2((uint64_t)(uint32_t)v.y | ((uint64_t)(uint32_t)v.x << 32), 0ull);
    }
}

// A batch entry carries the parent as queued, {key, slot, g, f}, so a level
// reads its parents in one 16-B LDS load and their pair cells in the next
// round trip.  A pile entry is {slot, f}.
typedef solo_v4 SoloEntry;

template <int N>
__device__ __forceinline__ void solo_body(const SoloArgs &a)
{
    static_assert(N >= 2 && N <= 8, "solo path: 2..8 sequences");
    constexpr int NP = N * (N - 1) / 2;
    constexpr int MASKS = 1 << N;
    constexpr int LPN = MASKS < 64 ? MASKS : 64;  // lanes per parent
    constexpr int PPW = 64 / LPN;                 // parents per pass
    constexpr int ROUNDS = MASKS / LPN;           // child rounds per parent
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const unsigned long long t_start = device_clock();
    const int tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    SOLO_LDS DevProblem *Pl = lds_at<DevProblem>(smem, a.off_prob);
    SOLO_LDS solo_v2 *HCl = lds_at<solo_v2>(smem, 0);
    SOLO_LDS int *sub = lds_at<int>(smem, a.off_sub);
    SOLO_LDS uint8_t *codes = lds_at<uint8_t>(smem, a.off_codes);
    SOLO_LDS uint32_t *keys = lds_at<uint32_t>(smem, a.off_keys);
    SOLO_LDS uint64_t *best = lds_at<uint64_t>(smem, a.off_best);
    SOLO_LDS solo_v2 *hcl = lds_at<solo_v2>(smem, a.off_hcl);  // {h, closed g}
    SOLO_LDS solo_v2 *pile = lds_at<solo_v2>(smem, a.off_open);  // {slot, f}
    SOLO_LDS SoloEntry *bat = lds_at<SoloEntry>(smem, a.off_batch);  // [2][C / 4]: this level, the next
    const int lgC = a.cap_log2;
    const int C = 1 << lgC;
    const int NBC = C >> 2;  // batch entries per level

    // 0. one round trip: the problem, the codes and the distance table into
    // LDS; the node table cleared
    {
        const int4 *src = reinterpret_cast<const int4 *>(a.P);
        SOLO_LDS solo_v4 *dst = (SOLO_LDS solo_v4 *)Pl;
        for (int k = tid; k < (int)(sizeof(DevProblem) / 16); k += kSoloThreads) {
            const int4 v = src[k];
            dst[k] = solo_v4{v.x, v.y, v.z, v.w};
        }
        for (int k = tid; k < a.codes_len; k += kSoloThreads)
            codes[k] = a.codes[k];
        for (int k = tid; k < a.alpha2; k += kSoloThreads)
            sub[k] = a.sub[k];
        for (int k = tid; k < C; k += kSoloThreads) {
            keys[k] = 0;
            best[k] = ~0ull;
            hcl[k] = solo_v2{0, kIntMax};
        }
    }
    static_assert(sizeof(DevProblem) % 16 == 0, "DevProblem staged in 16-B words");
    __syncthreads();
    const SOLO_LDS DevProblem &P = *Pl;

    // 1. PairAlign, pair p on wave p % 4
    SOLO_LDS int *subw = lds_at<int>(smem, a.off_subw) + wave * (a.alpha2 + 1);
    // the sinks of the cells outside a table: 64 words per wave in the pile,
    // unused until the search (C >= 256 slots of 8 B)
    static_assert((1 << kSoloMinCapLog2) >= kSoloThreads, "a pile word per PairAlign lane");
    for (int p = wave; p < NP; p += kSoloThreads / 64)
        solo_pairalign(P, p, HCl, sub, codes, subw, pile + wave * 64);
    __syncthreads();
    // what waves 1..3 need from the search: its status, whether the
    // backtrace lifts, and then they dump the node table (4.)
    // (in the distance tables' staging area, free after PairAlign; no
    // static LDS beside the dynamic 160 KB).  Every branch around a block
    // barrier is on a scalar (readfirstlane): a branch the compiler took
    // for divergent would run the other side's s_barrier with exec = 0
    SOLO_LDS int *shv = lds_at<int>(smem, a.off_subw);  // [0] status, [1] lift
    SOLO_LDS uint16_t *anc = (SOLO_LDS uint16_t *)pile;  // the backtrace's ancestor levels
    const int origin_slot = (int)solo_hash(0x80000000u, lgC);
    if (__builtin_amdgcn_readfirstlane(wave) != 0) {
        __syncthreads();  // wave 0's search
        if (__builtin_amdgcn_readfirstlane(shv[1]))
            solo_lift_levels(keys, best, anc, C, origin_slot);
        if (__builtin_amdgcn_readfirstlane(shv[0]) == 1)
            solo_dump(keys, best, hcl, C, a.dump, tid - 64, kSoloThreads - 64);
        return;
    }
    const unsigned long long t_tables = device_clock();

    // 2. the search, wave 0 alone (no block barriers: a wave's LDS accesses
    // are processed in order)
    const int group = lane / LPN, glane = lane % LPN;
    int ksh[N], kbm[N], len[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        ksh[i] = P.kshift[i];
        kbm[i] = (1 << P.kbits[i]) - 1;
        len[i] = P.len[i];
    }
    int poff[NP], prow[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        poff[p] = (int)P.h_off[p];
        prow[p] = P.h_row[p];
    }
    // what a lane's child mask m = r * LPN + glane contributes, fixed for the
    // whole search: its key increment, per pair the cell offset of its corner
    // (bx, by) from the parent's cell, and the gap terms of the pairs where
    // not both sequences move (gap_open == gap_ext here; Node.cpp:130-152)
    uint32_t kinc[ROUNDS];
    int coff[ROUNDS][NP], gconst[ROUNDS];
    uint32_t both[ROUNDS];  // pairs where both move: the substitution cost of the parent's cell
#pragma unroll
    for (int r = 0; r < ROUNDS; r++) {
        const int m = r * LPN + glane;
        kinc[r] = 0;
#pragma unroll
        for (int i = 0; i < N; i++)
            kinc[r] += ((m >> i) & 1u) << ksh[i];
        gconst[r] = 0;
        both[r] = 0;
        int p = 0;
#pragma unroll
        for (int x = 0; x < N - 1; x++) {
#pragma unroll
            for (int y = x + 1; y < N; y++, p++) {
                const int bx = (m >> x) & 1, by = (m >> y) & 1;
                coff[r][p] = (bx ? prow[p] : 0) + by;
                if (bx & by)
                    both[r] |= 1u << p;
                else
                    gconst[r] += (bx | by ? P.gap_open : P.gap_gap) * P.weight[p];
            }
        }
    }
    // two levels per pass (N <= 3, one parent): lane (group c, glane m)
    // takes child c of the parent (group 0: child m) and, for c >= 1, that
    // child's child m; the first move's constants per lane
    constexpr bool TWO = ROUNDS == 1 && MASKS * MASKS <= 64;
    const int c1 = group ? group : glane;
    uint32_t kincA = 0;
    int coffA[NP], gconstA = 0;
    uint32_t bothA = 0;
    {
#pragma unroll
        for (int i = 0; i < N; i++)
            kincA += ((c1 >> i) & 1u) << ksh[i];
        int p = 0;
#pragma unroll
        for (int x = 0; x < N - 1; x++) {
#pragma unroll
            for (int y = x + 1; y < N; y++, p++) {
                const int bx = (c1 >> x) & 1, by = (c1 >> y) & 1;
                coffA[p] = (bx ? prow[p] : 0) + by;
                if (bx & by)
                    bothA |= 1u << p;
                else
                    gconstA += (bx | by ? P.gap_open : P.gap_gap) * P.weight[p];
            }
        }
    }
    const uint32_t goal_key = (uint32_t)P.goal_key[0] | 0x80000000u;
    const uint32_t origin_key = 0x80000000u;
    int h0 = 0;
#pragma unroll
    for (int p = 0; p < NP; p++)
        h0 += HCl[poff[p]].x;
    // the pair cells (pos_x, pos_y) of a parent
    auto pair_bases = [&](uint32_t key, int (&base)[NP], int &blocked) {
        int pos[N];
        blocked = 0;
#pragma unroll
        for (int i = 0; i < N; i++) {
            pos[i] = (int)((key >> ksh[i]) & (uint32_t)kbm[i]);
            blocked |= (pos[i] >= len[i]) << i;
        }
        int p = 0;
#pragma unroll
        for (int x = 0; x < N - 1; x++) {
#pragma unroll
            for (int y = x + 1; y < N; y++, p++)
                base[p] = poff[p] + pos[x] * prow[p] + pos[y];
        }
    };
    // (delta g, h) of this lane's child in round r (HeuristicHPair.cpp:74-86;
    // a valid child never leaves the table: no bound checks).  Branch-free:
    // every lane issues all 2P reads back to back (an invalid child's cells
    // are read and dropped), so a level waits for one LDS round trip.
    auto child_gh = [&](const int (&base)[NP], int r, int &dg, int &hh) {
        int hv[NP], cv[NP];
#pragma unroll
        for (int p = 0; p < NP; p++) {
            hv[p] = HCl[base[p] + coff[r][p]].x;
            cv[p] = HCl[base[p]].y;
        }
        dg = gconst[r];
        hh = 0;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            hh += hv[p];
            dg += ((both[r] >> p) & 1) ? cv[p] : 0;
        }
    };

    // the band: a power of two near 1/8 (N <= 6) or 1/4 (N >= 7) of the mean
    // f increase of the origin's children (pastar_gpu.hip estimate_band_log2)
    int w = a.band_log2;
    if (w < 0) {
        int base[NP], blocked;
        pair_bases(origin_key, base, blocked);
        int sum = 0, cnt = 0;
#pragma unroll
        for (int r = 0; r < ROUNDS; r++) {
            const int m = r * LPN + glane;
            if (group == 0 && m >= 1 && m < MASKS) {
                int dg, hh;
                child_gh(base, r, dg, hh);
                sum += dg + hh - h0;
                cnt++;
            }
        }
        sum = wave_sum_i32(sum);
        cnt = wave_sum_i32(cnt);
        long long band = cnt ? (long long)sum / cnt / (N >= 7 ? 4 : 8) : 1;
        band = band < 1 ? 1 : band;
        w = 0;
        while ((2ll << w) <= band * 4 / 3 && w < 24)
            w++;
    }
    auto bucket = [&](int f) {
        const int b = (f - h0) >> w;
        return b < 0 ? 0 : (b >= kBuckets ? kBuckets - 1 : b);
    };

    // seed the origin (Sequences::get_initial_node, Sequences.cpp:70-77)
    if (lane == 0) {
        keys[origin_slot] = origin_key;
        best[origin_slot] = solo_best(0, MASKS - 1, 0xffff);
        hcl[origin_slot] = solo_v2{h0, kIntMax};
        bat[0] = SoloEntry{(int)origin_key, origin_slot, 0, h0};
    }
    lds_fence();
    int cur = 0, nb = 1, npile = 0, bsel = 0, goal_g = kIntMax, status = 0, levels = 0, claimed_n = 1, cuts = 0;
    int expanded = 0, reopen = 0, generated = 0, dropped = 0;
    const int claim_limit = C - C / 4;  // load <= 75%
    const uint64_t below_me = (1ull << lane) - 1ull;
#ifdef PASTAR_SOLO_PHASES
    // phase k accumulates the core clocks from mark k-1 to mark k (mark 0:
    // from the previous level's mark 3); s_memtime is a scalar memory read,
    // so each mark also waits for the outstanding LDS operations
    unsigned long long ph_acc[4] = {0, 0, 0, 0}, ph_last = __builtin_amdgcn_s_memtime();
#define SOLO_PHASE_MARK(k)                                     \
    {                                                          \
        const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
        ph_acc[k] += _t - ph_last;                             \
        ph_last = _t;                                          \
    }
#else
#define SOLO_PHASE_MARK(k)
#endif
    // next-level entries handed over in registers (see the pass loop)
    bool hand = false;
    uint64_t hand_bits = 0;
    int hand_key = 0, hand_slot = 0, hand_g = 0, hand_f = 0;
    for (;;) {
        if (nb == 0) {
            hand = false;
            // the bucket is exhausted: cut the lowest one left in the pile
            // (at or below the goal's; check_stop, PAStar.cpp:480-547)
            if (npile == 0) {
                status = goal_g < kIntMax ? 1 : 3;
                break;
            }
            int fmin = kIntMax;
            for (int b0 = 0; b0 < npile; b0 += 256) {
                int f[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = b0 + u * 64 + lane;
                    f[u] = k < npile ? pile[k].y : kIntMax;
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    fmin = f[u] < fmin ? f[u] : fmin;
            }
            fmin = wave_min_i32(fmin);
            bsel = bucket(fmin);
            if (goal_g < kIntMax && bsel > bucket(goal_g)) {
                status = 1;
                break;
            }
            cuts++;
            int nkeep = 0;
            for (int b0 = 0; b0 < npile; b0 += 64) {
                const int k = b0 + lane;
                const solo_v2 e = k < npile ? pile[k] : solo_v2{0, 0};
                bool sel = k < npile && bucket(e.y) == bsel;
                const uint64_t bs = __ballot(sel);
                const int at = nb + __popcll(bs & below_me);
                sel = sel && at < NBC;
                const bool keep = k < npile && !sel;
                const uint64_t bk = __ballot(keep);
                if (keep)
                    pile[nkeep + __popcll(bk & below_me)] = e;
                if (sel)
                    bat[cur * NBC + at] = SoloEntry{(int)keys[e.x], e.x, e.y - hcl[e.x].x, e.y};
                nkeep += __popcll(bk);
                nb += __popcll(__ballot(sel));
            }
            npile = nkeep;
        }
        if (levels >= a.max_levels) {
            status = 4;
            break;
        }
        levels++;
        SOLO_PHASE_MARK(0);
        if constexpr (TWO) {
            if (nb == 1 && levels < a.max_levels) {
                // one parent X: this level and the next in one pass.  The
                // next level of the one-level pass would expand exactly X's
                // improved children of this bucket (its whole batch, all
                // current), so expanding them here is the same search.
                SoloEntry be4;
                if (hand) {
                    const int L = __ffsll((long long)hand_bits) - 1;
                    be4 = SoloEntry{__builtin_amdgcn_readlane(hand_key, L), __builtin_amdgcn_readlane(hand_slot, L),
                                    __builtin_amdgcn_readlane(hand_g, L), __builtin_amdgcn_readlane(hand_f, L)};
                } else {
                    be4 = bat[cur * NBC];
                }
                const uint32_t xkey = (uint32_t)be4.x;
                const int xslot = be4.y, xg = be4.z, xf = be4.w;
                int posX[N], blockedX = 0;
#pragma unroll
                for (int i = 0; i < N; i++) {
                    posX[i] = (int)((xkey >> ksh[i]) & (uint32_t)kbm[i]);
                    blockedX |= (posX[i] >= len[i]) << i;
                }
                // child c1's position: blocked coordinates of its own moves
                int blockedC = 0;
#pragma unroll
                for (int i = 0; i < N; i++)
                    blockedC |= (posX[i] + ((c1 >> i) & 1) >= len[i]) << i;
                int baseX[NP], baseC[NP];
                {
                    int p = 0;
#pragma unroll
                    for (int x = 0; x < N - 1; x++) {
#pragma unroll
                        for (int y = x + 1; y < N; y++, p++) {
                            baseX[p] = poff[p] + posX[x] * prow[p] + posX[y];
                            baseC[p] = baseX[p] + coffA[p];
                        }
                    }
                }
                // X's node words and every lane's cells in one LDS round trip
                const uint64_t pbest = best[xslot];
                const int closedX = hcl[xslot].y;
                int hvA[NP], cvX[NP], cvC[NP], hvB[NP];
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    hvA[p] = HCl[baseC[p]].x;
                    cvX[p] = HCl[baseX[p]].y;
                    cvC[p] = HCl[baseC[p]].y;
                    hvB[p] = HCl[baseC[p] + coff[0][p]].x;
                }
                int dg1 = gconstA, h1 = 0, dg2 = gconst[0], h2 = 0;
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    h1 += hvA[p];
                    dg1 += ((bothA >> p) & 1) ? cvX[p] : 0;
                    h2 += hvB[p];
                    dg2 += ((both[0] >> p) & 1) ? cvC[p] : 0;
                }
                const bool okX = (int)(pbest >> 32) == xg && xf < goal_g;
                if (lane == 0) {
                    if (okX) {
                        reopen += closedX != kIntMax;
                        hcl[xslot].y = xg;  // ClosedList[current.pos] (PAStar.cpp:351)
                    }
                    expanded += okX;
                    dropped += !okX;
                }
                // level L: X's children on group 0
                const bool v1 = okX && c1 >= 1 && !(c1 & blockedX);
                const uint32_t ck1 = xkey + kincA;
                const int g1 = xg + dg1, f1 = g1 + h1;
                bool imp1 = false, cl1 = false;
                int slot1 = 0;
                if (group == 0 && v1) {
                    slot1 = solo_relax(keys, best, hcl, lgC, ck1, g1, c1, xslot, h1, imp1, cl1);
                    if (slot1 < 0)
                        imp1 = false;
                }
                generated += group == 0 && v1;
                claimed_n += (int)__popcll(__ballot(cl1));
                if (__ballot(group == 0 && v1 && slot1 < 0))
                    status = 2;
                const bool goal1 = imp1 && ck1 == goal_key;
                if (__ballot(goal1))
                    goal_g = wave_min_i32(goal1 ? (g1 < goal_g ? g1 : goal_g) : goal_g);
                const bool live1 = imp1 && f1 < goal_g;
                const bool next1 = live1 && bucket(f1) <= bsel;
                // children past the bucket: to the pile
                const bool pile1 = live1 && !next1;
                const uint64_t bp1 = __ballot(pile1);
                if (pile1)
                    pile[npile + __popcll(bp1 & below_me)] = solo_v2{slot1, f1};
                npile += __popcll(bp1);
                // level L + 1: group c expands child c (lane c of group 0)
                const uint64_t nextbits = __ballot(group == 0 && next1);
                const bool exp_c = group >= 1 && ((nextbits >> group) & 1ull);
                const int slot_c = __shfl(slot1, group);
                if (exp_c && glane == 0) {
                    reopen += hcl[slot_c].y != kIntMax;
                    hcl[slot_c].y = g1;
                    expanded++;
                }
                const bool v2 = exp_c && glane >= 1 && !(glane & blockedC);
                const uint32_t ck2 = ck1 + kinc[0];
                const int g2 = g1 + dg2, f2 = g2 + h2;
                bool imp2 = false, cl2 = false;
                int slot2 = 0;
                if (v2) {
                    slot2 = solo_relax(keys, best, hcl, lgC, ck2, g2, glane, slot_c, h2, imp2, cl2);
                    if (slot2 < 0)
                        imp2 = false;
                }
                generated += v2;
                claimed_n += (int)__popcll(__ballot(cl2));
                if (__ballot(v2 && slot2 < 0))
                    status = 2;
                const bool goal2 = imp2 && ck2 == goal_key;
                if (__ballot(goal2))
                    goal_g = wave_min_i32(goal2 ? (g2 < goal_g ? g2 : goal_g) : goal_g);
                const bool live2 = imp2 && f2 < goal_g;
                const bool next2 = live2 && bucket(f2) <= bsel;
                const uint64_t bn = __ballot(next2);
                const int at = __popcll(bn & below_me);
                const bool in_next = next2 && at < NBC;
                SOLO_LDS SoloEntry *nxt2 = bat + (cur ^ 1) * NBC;
                if (in_next)
                    nxt2[at] = SoloEntry{(int)ck2, slot2, g2, f2};
                const uint64_t nbits = __ballot(in_next);
                const bool pile2 = live2 && !in_next;
                const uint64_t bp2 = __ballot(pile2);
                if (pile2)
                    pile[npile + __popcll(bp2 & below_me)] = solo_v2{slot2, f2};
                npile += __popcll(bp2);
                if (npile + 64 > C || claimed_n > claim_limit)
                    status = 2;
                if (nextbits)
                    levels++;  // the pass ran level L + 1 too
                if (status)
                    break;
                cur ^= 1;
                nb = __popcll(nbits);
                hand = nb <= PPW;
                hand_bits = nbits;
                hand_key = (int)ck2;
                hand_slot = slot2;
                hand_g = g2;
                hand_f = f2;
                SOLO_PHASE_MARK(3);
                continue;
            }
        }
        // expand the batch: PPW parents per pass, LPN lanes (child masks) each
        int nn = 0;
        SOLO_LDS SoloEntry *nxt = bat + (cur ^ 1) * NBC;
        const bool from_regs = hand;
        hand = ROUNDS == 1 && nb <= PPW;  // one pass: its next-level entries can stay in registers
        uint64_t next_bits = 0;
        int hk_key = 0, hk_slot = 0, hk_g = 0, hk_f = 0;
        for (int b0 = 0; b0 < nb && !status; b0 += PPW) {
            const int k = b0 + group;
            const bool active = k < nb;
            SoloEntry be4;
            if (from_regs) {
                // the previous level's single pass left its entries in the
                // lanes that produced them: entry e comes from the e-th set
                // bit of that pass's ballot (no LDS round trip)
                be4 = SoloEntry{0, 0, 0, 0};
                uint64_t bits = hand_bits;
#pragma unroll
                for (int e = 0; e < PPW; e++) {
                    if (!bits)
                        break;
                    const int L = __ffsll((long long)bits) - 1;
                    bits &= bits - 1;
                    const SoloEntry v = SoloEntry{__builtin_amdgcn_readlane(hand_key, L),
                                                  __builtin_amdgcn_readlane(hand_slot, L),
                                                  __builtin_amdgcn_readlane(hand_g, L),
                                                  __builtin_amdgcn_readlane(hand_f, L)};
                    be4 = group == e ? v : be4;
                }
            } else {
                be4 = bat[cur * NBC + (active ? k : 0)];
            }
            const struct {
                uint32_t key;
                int slot, g, f;
            } be = {(uint32_t)be4.x, be4.y, be4.z, be4.w};
            int base[NP], blocked;
            pair_bases(be.key, base, blocked);
            // the parent's node words and its children's pair cells in one
            // round trip (the cells of every round are read before the
            // staleness verdict)
            const uint64_t pbest = best[be.slot];
            const int closed = hcl[be.slot].y;
            int dgr[ROUNDS], hhr[ROUNDS];
#pragma unroll
            for (int r = 0; r < ROUNDS; r++)
                child_gh(base, r, dgr[r], hhr[r]);
            // current iff nobody has lowered the node's g since it was queued,
            // and below the best goal (a goal's f is its g)
            const bool ok = active && (int)(pbest >> 32) == be.g && be.f < goal_g;
            SOLO_PHASE_MARK(1);
            if (ok && glane == 0) {
                reopen += closed != kIntMax;
                hcl[be.slot].y = be.g;  // ClosedList[current.pos] (PAStar.cpp:351)
            }
            if (glane == 0) {
                expanded += ok;
                dropped += active && !ok;
            }
#pragma unroll
            for (int r = 0; r < ROUNDS; r++) {
                const int m = r * LPN + glane;
                const bool valid = ok && m >= 1 && m < MASKS && !(m & blocked);
                const int dg = dgr[r], hh = hhr[r];
                const uint32_t ck = be.key + kinc[r];
                const int cg = be.g + dg, cf = cg + hh;
                bool improved = false, cl = false;
                int slot = 0;
                if (valid) {
                    slot = solo_relax(keys, best, hcl, lgC, ck, cg, m, (int)be.slot, hh, improved, cl);
                    if (slot < 0)
                        improved = false;
                }
                SOLO_PHASE_MARK(2);
                generated += valid;
                claimed_n += (int)__popcll(__ballot(cl));
                if (__ballot(valid && slot < 0))
                    status = 2;
                // the improved children: this bucket's to the next level,
                // the rest to the pile (an improved child at or above the
                // goal's g can never be expanded: dropped here)
                const bool live = improved && cf < goal_g;
                const bool to_next = live && bucket(cf) <= bsel;
                const uint64_t bn = __ballot(to_next);
                const int at = nn + __popcll(bn & below_me);
                const bool in_next = to_next && at < NBC;
                if (in_next)
                    nxt[at] = SoloEntry{(int)ck, slot, cg, cf};
                next_bits |= __ballot(in_next);
                hk_key = (int)ck;
                hk_slot = slot;
                hk_g = cg;
                hk_f = cf;
                const bool to_pile = live && !in_next;
                const uint64_t bp = __ballot(to_pile);
                if (to_pile)
                    pile[npile + __popcll(bp & below_me)] = solo_v2{slot, cf};
                nn += __popcll(__ballot(in_next));
                npile += __popcll(bp);
                // the goal: its g is the candidate score (atomicMin in the
                // batched engine)
                const bool at_goal = improved && ck == goal_key;
                if (__ballot(at_goal))
                    goal_g = wave_min_i32(at_goal ? (cg < goal_g ? cg : goal_g) : goal_g);
                if (npile + 64 > C || claimed_n > claim_limit)
                    status = 2;
            }
        }
        if (status)
            break;
        cur ^= 1;
        nb = nn;
        hand = hand && nn <= PPW;
        hand_bits = next_bits;
        SOLO_PHASE_MARK(3);
        hand_key = hk_key;
        hand_slot = hk_slot;
        hand_g = hk_g;
        hand_f = hk_f;
    }
    const unsigned long long t_search = device_clock();
    const int e_all = wave_sum_i32(expanded), r_all = wave_sum_i32(reopen);
    const int gen_all = wave_sum_i32(generated), d_all = wave_sum_i32(dropped);

    // 3. the backtrace (backtrace.cpp:47-69), by pointer jumping or by the
    // walk.  Lifted: the goal's distance D to the origin by jumps of 2^j
    // (greedy from the top level: a jump is taken while it stays short of
    // the origin), then lane k finds the goal's k-th ancestor from the bits
    // of k, and its mask is the path's k-th
    int goal_slot = -1;
    if (status == 1)
        goal_slot = __builtin_amdgcn_readfirstlane(solo_lookup(keys, lgC, goal_key));
    // the lift costs ~8 levels x C / 256 slot updates per thread, the walk
    // ~85 ns per step (at least the longest sequence's length): the lift
    // when the path is surely longer than C / 32 steps (PF08184: 59 against
    // 32 at 1024 slots, tail 5.6 -> 3.6 us), else the walk
    int maxlen = 0;
#pragma unroll
    for (int i = 0; i < N; i++)
        maxlen = len[i] > maxlen ? len[i] : maxlen;
    const bool found = status == 1 && goal_slot >= 0 && goal_slot != origin_slot;
    const bool lift = __builtin_amdgcn_readfirstlane(found && maxlen * 32 > C);
    if (lane == 0) {
        shv[0] = status;
        shv[1] = lift ? 1 : 0;
    }
    __syncthreads();
    int path_len = 0, path_status = 0;
    if (status == 1)
        path_status = goal_slot == origin_slot ? 1 : 2;
    if (lift) {
        solo_lift_levels(keys, best, anc, C, origin_slot);
        constexpr int kTop = 1 << (kLiftLevels - 1);
        const SOLO_LDS uint16_t *top = anc + (kLiftLevels - 1) * C;
        int x = goal_slot, D = 0;
        while (top[x] != origin_slot && D < a.max_path) {
            x = top[x];
            D += kTop;
        }
        for (int j = kLiftLevels - 2; j >= 0; j--) {
            const int y = anc[j * C + x];
            if (y != origin_slot) {
                x = y;
                D += 1 << j;
            }
        }
        D = __builtin_amdgcn_readfirstlane(D + 1);  // x is now one step from the origin
        if (anc[x] == origin_slot && D <= a.max_path) {
            path_status = 1;
            path_len = D;
            for (int k = lane; k < D; k += 64) {
                int y = goal_slot, r = k;
                for (; r >= kTop; r -= kTop)
                    y = top[y];
#pragma unroll
                for (int j = 0; j < kLiftLevels - 1; j++)
                    if ((r >> j) & 1)
                        y = anc[j * C + y];
                a.masks[k] = (int)((best[y] >> 16) & 0xffff);
            }
        }
    } else if (found) {
        // the walk on scalars: every lane reads the same parent word, the
        // next one is requested before the step's bookkeeping (the read of
        // the origin's parent, slot 0xffff masked into the table, is issued
        // and dropped), and mask k waits in lane k % 64 until 64 of them go
        // to host memory in one store
        int slot = goal_slot, mreg = 0;
        uint64_t b = best[slot];
        while (path_len < a.max_path) {
            const int nxt = __builtin_amdgcn_readfirstlane((int)(b & 0xffff));
            const uint64_t bn = best[nxt & (C - 1)];
            mreg = lane == (path_len & 63) ? (int)((b >> 16) & 0xffff) : mreg;
            path_len++;
            if ((path_len & 63) == 0)
                a.masks[path_len - 64 + lane] = mreg;
            if (nxt == origin_slot) {
                path_status = 1;
                break;
            }
            b = bn;
        }
        if (lane < (path_len & 63))
            a.masks[(path_len & ~63) + lane] = mreg;
    }
    if (lane == 0) {
        SoloOut o;
        o.status = status;
        o.score = goal_g;
        o.levels = levels;
        o.path_len = path_len;
        o.path_status = path_status;
        o.band_log2 = w;
        o.h0 = h0;
        o.cap = C;
        o.expanded = (unsigned long long)e_all;
        o.reopen = (unsigned long long)r_all;
        o.generated = (unsigned long long)gen_all;
        o.claimed = (unsigned long long)claimed_n;
        o.dropped = (unsigned long long)d_all;
        o.open_left = (unsigned long long)(npile + nb);
        o.t_start = t_start;
        o.t_end = device_clock();
        o.t_tables = t_tables;
        o.t_search = t_search;
        o.pile_cuts = (unsigned long long)cuts;
#ifdef PASTAR_SOLO_PHASES
        for (int k = 0; k < 4; k++)
            o.phase[k] = ph_acc[k];
#else
        for (int k = 0; k < 4; k++)
            o.phase[k] = 0;
#endif
        *a.out = o;
        // the host may stop waiting as soon as it sees the ticket: the
        // result and the path are in host memory before it (system fence)
        __threadfence_system();
        __hip_atomic_store(a.done, a.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // 4. the node table dump runs on waves 1..3 (solo_dump), beside the
    // result's publication: the host has its answer meanwhile, and
    // pastar_gpu_closed_lookup's kernel is stream-ordered after this one
}

template <int N>
__global__ __launch_bounds__(kSoloThreads, 1) void solo_kernel(SoloArgs a)
{
    solo_body<N>(a);
}

// Many independent searches in one launch: workgroup b runs the search
// args[b] describes (its own problem, LDS layout, result areas), each whole
// in its CU's LDS as above.  The workgroups share nothing.
template <int N>
__global__ __launch_bounds__(kSoloThreads, 1) void solo_many_kernel(const SoloArgs *__restrict__ args)
{
    const SoloArgs a = args[blockIdx.x];
    solo_body<N>(a);
}

// Closed-list lookup in a solo search's dumped node table (kernels.hpp
// lookup_kernel's output: found, best, aux).
__global__ void solo_lookup_kernel(const uint64_t *__restrict__ dump, int cap_log2, const uint64_t *__restrict__ key_in,
                                   uint64_t *__restrict__ out)
{
    const uint32_t key = (uint32_t)(key_in[0] & 0x7fffffffu) | 0x80000000u;
    const uint32_t cmask = (1u << cap_log2) - 1u;
    uint32_t idx = solo_hash(key, cap_log2);
    out[0] = 0;
    for (uint32_t probe = 0; probe <= cmask; probe++) {
        const uint64_t *s = dump + (size_t)idx * 4;
        if (s[0] == 0)
            return;
        if (s[0] == key_in[0]) {
            out[0] = 1;
            out[1] = s[1];
            out[2] = s[2];
            return;
        }
        idx = (idx + 1) & cmask;
    }
}

}  // namespace dev
}  // namespace pastar
