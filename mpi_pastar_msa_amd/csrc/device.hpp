// device.hpp -- gfx950 device code of the PAStar frontier-expansion engine.
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   DevProblem   problem constants (pair list, weights, key packing), read by
//                uniform (scalar) loads
//   H            PairAlign suffix tables, one row-major (L_x+1)*(L_y+1) int32
//                block per pair
//   codes / sub  residues as small integer codes + code x code distance table
//   table        open-addressing node table (Open U Closed), one 32-B slot
//                (64 B for 4-word keys):
//                  word 0..KW-1  packed coordinate (bit 63 set = written)
//                  word KW       best = g << 32 | parent mask  (atomicMin)
//                  word KW+1     lo: closed_g (atomicMin), hi: h
//   queues       open list: f-bucketed FIFO queues of 8-B entries {slot, f}
//                (kernels.hpp "Search kernels")
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pastar {
namespace dev {

constexpr int kMaxN = 16;
constexpr int kMaxPairs = kMaxN * (kMaxN - 1) / 2;
constexpr int kBlock = 256;           // threads per block (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kTPerWave = 512;        // int2 pair-corner terms per wave (LDS), any N <= kMaxN
// terms one wave stages for a fixed N: 64 / min(2^N, 64) parents x 4P
// (<= 112 for N <= 8), so the search kernel's LDS allows 4+ blocks per CU
__host__ __device__ constexpr int terms_per_wave(int n)
{
    return n == 0 ? kTPerWave : (64 / ((1 << n) < 64 ? (1 << n) : 64)) * 4 * (n * (n - 1) / 2);
}
constexpr uint64_t kMark = 1ull << 63;  // key word written / occupied
constexpr int kMaxProbe = 1 << 16;
constexpr int kIntMax = 0x7fffffff;

// Bounded device waits.  A wave waits on another wave in three places: a
// queue store on the chunk id its reserver publishes (queue_store), a relax on
// the tail words of a multi-word key being published (relax), and a PairAlign
// band on the band below it.  Each waits at most a fixed number of polls;
// one that runs out ORs its site into the context's fault word and carries
// on without the datum (the entry is dropped, the cell is garbage), so every
// kernel still ends, and the host turns a non-zero fault word into
// PASTAR_EDEVWAIT naming the site.
enum { kSiteQueueStore = 1, kSiteRelaxTail = 2, kSitePairAlign = 4, kSiteSelftest = 8 };
constexpr unsigned kSpinLimit = 1u << 22;  // polls of ~0.1-1 us each


struct DevProblem {
    int n, npairs, kw, alpha;
    int gap_open, gap_ext, gap_gap;
    int hash_type, hash_shift, n_shards, shard, pad0;
    int len[kMaxN];
    int kword[kMaxN], kshift[kMaxN], kbits[kMaxN];
    uint64_t goal_key[4];
    uint64_t origin_key[4];
    int pair_x[kMaxPairs], pair_y[kMaxPairs], weight[kMaxPairs];
    int h_row[kMaxPairs];
    int64_t h_off[kMaxPairs];
    int64_t seq_off[kMaxN];
    const int32_t *H;
    const uint8_t *codes;
    const int32_t *sub;  // alpha x alpha
    // search form of the pair tables: cell (i, j) of pair p holds
    // {H_p[i][j] * w_p, cost(s_x[i], s_y[j]) * w_p} (cost 0 on the last row
    // and column, where the reference reads the string's '\0'), so one 8-B
    // gather serves both g and h
    const int2 *HC;
};

// Per-pair constants staged in LDS by every block that expands nodes.
struct PairConst {
    int x, y, w, row, lx, ly;
    int64_t off;
};

__device__ __forceinline__ void stage_pairs(const DevProblem &P, PairConst *pc)
{
    for (int p = threadIdx.x; p < P.npairs; p += blockDim.x) {
        const int x = P.pair_x[p], y = P.pair_y[p];
        PairConst k;
        k.x = x;
        k.y = y;
        k.w = P.weight[p];
        k.row = P.h_row[p];
        k.lx = P.len[x];
        k.ly = P.len[y];
        k.off = P.h_off[p];
        pc[p] = k;
    }
}

struct Entry {  // open-pile entry
    uint32_t slot;
    int32_t f;
};
// Partial expansion (search kernels): a parent whose children at or past a
// cutoff were left ungenerated goes back to the open list under the lowest f
// among them, marked by the sign bit of f (f itself is never negative: costs
// and h are sums of non-negative terms).  Taken again, it generates the
// children from that f on, under the node's best g at that time.
constexpr int32_t kPartialBit = (int32_t)0x80000000;
__host__ __device__ inline int32_t entry_f(const Entry &e) { return e.f & 0x7fffffff; }

// Per-step counters.  The counters every wave adds to are spread over
// kStatRows rows (row = global wave index % kStatRows): a single word takes
// one atomic per wave and saturates at ~88 atomics/us, which at 5-10 K waves
// per step would serialise for 50-100 us; select sums the rows.
constexpr int kStatRows = 64;
enum { kStExpanded, kStReopen, kStGenerated, kStClaimed, kStDropped, kStOvfTable, kStPartQueued, kStPartTaken, kStFields = 8 };
struct StepStats {
    // expanded: parents that passed the stale/closed checks; reopen; generated:
    // border-valid children; claimed: new table slots; dropped: stale or
    // pruned parents; ovf_table: node table probe limit hit; part_queued /
    // part_taken: parents queued again with children left, and taken again
    unsigned long long row[kStatRows][2 * kStFields];  // one 128-B line per row
    unsigned long long ovf_near;  // chunk pool exhausted
    unsigned long long ovf_far;   // sub-queue chunk table exhausted
    unsigned long long ovf_out;   // outbox ring capacity exceeded
    unsigned long long pad;
};

__device__ __forceinline__ unsigned long long *stat_row(StepStats *st, unsigned wave_global)
{
    return st->row[wave_global % kStatRows];
}

// Remote record sent to the owner shard over RCCL.  flags bit 0: the sender
// expands the node itself at this g (block-local continuation), so the owner
// records it as closed at g instead of queueing it.
template <int KW>
struct Remote {
    uint64_t key[KW];
    int32_t g, h, pmask, flags;
};
constexpr int kRecSenderExpands = 1;

// ---------------------------------------------------------------------------
// Shard exchange state (sharded search only).  Children owned by another
// shard go to a ring per destination (positions are 64-bit counters: w
// reserved by the expand kernel's appends, r consumed by the pack kernel).
// Each step the pack kernel moves up to `block_recs` records per destination
// from the ring into a fixed-size block {XHdr, records}; the blocks travel by
// a fixed-size all-to-all (RCCL grouped send/recv, or peer reads in an
// in-process shard group), so no count ever has to reach the host; what does
// not fit stays in the ring for the next step (the header says how much).
// The expand kernel runs on the main stream, pack / all-to-all / insert on
// the side stream; per-step hand-over values live in kXSlots slots indexed
// by step, because the main stream may run ahead of the side stream.
// ---------------------------------------------------------------------------
constexpr int kMaxShards = 8;
constexpr int kXSlots = 4;
// Every field but n is the same in all blocks a shard sends in one step, and
// is computed from values that no longer change once the step's pack kernel
// may run (StepInfo, the ring snapshot, the consumed positions): every shard
// therefore folds the same G headers and takes the same decision.
struct XHdr {
    unsigned long long n;            // records in this block
    unsigned long long sent_all;     // records the sender sends to all shards in this step
    unsigned long long backlog_all;  // records still waiting in the sender's rings after this step
    unsigned long long has_work;     // the sender's batch of this step was not empty
    unsigned long long fail;         // kFail* bits / 0x100 step limit / 0x200 fault: the sender cannot go on
    long long goal;                  // the sender's best goal g
    unsigned long long step;         // (diagnostics)
    unsigned long long low_b;        // low half: the sender's lowest live bucket (kBuckets: none); high
                                     // half: most records it had for one destination in this step
};
static_assert(sizeof(XHdr) == 64, "block header");

struct XState {
    // ---- appended to by every expand wave (atomics): own line ----
    alignas(128) unsigned long long w[kMaxShards];
    // ---- published by pack, read by the expand kernel's overflow check ----
    alignas(128) unsigned long long r_pub[kMaxShards];
    // ---- per-step slots: the ring positions by the expand kernel's last
    // block, the rest by the select kernel (one thread, once per step) ----
    alignas(128) unsigned long long w_snap[kXSlots][kMaxShards];
    struct StepInfo {
        unsigned long long n_batch;
        long long goal;
        int fail, has_work, low_b, pad;
    } info[kXSlots];
    // lowest live bucket over all shards as of their last select (written by
    // the insert kernel from the headers; kBuckets: none)
    int gmin_b;
    // ---- side stream only (pack / insert) ----
    unsigned long long r[2][kMaxShards];  // consumed positions, by step parity
    unsigned long long sent, received, sent_steps, backlog_max, backlog_steps;
    unsigned long long demand_max;  // most records one shard had for one destination in a step, since the host's last reset
    unsigned long long claimed_b, dropped_b;  // insert's table claims, folded by pack
    int fail_b, fault_b;
    unsigned long long steps_done;  // steps up to and including the one that ended the search
    int quiet_run;  // consecutive steps in which no shard had work, records or backlog
    int pad0;
};


__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Broadcast from a wave-uniform lane (a ballot's leader): v_readlane into a
// scalar register, where __shfl would take an LDS round trip (ds_bpermute)
__device__ __forceinline__ int bcast_lane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ unsigned long long bcast_lane(unsigned long long v, int lane)
{
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), lane);
    return ((unsigned long long)hi << 32) | lo;
}

// Wave-wide reductions on DPP lane moves (no LDS round trip): an inclusive
// row scan (row_shr 1, 2, 4, 8), then row_bcast 15 and 31; lane 63 holds the
// total.  Every lane of the wave must be active.
template <typename Op>
__device__ __forceinline__ int wave_reduce_dpp(int v, int identity, Op op)
{
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x111, 0xf, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x112, 0xf, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x114, 0xf, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x118, 0xf, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x142, 0xa, 0xf, false));
    v = op(v, __builtin_amdgcn_update_dpp(identity, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_min_i32(int v)
{
    return wave_reduce_dpp(v, kIntMax, [](int x, int y) { return x < y ? x : y; });
}

__device__ __forceinline__ int wave_sum_i32(int v)
{
    return wave_reduce_dpp(v, 0, [](int x, int y) { return x + y; });
}

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int KW>
__device__ __forceinline__ uint64_t key_hash(const uint64_t (&k)[KW])
{
    uint64_t h = mix64(k[0]);
#pragma unroll
    for (int w = 1; w < KW; w++)
        h = mix64(h ^ k[w]);
    return h;
}

template <int KW>
__host__ __device__ constexpr int slot_words()
{
    return KW <= 2 ? 4 : 8;
}

// Slots per 128-B cache line.  With 1-word keys a probe sequence starts at
// the first slot of the line its hash falls in (then linear, across lines),
// so the first probes of a key are one line: a prefetch of that line's key
// words resolves most collisions without another memory round trip.  Longer
// keys start at their hash slot: their prefetch covers one slot, and aligned
// starts would only cluster the first probes (syn8x400 10% slower).
template <int KW>
__host__ __device__ constexpr int line_slots()
{
    return 128 / (slot_words<KW>() * 8);
}

template <int KW>
__device__ __forceinline__ uint64_t probe_start(const uint64_t (&k)[KW], uint64_t cap_mask)
{
    const uint64_t h = key_hash<KW>(k) & cap_mask;
    return KW == 1 ? h & ~(uint64_t)(line_slots<KW>() - 1) : h;
}

// Wave-aggregated append: one atomic per wave, lanes write compacted
// (ballot + prefix popcount).  Must be reached by every lane of the wave.
template <typename T>
__device__ __forceinline__ void wave_append(bool pred, unsigned long long *counter, T *out,
                                            unsigned long long cap, const T &v,
                                            unsigned long long *overflow)
{
    const uint64_t mask = __ballot(pred);
    if (!mask)
        return;
    const int lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    unsigned long long base = 0;
    if (lane == leader)
        base = atomicAdd(counter, (unsigned long long)__popcll(mask));
    base = bcast_lane(base, leader);
    if (pred) {
        const unsigned long long idx = base + __popcll(mask & ((1ull << lane) - 1ull));
        if (idx < cap)
            out[idx] = v;
        else if (overflow)
            atomicAdd(overflow, 1ull);
    }
}

// Relax (key, g, parent mask) into the node table.  Returns the slot (-1
// when the probe limit is hit, -2 when a key's tail words were not published
// within kSpinLimit re-reads) and sets `improved` when g is strictly better
// than every g recorded for the key so far; `claimed` when the slot is new.
//
// Concurrency: slots are never freed, and every key word goes 0 -> final
// exactly once, so a non-zero key word is always current and a plain load
// may only lag (reading 0).  The claim is a CAS on word 0; 2- and 4-word keys
// publish their tail words with agent-scope atomic stores, and a reader that
// matched word 0 re-reads a zero tail word until it is written (the claimant
// writes it in the same loop iteration, so no wave can stall on itself).
// best only decreases, so a lagging read of it can only skip a relaxation
// that would not improve anything.  *lowered (optional; the caller sets it
// false) reports that best itself decreased: a better g, or the same g with
// a smaller parent mask.
//
// pre (has_pre): the key words and best of the first PFS slots of the probe
// sequence, read by the caller ahead of time (slot_prefetch); a read taken
// earlier can only lag more, which the protocol already tolerates (a slot
// seen empty may have been claimed since: the CAS then fails and the slot is
// re-read).
template <int KW, int PFS>
struct SlotWords {
    uint64_t w[PFS][KW + 1];
    uint32_t start;  // the key's probe start (its hash, computed once)
};

template <int KW, int PFS>
__device__ __forceinline__ int64_t relax(uint64_t *__restrict__ table, uint64_t cap_mask,
                                         const uint64_t (&key)[KW], int g, int pmask, int h,
                                         bool &improved, bool &claimed, bool has_pre,
                                         const SlotWords<KW, PFS> &pre, bool *lowered = nullptr)
{
    constexpr int SW = slot_words<KW>();
    improved = false;
    claimed = false;
    uint64_t idx;
    if (has_pre)
        idx = pre.start;
    else
        idx = probe_start<KW>(key, cap_mask);
    int probe = 0;
    // the prefetched slots: skip those holding other keys (key word 0 set
    // and different), and start at the first empty or candidate one with
    // its prefetched words (constant indices only: no register array is
    // indexed at run time)
    bool use_pre = false;
    uint64_t pw[KW + 1];
#pragma unroll
    for (int w = 0; w <= KW; w++)
        pw[w] = 0;
    if (has_pre) {
        int j0 = PFS;
#pragma unroll
        for (int t = 0; t < PFS; t++) {
            const bool hit = j0 == PFS && (pre.w[t][0] == 0 || pre.w[t][0] == key[0]);
            if (hit) {
                j0 = t;
#pragma unroll
                for (int w = 0; w <= KW; w++)
                    pw[w] = pre.w[t][w];
            }
        }
        idx = (idx + j0) & cap_mask;
        probe = j0;
        use_pre = j0 < PFS;
    }
    for (; probe < kMaxProbe;) {
        uint64_t *s = table + idx * SW;
        // one plain (vector) read of the key words and best: it can only lag,
        // showing 0 for a key word being published or a larger best
        uint64_t wv[KW + 1];
        if (KW <= 2 && use_pre) {
#pragma unroll
            for (int w = 0; w <= KW; w++)
                wv[w] = pw[w];
        } else {
            const ulonglong2 v0 = *reinterpret_cast<const ulonglong2 *>(s);
            wv[0] = v0.x;
            if constexpr (KW == 1) {
                wv[1] = v0.y;
            } else {
                const ulonglong2 v1 = *reinterpret_cast<const ulonglong2 *>(s + 2);
                wv[1] = v0.y;
                wv[2] = v1.x;
                if constexpr (KW == 4) {
                    wv[3] = v1.y;
                    wv[4] = s[4];
                }
            }
        }
        use_pre = false;
        bool mine = false;
        if (wv[0] == 0) {
            const uint64_t prev = atomicCAS((unsigned long long *)s, 0ull, (unsigned long long)key[0]);
            if (prev == 0) {
#pragma unroll
                for (int w = 1; w < KW; w++)
                    __hip_atomic_store(s + w, key[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                reinterpret_cast<int32_t *>(s + KW + 1)[1] = h;
                claimed = true;
                mine = true;
                wv[KW] = ~0ull;
            } else {
                wv[0] = prev;
#pragma unroll
                for (int w = 1; w < KW; w++)
                    wv[w] = 0;  // unknown: re-read below
            }
        }
        if (!mine) {
            if (wv[0] != key[0]) {
                idx = (idx + 1) & cap_mask;
                probe++;
                continue;
            }
            bool same = true;
#pragma unroll
            for (int w = 1; w < KW; w++) {
                uint64_t v = wv[w];
                if (v == 0) {
                    // unknown, or still being published by a claimant that
                    // is past its CAS and stores the tail next: read it, a
                    // bounded number of times (the counter lives only here)
                    unsigned poll = 0;
                    do
                        v = __hip_atomic_load(s + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    while (v == 0 && ++poll < kSpinLimit);
                    if (v == 0)
                        return -2;
                }
                same &= (v == key[w]);
            }
            if (!same) {
                idx = (idx + 1) & cap_mask;
                probe++;
                continue;
            }
        }
        const uint64_t packed = ((uint64_t)(uint32_t)g << 32) | (uint32_t)pmask;
        if (mine) {
            // the claimant counts as improving without waiting for the
            // result: if a racing relaxer already stored a smaller g, this
            // entry is simply stale (f != best g + h) when popped
            __hip_atomic_fetch_min((unsigned long long *)(s + KW), (unsigned long long)packed, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            improved = true;
            if (lowered)
                *lowered = true;
        } else if (packed < wv[KW]) {
            const uint64_t old = atomicMin((unsigned long long *)(s + KW), (unsigned long long)packed);
            improved = (int64_t)(old >> 32) > (int64_t)g || old == ~0ull;
            // lowered: also a tie on g with a smaller parent mask (no
            // re-expansion, but the record's mask changed)
            if (lowered)
                *lowered = packed < old;
        }
        return (int64_t)idx;
    }
    return -1;
}

// Key words and best of the first PFS slots of key's probe sequence (one
// cache line), for relax's `pre`: issued before the parent's pair terms are
// staged, so the probe's memory round trip overlaps the pair-table gathers.
template <int KW, int PFS>
__device__ __forceinline__ SlotWords<KW, PFS> slot_prefetch(const uint64_t *__restrict__ table, uint64_t cap_mask,
                                                            const uint64_t (&key)[KW])
{
    static_assert(KW <= 2 && PFS <= line_slots<KW>() && (KW == 1 || PFS == 1),
                  "prefetch: one line of 1-word keys, or one slot of a 2-word key");
    constexpr int SW = slot_words<KW>();
    SlotWords<KW, PFS> o;
    const uint64_t start = probe_start<KW>(key, cap_mask);
    o.start = (uint32_t)start;
    const uint64_t *s0 = table + start * SW;
#pragma unroll
    for (int t = 0; t < PFS; t++) {
        const uint64_t *s = s0 + t * SW;
        const ulonglong2 v0 = *reinterpret_cast<const ulonglong2 *>(s);
        o.w[t][0] = v0.x;
        o.w[t][1] = v0.y;
        if constexpr (KW == 2)
            o.w[t][2] = s[2];
    }
    return o;
}

// Lookup without insertion (closed list / backtrace).
template <int KW>
__device__ __forceinline__ int64_t lookup(const uint64_t *__restrict__ table, uint64_t cap_mask,
                                          const uint64_t (&key)[KW])
{
    constexpr int SW = slot_words<KW>();
    uint64_t idx = probe_start<KW>(key, cap_mask);
    for (int probe = 0; probe < kMaxProbe; probe++) {
        const uint64_t *s = table + idx * SW;
        if (s[0] == 0)
            return -1;
        bool same = true;
#pragma unroll
        for (int w = 0; w < KW; w++)
            same &= (s[w] == key[w]);
        if (same)
            return (int64_t)idx;
        idx = (idx + 1) & cap_mask;
    }
    return -1;
}

// The DevProblem fields the per-level code of the search kernel reads (key
// packing, lengths, goal, gap costs, shard partition), copied into registers
// once at kernel start.  Read through the DevProblem reference inside the
// level loop, each would be a vector load the compiler cannot hoist past the
// loop's table writes (it cannot prove they do not alias), i.e. a chain of
// dependent global round trips on every level.  Same field names as
// DevProblem, so the helpers take either.
template <int N, int KW>
struct KConst {
    static constexpr int NMAX = N ? N : kMaxN;
    int len[NMAX], kword[NMAX], kshift[NMAX], kbits[NMAX];
    uint64_t goal_key[KW];
    int gap_open, gap_ext, gap_gap;
    int hash_type, hash_shift, n_shards, shard;
    const int2 *HC;
};

template <int N, int KW>
__device__ __forceinline__ KConst<N, KW> load_kconst(const DevProblem &P)
{
    KConst<N, KW> k;
#pragma unroll
    for (int i = 0; i < KConst<N, KW>::NMAX; i++) {
        k.len[i] = P.len[i];
        k.kword[i] = KW == 1 ? 0 : P.kword[i];
        k.kshift[i] = P.kshift[i];
        k.kbits[i] = P.kbits[i];
    }
#pragma unroll
    for (int w = 0; w < KW; w++)
        k.goal_key[w] = P.goal_key[w];
    k.gap_open = P.gap_open;
    k.gap_ext = P.gap_ext;
    k.gap_gap = P.gap_gap;
    k.hash_type = P.hash_type;
    k.hash_shift = P.hash_shift;
    k.n_shards = P.n_shards;
    k.shard = P.shard;
    k.HC = P.HC;
    return k;
}

// ---------------------------------------------------------------------------
// CoordHash owner (CoordHash.cpp:107-245) on device, for the shard partition.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int ilog2_floor(int v) { return 31 - __clz(v); }

template <int NMAX, typename PP>
__device__ __forceinline__ int owner_dev(const PP &P, int n, const int (&pos)[NMAX], int size)
{
    if (size <= 1)
        return 0;
    const int shift = P.hash_shift;
    if (P.hash_type == 2 || P.hash_type == 3) {
        unsigned s = 0;
        const int lim = P.hash_type == 2 ? n : 2;
#pragma unroll
        for (int i = 0; i < NMAX; i++)
            if (i < lim)
                s += (unsigned)pos[i];
        return (int)((s >> shift) % (unsigned)size);
    }
    const int dims = P.hash_type == 1 ? 2 : n;
    // (unsigned)(log2(size) + shift % dims + 1): exact for integer log2 of a
    // power of two, floor otherwise (log2 of a non-power is not an integer).
    const unsigned bits = (unsigned)(ilog2_floor(size) + (shift % dims) + 1);
    const unsigned total = bits >= 31 ? 0x80000000u : (1u << bits);
    int hash = 0;
    int bit_to_read = shift / dims;
    for (unsigned bit = 1; bit != 0 && bit <= total;) {
        for (int j = 0; j < dims && bit != 0 && bit <= total; ++j) {
            int c = 0;
#pragma unroll
            for (int i = 0; i < NMAX; i++)
                if (i == j)
                    c = pos[i];
            if (bit_to_read < 16 && (c & (1 << bit_to_read)))
                hash = (int)((unsigned)hash | bit);
            bit <<= 1;
        }
        ++bit_to_read;
    }
    return (int)((unsigned)((hash >> (shift % dims)) % size));
}

// ---------------------------------------------------------------------------
// Parent setup: decode the coordinate and stage the 4 corner terms of every
// pair in LDS.  For a parent p and neighbour mask m, pair (x, y) contributes
//   g: w * {GapGap, gap(x idle), gap(y idle), cost(s_x[p_x], s_y[p_y])}
//   h: w * H_xy[p_x + b_x][p_y + b_y]
// selected by corner c = b_x << 1 | b_y (Node.cpp:130-152, 206-248;
// HeuristicHPair.cpp:74-86).  One expansion reads 4P H cells, not 4P per
// neighbour.
// ---------------------------------------------------------------------------
template <int N, int KW>
struct Parent {
    static constexpr int NMAX = N ? N : kMaxN;
    uint64_t key[KW];
    int pos[NMAX];
    int g, pmask, blocked;
};

template <int N, int KW, typename PP>
__device__ __forceinline__ void decode_key(const PP &P, int n, const uint64_t (&key)[KW],
                                           int (&pos)[Parent<N, KW>::NMAX])
{
#pragma unroll
    for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
        if (N == 0 && i >= n) {
            pos[i] = 0;
            continue;
        }
        const int w = KW == 1 ? 0 : P.kword[i];  // one word: no table read
        uint64_t word = key[0];
#pragma unroll
        for (int k = 1; k < KW; k++)
            if (w == k)
                word = key[k];
        pos[i] = (int)((word >> P.kshift[i]) & ((1ull << P.kbits[i]) - 1ull));
    }
}

// Fills terms[q], q = p*4 + c, for q in [glane, 4P) step lpn: one HC
// gather per term (the c = 3 term also reads the substitution cost of the
// parent's cell).
template <int N, int KW, typename PP>
__device__ __forceinline__ void stage_terms(const PP &P, int n, int npairs, const PairConst *pc,
                                            const Parent<N, KW> &par, int2 *terms, int glane, int lpn)
{
    for (int q = glane; q < 4 * npairs; q += lpn) {
        const int p = q >> 2, c = q & 3;
        const PairConst k = pc[p];
        int px = 0, py = 0;
#pragma unroll
        for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
            if (i == k.x)
                px = par.pos[i];
            if (i == k.y)
                py = par.pos[i];
        }
        const int bx = c >> 1, by = c & 1;
        const int2 *cells = P.HC + k.off;
        int hc = 0;
        if (px + bx <= k.lx && py + by <= k.ly)
            hc = cells[(int64_t)(px + bx) * k.row + (py + by)].x;
        int gc;
        if (c == 3) {
            gc = cells[(int64_t)px * k.row + py].y;
        } else {
            int g0;
            if (c == 2)  // x moves, y idle: open iff y moved into the parent
                g0 = ((par.pmask >> k.y) & 1) ? P.gap_open : P.gap_ext;
            else if (c == 1)
                g0 = ((par.pmask >> k.x) & 1) ? P.gap_open : P.gap_ext;
            else
                g0 = P.gap_gap;
            gc = g0 * k.w;
        }
        terms[q] = make_int2(gc, hc);
    }
}

// stage_terms for a fixed N: the gathers of a lane's terms (a compile-time
// count) are all issued before the first is waited for, one memory round
// trip per parent instead of one per term.
template <int N, int KW, typename PP, typename F>
__device__ __forceinline__ void stage_terms_fixed(const PP &P, const PairConst *pc, const Parent<N, KW> &par,
                                                  int2 *terms, int glane, F &&after_issue)
{
    static_assert(N > 0, "fixed N only");
    constexpr int NP = N * (N - 1) / 2;
    constexpr int LPN = (1 << N) < 64 ? (1 << N) : 64;
    constexpr int NT = (4 * NP + LPN - 1) / LPN;
    // branch-free: every address is clamped into its table (a term past 4P
    // reads pair 0's cell and is dropped), so the compiler issues all 2*NT
    // gathers back to back and waits once
    int hraw[NT], graw[NT], g0w[NT];
    bool hin[NT], mm[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int q0 = glane + t * LPN;
        const int q = q0 < 4 * NP ? q0 : 0;
        const int p = q >> 2, c = q & 3;
        const PairConst k = pc[p];
        int px = 0, py = 0;
#pragma unroll
        for (int i = 0; i < N; i++) {
            if (i == k.x)
                px = par.pos[i];
            if (i == k.y)
                py = par.pos[i];
        }
        const int bx = c >> 1, by = c & 1;
        // global address space: a generic pointer would make these flat
        // loads, which also count on the LDS counter (the pc reads of the
        // next term would then wait for them)
        const __attribute__((address_space(1))) int2 *cells =
            (const __attribute__((address_space(1))) int2 *)(P.HC + k.off);
        hin[t] = px + bx <= k.lx && py + by <= k.ly;
        const int ix = px + bx <= k.lx ? px + bx : k.lx, iy = py + by <= k.ly ? py + by : k.ly;
        hraw[t] = cells[(int64_t)ix * k.row + iy].x;
        graw[t] = cells[(int64_t)px * k.row + py].y;
        mm[t] = c == 3;
        // c = 2: x moves, y idle: gap open iff y moved into the parent
        const int g0 = c == 2 ? (((par.pmask >> k.y) & 1) ? P.gap_open : P.gap_ext)
                              : (c == 1 ? (((par.pmask >> k.x) & 1) ? P.gap_open : P.gap_ext) : P.gap_gap);
        g0w[t] = g0 * k.w;
    }
    after_issue();  // more loads the caller overlaps with the gathers
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int q = glane + t * LPN;
        if (q < 4 * NP)
            terms[q] = make_int2(mm[t] ? graw[t] : g0w[t], hin[t] ? hraw[t] : 0);
    }
}

// Sum of the staged terms for neighbour mask m: (delta g, h).
template <int N>
__device__ __forceinline__ int2 child_cost(const DevProblem &P, int npairs, const int2 *terms, int m)
{
    int dg = 0, hh = 0;
    if constexpr (N > 0) {
        int p = 0;
#pragma unroll
        for (int x = 0; x < N - 1; x++) {
#pragma unroll
            for (int y = x + 1; y < N; y++, p++) {
                const int c = (((m >> x) & 1) << 1) | ((m >> y) & 1);
                const int2 t = terms[p * 4 + c];
                dg += t.x;
                hh += t.y;
            }
        }
    } else {
        for (int p = 0; p < npairs; p++) {
            const int x = P.pair_x[p], y = P.pair_y[p];
            const int c = (((m >> x) & 1) << 1) | ((m >> y) & 1);
            const int2 t = terms[p * 4 + c];
            dg += t.x;
            hh += t.y;
        }
    }
    return make_int2(dg, hh);
}

// ---------------------------------------------------------------------------
// Split tables for wide fan-outs (fixed N >= 7, one parent per wave).  A
// child's cost is a sum over all P pairs of the term its mask selects, 28
// LDS reads a child for N = 8, times 255 children.  With the sequences split
// into a low half (NL = N / 2 of them) and a high half, m = m_hi << NL | m_lo,
//   cost(m) = A[m_lo] + B[m_hi] + sum over y in the high half of D[y][bit y of m][m_lo]
// where A and B hold the pairs inside one half and D[y][b][m_lo] the NL pairs
// of y with the low half: 1 + NH + 1 reads a child, from tables of
// 2^NL + 2^NH + 2 NH 2^NL entries that the wave builds once per parent out of
// the staged terms (160 entries for N = 8, 704 term reads for 7140).  Integer
// sums in another order: the same values.
// ---------------------------------------------------------------------------
template <int N>
struct SplitCost {
    static constexpr int NL = N / 2, NH = N - NL;
    static constexpr int kA = 0, kB = 1 << NL, kD = kB + (1 << NH);
    static constexpr int kEntries = kD + 2 * NH * (1 << NL);
    __host__ __device__ static constexpr int pair_index(int x, int y) { return x * (2 * N - x - 1) / 2 + (y - x - 1); }
};

// Builds the wave's tables `tab` (SplitCost<N>::kEntries int2) from its staged
// terms; every lane of the wave calls it, and waits for LDS before reading.
template <int N>
__device__ __forceinline__ void split_cost_build(const int2 *terms, int2 *tab, int lane)
{
    using S = SplitCost<N>;
    for (int e = lane; e < S::kEntries; e += 64) {
        int dg = 0, hh = 0;
        if (e < S::kD) {
            // pairs inside one half: the low half's by m_lo, the high half's by m_hi
            const bool hi = e >= S::kB;
            const int bits = hi ? e - S::kB : e, off = hi ? S::NL : 0, cnt = hi ? S::NH : S::NL;
#pragma unroll
            for (int xl = 0; xl < S::NH - 1; xl++) {
#pragma unroll
                for (int yl = xl + 1; yl < S::NH; yl++) {
                    if (yl < cnt) {
                        const int x = xl + off, y = yl + off;
                        const int p = x * (2 * N - x - 1) / 2 + (y - x - 1);
                        const int c = (((bits >> xl) & 1) << 1) | ((bits >> yl) & 1);
                        const int2 t = terms[p * 4 + c];
                        dg += t.x;
                        hh += t.y;
                    }
                }
            }
        } else {
            // y of the high half against every x of the low half
            const int k = e - S::kD, mlo = k & ((1 << S::NL) - 1), by = (k >> S::NL) & 1, y = S::NL + (k >> (S::NL + 1));
#pragma unroll
            for (int x = 0; x < S::NL; x++) {
                const int p = x * (2 * N - x - 1) / 2 + (y - x - 1);
                const int c = (((mlo >> x) & 1) << 1) | by;
                const int2 t = terms[p * 4 + c];
                dg += t.x;
                hh += t.y;
            }
        }
        tab[e] = make_int2(dg, hh);
    }
}

// (delta g, h) of the child with mask m from the wave's split tables.
template <int N>
__device__ __forceinline__ int2 split_cost(const int2 *tab, int m)
{
    using S = SplitCost<N>;
    const int mlo = m & ((1 << S::NL) - 1), mhi = m >> S::NL;
    const int2 a = tab[S::kA + mlo], b = tab[S::kB + mhi];
    int dg = a.x + b.x, hh = a.y + b.y;
#pragma unroll
    for (int yl = 0; yl < S::NH; yl++) {
        const int2 d = tab[S::kD + ((yl * 2 + ((mhi >> yl) & 1)) << S::NL) + mlo];
        dg += d.x;
        hh += d.y;
    }
    return make_int2(dg, hh);
}

template <int N, int KW, typename PP>
__device__ __forceinline__ void child_key(const PP &P, int n, const uint64_t (&key)[KW], int m,
                                          uint64_t (&out)[KW])
{
#pragma unroll
    for (int w = 0; w < KW; w++)
        out[w] = key[w];
#pragma unroll
    for (int i = 0; i < Parent<N, KW>::NMAX; i++) {
        if ((N == 0 && i >= n) || !((m >> i) & 1))
            continue;
        const uint64_t inc = 1ull << P.kshift[i];
        const int w = KW == 1 ? 0 : P.kword[i];  // one word: no table read
#pragma unroll
        for (int k = 0; k < KW; k++)
            if (w == k)
                out[k] += inc;
    }
}

}  // namespace dev
}  // namespace pastar
