// pastar_gpu.hip -- host side of the C-ABI (include/pastar_gpu.h): device
// context, Phase 1 (PairAlign wavefront), the batched expansion API and the
// device-resident search loop with the RCCL shard exchange.
//
// Search loop, one step (DESIGN.md "Search step"):
//   partition_kernel   near pile -> batch (f <= t) + next near pile
//   expand_kernel      batch -> neighbours relaxed into the node table;
//                      improved ones appended to near (f < t_near) / far;
//                      remote-owned ones posted to per-shard outboxes
//   [n_shards > 1]     RCCL send/recv of the outboxes, insert_remote_kernel,
//                      allreduce of {goal g, remaining work}
//   status D2H         counters + near histogram -> next t, refill decision
// Termination: no open entry with f < best goal g remains on any shard
// (PAStar::check_stop's goal-f <= every open f, PAStar.cpp:480-547).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "host_model.hpp"
#include "kernels.hpp"
#include "pastar_gpu.h"
#include "lists.hpp"
#include "solo.hpp"
#include "selftest.hpp"

using namespace pastar;
using namespace pastar::dev;

// Device scratch of pastar_gpu_expand_noalloc: one array per GPU the library
// runs on, held until the process ends.  `scratch` is a host-side stand-in for
// the symbol, never a device address: host code uses the address
// hipGetSymbolAddress returns for the current device (pastar_ctx::scratch).
constexpr size_t scr_align(size_t v) { return (v + 255) & ~(size_t)255; }
constexpr size_t kScrIn = 0;
constexpr size_t kScrOff = scr_align(kScrIn + sizeof(pastar_node) * PASTAR_NOALLOC_MAX_IN);
constexpr size_t kScrOut = scr_align(kScrOff + sizeof(int64_t) * PASTAR_NOALLOC_MAX_IN);
constexpr size_t kScrOwner = scr_align(kScrOut + sizeof(pastar_node) * PASTAR_NOALLOC_MAX_OUT);
constexpr size_t kScrSrc = scr_align(kScrOwner + sizeof(int32_t) * PASTAR_NOALLOC_MAX_OUT);
constexpr size_t kScratchBytes = scr_align(kScrSrc + sizeof(int32_t) * PASTAR_NOALLOC_MAX_OUT);
static __device__ __align__(256) unsigned char scratch[kScratchBytes];

namespace {

thread_local std::string g_err;
std::atomic<uint64_t> g_many_stamp{0};

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail(PASTAR_ENODEV, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                        __FILE__, __LINE__);                                                       \
    } while (0)

#define NCCL_TRY(expr)                                                                             \
    do {                                                                                           \
        ncclResult_t _r = (expr);                                                                  \
        if (_r != ncclSuccess)                                                                     \
            return fail(PASTAR_ECOMM, "%s failed: %s", #expr, ncclGetErrorString(_r));            \
    } while (0)

#define PA_TRY(expr)          \
    do {                      \
        int _rc = (expr);     \
        if (_rc != PASTAR_OK) \
            return _rc;       \
    } while (0)

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { reset(); }
    void reset()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    int alloc(size_t count)
    {
        reset();
        if (count == 0)
            return PASTAR_OK;
        hipError_t e = hipMalloc(&p, sizeof(T) * count);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(PASTAR_ENOMEM, "hipMalloc(%zu bytes) failed: %s", sizeof(T) * count, hipGetErrorString(e));
        }
        n = count;
        return PASTAR_OK;
    }
};

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------------------
// Shard transports.  The search talks to the other shards through four
// operations; RCCL implements them for one process per GPU (the reference's
// MPI ranks), LocalGroup for several shards driven by threads of one process
// (peer copies; also how the sharded path is tested on a single GPU).
// ---------------------------------------------------------------------------
enum RedOp { kRedSum, kRedMin, kRedMax };

struct Transport {
    virtual ~Transport() = default;
    // element-wise reduction of host int64 values over all shards
    virtual int allreduce(pastar_ctx *c, int64_t *vals, int count, RedOp op) = 0;
    // device buffer of `root` copied to every shard's same buffer
    virtual int broadcast(pastar_ctx *c, void *dev, size_t bytes, int root) = 0;
    // once per search, after the exchange buffers are allocated (collective)
    virtual int xchg_setup(pastar_ctx *c) = 0;
    // one step's all-to-all of the fixed-size blocks, enqueued on the side
    // stream behind the step's pack kernel: block d of this shard's send
    // area (parity step & 1) becomes block `shard` of shard d's receive area.
    // Nothing here waits for the device.
    virtual int xchg(pastar_ctx *c, int step) = 0;
    // this shard cannot go on: release the shards that wait for it on the
    // host, where the transport can (an in-process group; RCCL peers are
    // left to their own time limits, as MPI ranks are)
    virtual void abort() {}
};
constexpr int kEvRing = 8;  // events per stream hand-over, reused round-robin by step

}  // namespace

struct pastar_group {
    int G = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long long gen = 0;
    bool broken = false;
    std::vector<std::array<int64_t, 16>> vals;
    std::vector<std::vector<unsigned long long>> counts;
    std::vector<std::array<const unsigned char *, 2>> xsend;  // each shard's send areas, by parity
    std::vector<std::array<hipEvent_t, kEvRing>> ev_pack;     // each shard's "blocks packed" events
    std::vector<void *> bufs;
    std::vector<int> device;
    std::atomic<int> members{0};

    // returns false when the group is broken (a member failed) or on timeout
    bool barrier()
    {
        std::unique_lock<std::mutex> l(mu);
        if (broken)
            return false;
        const long long g = gen;
        if (++arrived == G) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(l, std::chrono::seconds(600), [&] { return gen != g || broken; });
        if (!ok || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
    void breakdown()
    {
        std::lock_guard<std::mutex> l(mu);
        broken = true;
        cv.notify_all();
    }
};

namespace {

class LocalTransport : public Transport {
   public:
    LocalTransport(pastar_group *g, int rank) : g_(g), rank_(rank) {}
    ~LocalTransport() override { g_->members--; }

    int sync()
    {
        if (!g_->barrier())
            return fail(PASTAR_ECOMM, "shard group broken (a shard failed or timed out)");
        return PASTAR_OK;
    }
    int allreduce(pastar_ctx *, int64_t *vals, int count, RedOp op) override
    {
        for (int k = 0; k < count; k++)
            g_->vals[rank_][k] = vals[k];
        PA_TRY(sync());
        for (int k = 0; k < count; k++) {
            int64_t r = g_->vals[0][k];
            for (int s = 1; s < g_->G; s++)
                r = op == kRedSum ? r + g_->vals[s][k]
                                  : (op == kRedMin ? std::min(r, g_->vals[s][k]) : std::max(r, g_->vals[s][k]));
            vals[k] = r;
        }
        return sync();
    }
    int broadcast(pastar_ctx *c, void *dev, size_t bytes, int root) override;
    int xchg_setup(pastar_ctx *c) override;
    int xchg(pastar_ctx *c, int step) override;
    void abort() override { g_->breakdown(); }

   private:
    pastar_group *g_;
    int rank_;
};

class RcclTransport : public Transport {
   public:
    // xcomm: the record exchange's own communicator (ncclCommSplit of comm),
    // so that the side stream's send/recv and the main stream's collectives
    // are never ordered against each other on one communicator; nullptr
    // when the split is unavailable (everything then runs on comm)
    RcclTransport(ncclComm_t comm, ncclComm_t xcomm) : comm_(comm), xcomm_(xcomm) {}
    ~RcclTransport() override
    {
        if (xcomm_)
            ncclCommDestroy(xcomm_);
        ncclCommDestroy(comm_);
    }
    int allreduce(pastar_ctx *c, int64_t *vals, int count, RedOp op) override;
    int broadcast(pastar_ctx *c, void *dev, size_t bytes, int root) override;
    int xchg_setup(pastar_ctx *) override { return PASTAR_OK; }
    int xchg(pastar_ctx *c, int step) override;

   private:
    ncclComm_t comm_, xcomm_;
};

}  // namespace

struct pastar_ctx {
    int device = 0, n_shards = 1, shard = 0;
    // set when the search runs the sharded protocol: n_shards > 1, or one
    // shard with an RCCL communicator of its own (the protocol at world 1)
    std::unique_ptr<Transport> tr;
    DevBuf<int64_t> xred;           // RCCL staging of small collectives
    unsigned char *scratch = nullptr;  // this device's copy of the static scratch array (hipGetSymbolAddress)
    unsigned spin_limit = kSpinLimit;  // (the fault word of bounded device waits is Ctl::fault)
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // sharded search: the side stream of the record exchange and the event
    // rings that hand steps over between the two streams
    hipStream_t stream_b = nullptr;
    hipEvent_t ev_a[kEvRing] = {}, ev_b[kEvRing] = {};
    DevBuf<XState> xstate;
    DevBuf<StepStats> stats_b;         // the insert kernel's step statistics
    DevBuf<unsigned char> xsend, xrecv;  // [2][G] and [G] blocks of xblock_bytes
    // xchg_lag = 1: the open-list entries of the records an insert received, by step parity, appended by
    // xdrain_kernel on the main stream; their counts [2], the drain launch's arrival counter
    DevBuf<Entry> xstage;
    DevBuf<unsigned long long> xstage_n;
    DevBuf<unsigned> xdrain_arrive;
    size_t xstage_cap = 0;  // entries per parity
    // the exchange block in use (sized per round from the demand seen, up
    // to the allocated maximum) and the fixed stride between the send areas
    unsigned long long xblock_bytes = 0, xblock_recs = 0, xblock_recs_max = 0, xarea = 0;
    unsigned long long xblock_learned = 0;  // the block size the last completed search ended with

    // problem
    int n = 0, npairs = 0, kw = 1;
    std::vector<std::string> seqs;
    std::vector<int> weights;
    DevProblem hp{};
    DevBuf<DevProblem> dP;
    DevBuf<int32_t> dH;
    DevBuf<int2> dHC;
    DevBuf<uint8_t> dcodes;
    DevBuf<int32_t> dsub;
    bool heuristic_ready = false;  // pastar_gpu_build_heuristic called
    bool hc_built = false;         // HC written in HBM (launched lazily: the LDS-resident search builds its own)
    bool plain_h_ready = false;  // H written (pastar_gpu_pair_table)
    size_t codes_len = 0;
    // LDS-resident search of small problems (solo.hpp)
    bool solo_failed = false;  // a solo search of this problem overflowed its LDS capacity
    bool solo_active = false;  // the last search ran on the solo path (its node table is solo_dump)
    unsigned solo_attr_done = 0;  // per N: dynamic LDS limit raised
    unsigned solo_many_attr_done = 0;
    // pastar_gpu_search_many: this context's launch record as last prepared
    // (valid while its options and buffers stay the same)
    bool many_cached = false;
    long long many_band = 0, many_max_steps = 0;
    SoloArgs many_a{};
    uint64_t many_stamp = 0;
    size_t many_lds = 0;
    volatile uint32_t *many_done = nullptr;
    DevBuf<unsigned char> many_args;  // pastar_gpu_search_many: the launch's argument records
    DevBuf<uint64_t> solo_dump;   // the solo node table in the main slot layout
    int solo_cap_log2 = 0;
    unsigned char *h_solo = nullptr;  // pinned: SoloOut + backtrace masks, written by the kernel
    uint32_t solo_ticket = 0;         // the completion word's value of the last solo launch
    uint32_t tail_ticket = 0;         // the same for the one-shard replay tail (tail_kernel)
    size_t h_solo_n = 0;
    // host-driven OpenList / ClosedList session (lists.hpp)
    bool lists_ready = false;
    SearchArgs lists_args{};
    DevBuf<uint8_t> lists_io;           // nodes in / out, flags, results
    unsigned char *h_lists = nullptr;   // pinned
    size_t h_lists_n = 0;
    long long lists_reopen = 0;

    // search state
    DevBuf<uint64_t> table;
    uint64_t nslots = 0;
    DevBuf<Queues> queues;
    DevBuf<uint32_t> chunk_tab;
    DevBuf<Entry> pool;
    DevBuf<StepStats> stats;
    DevBuf<Ctl> ctl;
    DevBuf<unsigned long long> stamps;
    DevBuf<int> goal;
    DevBuf<uint8_t> outbox;  // rings of records for the other shards
    Ctl *h_ctl = nullptr;                 // pinned
    bool searched = false;
    bool walk_ready = false;  // one shard: the search already walked the goal's chain (h_walk_masks, h_walk info)
    int64_t score = -1;
    // capacities of the current search buffers (reused across searches)
    unsigned long long cap_kmax = 0, cap_pool = 0, cap_maxch = 0, cap_outbox = 0;
    int cap_log2 = 0;
    // capacities learned by automatic growth, kept for later searches
    unsigned long long grown_pool = 0, grown_maxch = 0, grown_outbox = 0;
    int grown_log2 = 0;
    int last_fail_mask = 0;
    unsigned long long last_pool_chunks = 0;  // chunks the last search took
    bool graph_used = false;
    // the captured step graph, reused while the search buffers (and so the
    // kernel arguments) stay the same: capture + instantiate + destroy cost
    // ~0.5 ms per search
    hipGraph_t step_graph[4] = {nullptr, nullptr, nullptr, nullptr};  // runs of kStepRuns[g] launches
    hipGraphExec_t step_exec[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<unsigned char> step_key;
    long long last_steps = 0;  // steps the last completed search took
    // per-problem search constants, computed once per context
    bool origin_ready = false;
    int32_t h0 = 0;
    int auto_band_log2 = 0;
    // open list known to be consistent (cursors and chunk table as a search
    // left them), so the next search resets only what it used
    bool queues_clean_known = false;
    // node-table size learned from the last search's use (0: none yet)
    int learned_log2 = 0;
    // preallocated backtrace buffers (pastar_gpu_alignment)
    DevBuf<uint64_t> walk_key, walk_last;
    DevBuf<uint64_t> walk_goal;  // the goal's key (the one-shard search's walk start)
    DevBuf<int32_t> walk_masks;
    DevBuf<int> walk_info;
    DevBuf<unsigned> tail_arrive;  // tail_kernel's arrival counter (zero between launches)
    uint64_t *h_walk = nullptr;  // pinned: key in, {info, masks} out
    int32_t *h_walk_masks = nullptr;  // pinned: a walked stretch of parent masks
    size_t h_walk_masks_n = 0;
    unsigned char *h_stage = nullptr;  // pinned: per-search uploads (Ctl, origin record)
    DevBuf<unsigned long long> census;  // open-list census of a search
};

namespace {

int slot_words_rt(int kw) { return kw <= 2 ? 4 : 8; }

// ---------------------------------------------------------------------------
// Problem setup (host)
// ---------------------------------------------------------------------------
int setup_problem(pastar_ctx *c, const pastar_problem *p)
{
    if (!p || p->n < 2 || p->n > PASTAR_MAX_SEQ || !p->lengths || !p->residues)
        return fail(PASTAR_EINVAL, "invalid problem (n=%d)", p ? p->n : -1);
    c->n = p->n;
    c->npairs = p->n * (p->n - 1) / 2;
    for (int i = 0; i < p->n; i++) {
        if (p->lengths[i] < 1 || p->lengths[i] > 8000 || !p->residues[i])
            return fail(PASTAR_EINVAL, "sequence %d: length %d outside [1, 8000]", i, p->lengths[i]);
        c->seqs.emplace_back(p->residues[i], (size_t)p->lengths[i]);
    }
    if (p->hash_shift < 0 || p->hash_shift > 21)
        return fail(PASTAR_EINVAL, "Invalid Hash Shift %d", p->hash_shift);
    if (p->hash_type < 0 || p->hash_type > 3)
        return fail(PASTAR_EINVAL, "Invalid hash type %d", p->hash_type);

    // pair weights: given, or Altschul rationale-2 on the host
    if (p->weights) {
        c->weights.assign(p->weights, p->weights + c->npairs);
    } else {
        std::vector<float> wf = altschul_weights(c->seqs);
        for (int x = 0; x < c->n - 1; x++)
            for (int y = x + 1; y < c->n; y++)
                c->weights.push_back((int)wf[(size_t)x * c->n + y]);
    }

    // (the reference's weighting gives negative pair weights to some families
    // of near-identical sequences, WeightedSP.cpp:464-509, and searches with
    // them all the same: h is then no lower bound, and which alignment A*
    // ends with depends on the order of expansion, in the reference too)
    for (int k = 0; k < c->npairs; k++)
        if (c->weights[(size_t)k] < 0) {
            std::fprintf(stderr, "[pastar] warning: pair weight %d is negative (%d): the heuristic is no lower bound, "
                         "the alignment returned need not be optimal\n", k, c->weights[(size_t)k]);
            break;
        }

    DevProblem &hp = c->hp;
    std::memset(&hp, 0, sizeof(hp));
    hp.n = c->n;
    hp.npairs = c->npairs;
    hp.gap_open = p->gap_open;
    hp.gap_ext = p->gap_ext;
    hp.gap_gap = p->gap_gap;
    hp.hash_type = p->hash_type;
    hp.hash_shift = p->hash_shift;
    hp.n_shards = c->n_shards;
    hp.shard = c->shard;

    // residue codes: every byte value present, plus code 0 for the string end
    int code_of[256];
    for (int i = 0; i < 256; i++)
        code_of[i] = -1;
    std::vector<int> chars = {0};
    code_of[0] = 0;
    for (const auto &s : c->seqs)
        for (unsigned char ch : s)
            if (code_of[ch] < 0) {
                code_of[ch] = (int)chars.size();
                chars.push_back(ch);
            }
    hp.alpha = (int)chars.size();
    std::vector<int32_t> sub((size_t)hp.alpha * hp.alpha);
    for (int a = 0; a < hp.alpha; a++)
        for (int b = 0; b < hp.alpha; b++) {
            const int r = chars[a], l = chars[b];
            int v;
            if (p->sub)
                v = (r < 128 && l < 128) ? p->sub[r * 128 + l] : 0;
            else
                v = ref_cost((signed char)r, (signed char)l);
            sub[(size_t)a * hp.alpha + b] = v;
        }
    std::vector<uint8_t> codes;
    int64_t off = 0;
    for (int i = 0; i < c->n; i++) {
        hp.len[i] = (int)c->seqs[i].size();
        hp.seq_off[i] = off;
        for (unsigned char ch : c->seqs[i])
            codes.push_back((uint8_t)code_of[ch]);
        codes.push_back(0);
        off += (int64_t)c->seqs[i].size() + 1;
    }

    // key packing: coordinates never straddle a word; bit 63 marks a word
    int word = 0, used = 0;
    for (int i = 0; i < c->n; i++) {
        int bits = 1;
        while ((1 << bits) <= hp.len[i])
            bits++;
        if (used + bits > 63) {
            word++;
            used = 0;
        }
        hp.kword[i] = word;
        hp.kshift[i] = used;
        hp.kbits[i] = bits;
        used += bits;
    }
    const int words = word + 1;
    c->kw = words <= 1 ? 1 : (words <= 2 ? 2 : (words <= 4 ? 4 : -1));
    if (c->kw < 0)
        return fail(PASTAR_EINVAL, "coordinate key needs %d words (> 4)", words);
    hp.kw = c->kw;
    for (int w = 0; w < 4; w++)
        hp.goal_key[w] = hp.origin_key[w] = (w < c->kw) ? kMark : 0;
    for (int i = 0; i < c->n; i++)
        hp.goal_key[hp.kword[i]] += (uint64_t)hp.len[i] << hp.kshift[i];

    int64_t hoff = 0, k = 0;
    for (int x = 0; x < c->n - 1; x++)
        for (int y = x + 1; y < c->n; y++, k++) {
            hp.pair_x[k] = x;
            hp.pair_y[k] = y;
            hp.weight[k] = c->weights[k];
            hp.h_row[k] = hp.len[y] + 1;
            hp.h_off[k] = hoff;
            hoff += (int64_t)(hp.len[x] + 1) * (hp.len[y] + 1);
        }

    c->codes_len = codes.size();
    PA_TRY(c->dH.alloc((size_t)hoff));
    PA_TRY(c->dHC.alloc((size_t)hoff));
    PA_TRY(c->dcodes.alloc(codes.size()));
    PA_TRY(c->dsub.alloc(sub.size()));
    PA_TRY(c->dP.alloc(1));
    hp.H = c->dH.p;
    hp.HC = c->dHC.p;
    hp.codes = c->dcodes.p;
    hp.sub = c->dsub.p;
    HIP_TRY(hipMemcpy(c->dcodes.p, codes.data(), codes.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->dsub.p, sub.data(), sub.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->dP.p, &hp, sizeof(hp), hipMemcpyHostToDevice));
    return PASTAR_OK;
}

void pack_key(const pastar_ctx *c, const uint16_t *pos, uint64_t *key)
{
    for (int w = 0; w < 4; w++)
        key[w] = (w < c->kw) ? kMark : 0;
    for (int i = 0; i < c->n; i++)
        key[c->hp.kword[i]] += (uint64_t)pos[i] << c->hp.kshift[i];
}

int check_launch()
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(PASTAR_ENODEV, "kernel launch failed: %s", hipGetErrorString(e));
    return PASTAR_OK;
}

const char *fault_site_name(int sites)
{
    if (sites & kSiteQueueStore)
        return "open-list chunk hand-over (queue_store)";
    if (sites & kSiteRelaxTail)
        return "node-table key publication (relax)";
    if (sites & kSitePairAlign)
        return "PairAlign band hand-over";
    if (sites & kSiteSelftest)
        return "self-test handshake";
    return "unknown site";
}

// A bounded device wait that ran out leaves its site in the context's fault
// word: report it as PASTAR_EDEVWAIT and clear the word (the stream is idle).
int report_fault(pastar_ctx *c, int sites)
{
    (void)hipMemset(&c->ctl.p->fault, 0, sizeof(int));
    return fail(PASTAR_EDEVWAIT, "a device wait ran out of its bound at: %s (sites 0x%x); results discarded",
                fault_site_name(sites), sites);
}

// Read the fault word after the stream has drained (calls outside the search,
// whose select reads the word on the device).
int check_fault(pastar_ctx *c)
{
    int sites = 0;
    HIP_TRY(hipMemcpy(&sites, &c->ctl.p->fault, sizeof(int), hipMemcpyDeviceToHost));
    return sites ? report_fault(c, sites) : PASTAR_OK;
}

// Longest the host waits for one replay or one LDS-resident launch to report
// completion (PASTAR_WAIT_TIMEOUT_S, default 600 s), after which the call
// fails instead of polling forever.
double host_wait_limit_s()
{
    static const double lim = [] {
        const char *e = std::getenv("PASTAR_WAIT_TIMEOUT_S");
        const double v = e && *e ? std::atof(e) : 600.0;
        return v > 0 ? v : 600.0;
    }();
    return lim;
}

// ---------------------------------------------------------------------------
// Per-(N, KW) dispatch
// ---------------------------------------------------------------------------
struct Ops {
    void (*expand_api)(dim3, dim3, hipStream_t, const DevProblem *, const pastar_node *, int, const int64_t *, int,
                       pastar_node *, int32_t *, int32_t *);
    void (*expand)(dim3, dim3, hipStream_t, const SearchArgs &);
    void (*expand_one_shard)(dim3, dim3, hipStream_t, const SearchArgs &);
    void (*insert_remote)(dim3, dim3, hipStream_t, const SearchArgs &, const void *, unsigned long long);
    void (*xpack)(dim3, dim3, hipStream_t, const XArgs &);
    void (*xinsert)(dim3, dim3, hipStream_t, const SearchArgs &, const XArgs &);
    void (*walk)(hipStream_t, const DevProblem *, const uint64_t *, uint64_t, const uint64_t *, int, int, int32_t *,
                 uint64_t *, int *, const int *);
    void (*lookup)(hipStream_t, const uint64_t *, uint64_t, const uint64_t *, uint64_t *);
    void (*tail)(hipStream_t, const TailArgs &);
};

template <int N, int KW>
struct Impl {
    static void expand_api(dim3 g, dim3 b, hipStream_t s, const DevProblem *P, const pastar_node *in, int n_in,
                           const int64_t *off, int vec, pastar_node *out, int32_t *own, int32_t *src)
    {
        hipLaunchKernelGGL((expand_api_kernel<N, KW>), g, b, 0, s, P, in, n_in, off, vec, out, own, src);
    }
    static void expand(dim3 g, dim3 b, hipStream_t s, const SearchArgs &a)
    {
        hipLaunchKernelGGL((expand_kernel<N, KW, true>), g, b, 0, s, a);
    }
    static void expand_one_shard(dim3 g, dim3 b, hipStream_t s, const SearchArgs &a)
    {
        hipLaunchKernelGGL((expand_kernel<N, KW, false>), g, b, 0, s, a);
    }
    static void insert_remote(dim3 g, dim3 b, hipStream_t s, const SearchArgs &a, const void *recs,
                              unsigned long long count)
    {
        hipLaunchKernelGGL((insert_remote_kernel<KW>), g, b, 0, s, a, (const Remote<KW> *)recs, count);
    }
    static void xpack(dim3 g, dim3 b, hipStream_t s, const XArgs &t)
    {
        hipLaunchKernelGGL((xpack_kernel<KW>), g, b, 0, s, t);
    }
    static void xinsert(dim3 g, dim3 b, hipStream_t s, const SearchArgs &a, const XArgs &t)
    {
        hipLaunchKernelGGL((xinsert_kernel<KW>), g, b, 0, s, a, t);
    }
    static void walk(hipStream_t s, const DevProblem *P, const uint64_t *t, uint64_t cm, const uint64_t *start, int max,
                     int local, int32_t *masks, uint64_t *last, int *info, const int *gate)
    {
        if constexpr (walk_ahead_ok(N, KW)) {
            if (!local) {
                hipLaunchKernelGGL((walk2_kernel<N, KW>), dim3(1), dim3(64), 0, s, P, t, cm, start, max, masks, last, info,
                                   gate);
                return;
            }
        }
        hipLaunchKernelGGL((walk_kernel<N, KW>), dim3(1), dim3(1), 0, s, P, t, cm, start, max, local, masks, last, info,
                           gate);
    }
    static void tail(hipStream_t s, const TailArgs &t)
    {
        hipLaunchKernelGGL((tail_kernel<N, KW>), dim3(64), dim3(kBlock), 0, s, t);
    }
    static void lookup(hipStream_t s, const uint64_t *t, uint64_t cm, const uint64_t *key, uint64_t *out)
    {
        hipLaunchKernelGGL((lookup_kernel<KW>), dim3(1), dim3(1), 0, s, t, cm, key, out);
    }
    static Ops ops() { return Ops{expand_api, expand, expand_one_shard, insert_remote, xpack, xinsert, walk, lookup, tail}; }
};

template <int KW>
Ops ops_for_kw(int n)
{
    switch (n) {
    case 3: return Impl<3, KW>::ops();
    case 4: return Impl<4, KW>::ops();
    case 5: return Impl<5, KW>::ops();
    case 6: return Impl<6, KW>::ops();
    case 7: return Impl<7, KW>::ops();
    case 8: return Impl<8, KW>::ops();
    default: return Impl<0, KW>::ops();
    }
}

Ops ops_for(const pastar_ctx *c)
{
    if (c->kw == 1)
        return ops_for_kw<1>(c->n);
    if (c->kw == 2)
        return ops_for_kw<2>(c->n);
    return ops_for_kw<4>(c->n);
}

size_t remote_bytes(int kw) { return (size_t)kw * 8 + 16; }

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char *pastar_last_error(void) { return g_err.c_str(); }
int pastar_abi_version(void) { return PASTAR_ABI_VERSION; }

int pastar_cost(int r, int l) { return ref_cost(r, l); }

int pastar_owner(int n, const uint16_t *pos, int size, int hash_type, int shift)
{
    if (!pos || n < 2 || n > PASTAR_MAX_SEQ)
        return -1;
    return owner_of(n, pos, size, hash_type, shift);
}

int pastar_read_fasta(const char *path, char *buf, int64_t cap, int *n, int *lengths)
{
    if (!path || !n)
        return fail(PASTAR_EINVAL, "null argument");
    std::vector<std::string> seqs;
    if (!read_fasta(path, seqs))
        return fail(PASTAR_EIO, "Can't open file %s", path);
    if ((int)seqs.size() > *n)
        return fail(PASTAR_EINVAL, "%zu sequences exceed capacity %d", seqs.size(), *n);
    int64_t off = 0;
    for (size_t i = 0; i < seqs.size(); i++) {
        if (off + (int64_t)seqs[i].size() > cap)
            return fail(PASTAR_EINVAL, "residue buffer too small");
        if (buf)
            std::memcpy(buf + off, seqs[i].data(), seqs[i].size());
        if (lengths)
            lengths[i] = (int)seqs[i].size();
        off += (int64_t)seqs[i].size();
    }
    *n = (int)seqs.size();
    return PASTAR_OK;
}

int pastar_compute_weights(int n, const char *const *residues, const int *lengths, float *out)
{
    if (n < 2 || n > PASTAR_MAX_SEQ || !residues || !lengths || !out)
        return fail(PASTAR_EINVAL, "invalid arguments");
    std::vector<std::string> seqs;
    for (int i = 0; i < n; i++)
        seqs.emplace_back(residues[i], (size_t)lengths[i]);
    std::vector<float> w = altschul_weights(seqs);
    std::memcpy(out, w.data(), sizeof(float) * (size_t)n * n);
    return PASTAR_OK;
}

int pastar_rccl_unique_id(unsigned char out[128])
{
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, sizeof(id));
    return PASTAR_OK;
}

// The side stream of the sharded search and its hand-over events (default
// priority, like the main stream).
static int create_side_stream(pastar_ctx *c)
{
    if (c->stream_b)
        return PASTAR_OK;
    HIP_TRY(hipStreamCreateWithFlags(&c->stream_b, hipStreamNonBlocking));
    for (int k = 0; k < kEvRing; k++) {
        HIP_TRY(hipEventCreateWithFlags(&c->ev_a[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_b[k], hipEventDisableTiming));
    }
    return PASTAR_OK;
}

int pastar_gpu_create(const pastar_problem *p, int device, int n_shards, int shard_rank, const void *rccl_id,
                      pastar_ctx **out)
{
    if (!out)
        return fail(PASTAR_EINVAL, "null out");
    *out = nullptr;
    if (n_shards < 1 || n_shards > 8 || shard_rank < 0 || shard_rank >= n_shards)
        return fail(PASTAR_EINVAL, "invalid shard %d of %d (1..8 shards)", shard_rank, n_shards);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(PASTAR_ENODEV, "no HIP device available (the engine has no CPU fallback)");
    if (device < 0 || device >= ndev)
        return fail(PASTAR_ENODEV, "device %d out of range (%d devices)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(PASTAR_ENODEV, "device %d is %s; this build targets gfx950 only", device, prop.gcnArchName);
    std::unique_ptr<pastar_ctx> c(new pastar_ctx());
    c->device = device;
    c->n_shards = n_shards;
    c->shard = shard_rank;
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&c->ev0));
    HIP_TRY(hipEventCreate(&c->ev1));
    PA_TRY(setup_problem(c.get(), p));
    // the control block (and the search's origin record behind it) exists
    // from the start: it holds the fault word every kernel with a bounded
    // wait reports to
    PA_TRY(c->ctl.alloc(2));
    HIP_TRY(hipMemset(c->ctl.p, 0, 2 * sizeof(Ctl)));
    // each GPU holds its own copy of the scratch array at its own address:
    // resolved here, with this context's device current
    HIP_TRY(hipGetSymbolAddress((void **)&c->scratch, HIP_SYMBOL(scratch)));
    {
        // load the code object now (the runtime loads it at the first use of
        // one of its kernels): a context's first search then pays only its
        // own setup (tools/gpu/cold_probe.py)
        hipFuncAttributes fa;
        HIP_TRY(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&h_kernel)));
    }
    if (n_shards > 1 || rccl_id) {
        if (!rccl_id)
            return fail(PASTAR_EINVAL, "rccl_id required for n_shards > 1");
        ncclUniqueId id;
        std::memcpy(&id, rccl_id, sizeof(id));
        ncclComm_t comm = nullptr, xcomm = nullptr;
        NCCL_TRY(ncclCommInitRank(&comm, n_shards, id, shard_rank));
        // the record exchange's own communicator (same ranks); without it the
        // exchange shares comm, which is still correct: the search's two
        // streams never both hold RCCL work at once
        if (ncclCommSplit(comm, 0, shard_rank, &xcomm, nullptr) != ncclSuccess)
            xcomm = nullptr;
        c->tr.reset(new RcclTransport(comm, xcomm));
        PA_TRY(c->xred.alloc(64));
    }
    if (c->tr)
        PA_TRY(create_side_stream(c.get()));
    HIP_TRY(hipHostMalloc((void **)&c->h_ctl, sizeof(Ctl) + 64, hipHostMallocDefault));  // + pinned scratch
    HIP_TRY(hipHostMalloc((void **)&c->h_stage, sizeof(Ctl) + 256, hipHostMallocDefault));
    *out = c.release();
    return PASTAR_OK;
}

void pastar_gpu_destroy(pastar_ctx *c)
{
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    if (c->stream)
        (void)hipStreamSynchronize(c->stream);
    if (c->stream_b)
        (void)hipStreamSynchronize(c->stream_b);
    c->tr.reset();
    for (int k = 0; k < kEvRing; k++) {
        if (c->ev_a[k])
            (void)hipEventDestroy(c->ev_a[k]);
        if (c->ev_b[k])
            (void)hipEventDestroy(c->ev_b[k]);
    }
    if (c->stream_b)
        (void)hipStreamDestroy(c->stream_b);
    for (int gi = 0; gi < 4; gi++) {
        if (c->step_exec[gi])
            (void)hipGraphExecDestroy(c->step_exec[gi]);
        if (c->step_graph[gi])
            (void)hipGraphDestroy(c->step_graph[gi]);
    }
    if (c->h_ctl)
        (void)hipHostFree(c->h_ctl);
    if (c->h_stage)
        (void)hipHostFree(c->h_stage);
    if (c->h_walk)
        (void)hipHostFree(c->h_walk);
    if (c->h_walk_masks)
        (void)hipHostFree(c->h_walk_masks);
    if (c->h_solo)
        (void)hipHostFree(c->h_solo);
    if (c->h_lists)
        (void)hipHostFree(c->h_lists);
    if (c->ev0)
        (void)hipEventDestroy(c->ev0);
    if (c->ev1)
        (void)hipEventDestroy(c->ev1);
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    delete c;
}

// One launch of the PairAlign wavefront (one workgroup per pair): LDS holds
// the rows below the current bands, the codes of sequence y and, when it
// fits, the distance table.  write_h also stores the plain tables H.
static int launch_pairalign(pastar_ctx *c, bool write_h)
{
    int maxl2 = 0;
    for (int k = 0; k < c->npairs; k++)
        maxl2 = std::max(maxl2, c->hp.len[c->hp.pair_y[k]]);
    const bool sub_lds = c->hp.alpha * c->hp.alpha * 4 <= 32 * 1024;
    if (maxl2 >= 65536 - 64)
        return fail(PASTAR_EINVAL, "sequence too long for the PairAlign kernel (%d)", maxl2);
    const size_t lds = pairalign_lds_bytes(maxl2, c->hp.alpha, sub_lds);
    if (lds > 160 * 1024)
        return fail(PASTAR_EINVAL, "sequence too long for the LDS wavefront (%d)", maxl2);
    // the reference's gap constants are equal (Cost.h:13); the general form
    // stays for patched constants
    const bool eq = c->hp.gap_open == c->hp.gap_ext;
    const void *fn =
        sub_lds ? (write_h ? (eq ? (const void *)pairalign_wave_kernel<true, true, true>
                                 : (const void *)pairalign_wave_kernel<true, true, false>)
                           : (eq ? (const void *)pairalign_wave_kernel<true, false, true>
                                 : (const void *)pairalign_wave_kernel<true, false, false>))
                : (write_h ? (eq ? (const void *)pairalign_wave_kernel<false, true, true>
                                 : (const void *)pairalign_wave_kernel<false, true, false>)
                           : (eq ? (const void *)pairalign_wave_kernel<false, false, true>
                                 : (const void *)pairalign_wave_kernel<false, false, false>));
    if (lds > 64 * 1024)
        HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int *fault = &c->ctl.p->fault;
    void *args[] = {(void *)&c->dP.p, (void *)&c->dH.p, (void *)&c->dHC.p, (void *)&fault, (void *)&c->spin_limit};
    HIP_TRY(hipLaunchKernel(fn, dim3(c->npairs), dim3(64 * kPaWaves), args, lds, c->stream));
    PA_TRY(check_launch());
    // the search and h run on the same stream, so the search-form tables
    // need no host wait (the first search step overlaps this launch's tail);
    // the plain tables are read back by the caller
    if (write_h)
        HIP_TRY(hipStreamSynchronize(c->stream));
    return PASTAR_OK;
}

// The search form of the pair tables in HBM, built on first use.
static int ensure_hc(pastar_ctx *c)
{
    if (c->hc_built)
        return PASTAR_OK;
    PA_TRY(launch_pairalign(c, false));
    c->hc_built = true;
    return PASTAR_OK;
}

int pastar_gpu_build_heuristic(pastar_ctx *c)
{
    if (!c)
        return fail(PASTAR_EINVAL, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    // the search and h read only HC; H is written on demand (pair_table).
    // The wavefront launch itself is deferred to the first call that reads
    // HC from HBM (ensure_hc): the LDS-resident search of a small problem
    // runs PairAlign inside its own launch
    c->heuristic_ready = true;
    c->hc_built = false;
    c->plain_h_ready = false;
    return PASTAR_OK;
}

int pastar_gpu_pair_table(pastar_ctx *c, int pair, int32_t *out)
{
    if (!c || !out || pair < 0 || pair >= c->npairs)
        return fail(PASTAR_EINVAL, "invalid pair %d", pair);
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->plain_h_ready) {
        PA_TRY(launch_pairalign(c, true));
        PA_TRY(check_fault(c));
        c->plain_h_ready = true;
        c->hc_built = true;
    }
    const size_t cells = (size_t)(c->hp.len[c->hp.pair_x[pair]] + 1) * (c->hp.len[c->hp.pair_y[pair]] + 1);
    HIP_TRY(hipMemcpy(out, c->dH.p + c->hp.h_off[pair], cells * 4, hipMemcpyDeviceToHost));
    return PASTAR_OK;
}

int pastar_gpu_weights(pastar_ctx *c, int32_t *out)
{
    if (!c || !out)
        return fail(PASTAR_EINVAL, "null argument");
    std::memcpy(out, c->weights.data(), sizeof(int32_t) * c->weights.size());
    return PASTAR_OK;
}

int pastar_gpu_h(pastar_ctx *c, const uint16_t *pos, int count, int32_t *out)
{
    if (!c || !pos || !out || count < 0)
        return fail(PASTAR_EINVAL, "invalid arguments");
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    if (count == 0)
        return PASTAR_OK;
    for (int k = 0; k < count; k++)
        for (int i = 0; i < c->n; i++)
            if (pos[(size_t)k * PASTAR_MAX_SEQ + i] > c->hp.len[i])
                return fail(PASTAR_EINVAL, "coordinate %d outside the lattice", k);
    HIP_TRY(hipSetDevice(c->device));
    PA_TRY(ensure_hc(c));
    DevBuf<uint16_t> dpos;
    DevBuf<int32_t> dout;
    PA_TRY(dpos.alloc((size_t)count * PASTAR_MAX_SEQ));
    PA_TRY(dout.alloc((size_t)count));
    HIP_TRY(hipMemcpy(dpos.p, pos, (size_t)count * PASTAR_MAX_SEQ * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(h_kernel, dim3((count + 255) / 256), dim3(256), 0, c->stream, c->dP.p, dpos.p, count, dout.p);
    PA_TRY(check_launch());
    HIP_TRY(hipStreamSynchronize(c->stream));
    PA_TRY(check_fault(c));
    HIP_TRY(hipMemcpy(out, dout.p, (size_t)count * 4, hipMemcpyDeviceToHost));
    return PASTAR_OK;
}

// The batched getNeigh over device buffers the caller of this helper owns:
// din [n_in], doff [n_in], dout / down / dsrc [total].  off: host offsets.
static int expand_on(pastar_ctx *c, const pastar_node *in, int n_in, int vec_size, const int64_t *off, int64_t total,
                     pastar_node *din, int64_t *doff, pastar_node *dout, int32_t *down, int32_t *dsrc,
                     pastar_node *out, int32_t *out_owner, int32_t *out_src)
{
    HIP_TRY(hipMemcpy(din, in, sizeof(pastar_node) * (size_t)n_in, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(doff, off, sizeof(int64_t) * (size_t)n_in, hipMemcpyHostToDevice));
    const int lpn = std::min(64, 1 << c->n);
    const int per_block = kWaves * (64 / lpn);
    const int blocks = std::min(4096, (n_in + per_block - 1) / per_block);
    ops_for(c).expand_api(dim3(blocks), dim3(kBlock), c->stream, c->dP.p, din, n_in, doff, vec_size, dout, down, dsrc);
    PA_TRY(check_launch());
    HIP_TRY(hipStreamSynchronize(c->stream));
    PA_TRY(check_fault(c));
    if (total) {
        if (out)
            HIP_TRY(hipMemcpy(out, dout, sizeof(pastar_node) * (size_t)total, hipMemcpyDeviceToHost));
        if (out_owner)
            HIP_TRY(hipMemcpy(out_owner, down, 4 * (size_t)total, hipMemcpyDeviceToHost));
        if (out_src)
            HIP_TRY(hipMemcpy(out_src, dsrc, 4 * (size_t)total, hipMemcpyDeviceToHost));
    }
    return PASTAR_OK;
}

// per-node output offsets: 2^(free dimensions) - 1 neighbours each
static int expand_offsets(const pastar_ctx *c, const pastar_node *in, int n_in, int64_t *off, int64_t *total_out)
{
    int64_t total = 0;
    for (int k = 0; k < n_in; k++) {
        int free_dims = 0;
        for (int i = 0; i < c->n; i++) {
            if (in[k].pos[i] > c->hp.len[i])
                return fail(PASTAR_EINVAL, "node %d outside the lattice", k);
            free_dims += in[k].pos[i] < c->hp.len[i];
        }
        off[k] = total;
        total += (1ll << free_dims) - 1;
    }
    *total_out = total;
    return PASTAR_OK;
}

int pastar_gpu_expand(pastar_ctx *c, const pastar_node *in, int n_in, int vec_size, pastar_node *out,
                      int32_t *out_owner, int32_t *out_src, int64_t *n_out)
{
    if (!c || (!in && n_in) || n_in < 0 || !n_out || vec_size < 1)
        return fail(PASTAR_EINVAL, "invalid arguments");
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    *n_out = 0;
    if (n_in == 0)
        return PASTAR_OK;
    std::vector<int64_t> off((size_t)n_in);
    int64_t total = 0;
    PA_TRY(expand_offsets(c, in, n_in, off.data(), &total));
    HIP_TRY(hipSetDevice(c->device));
    PA_TRY(ensure_hc(c));
    DevBuf<pastar_node> din, dout;
    DevBuf<int64_t> doff;
    DevBuf<int32_t> down, dsrc;
    PA_TRY(din.alloc((size_t)n_in));
    PA_TRY(doff.alloc((size_t)n_in));
    PA_TRY(dout.alloc((size_t)std::max<int64_t>(total, 1)));
    PA_TRY(down.alloc((size_t)std::max<int64_t>(total, 1)));
    PA_TRY(dsrc.alloc((size_t)std::max<int64_t>(total, 1)));
    PA_TRY(expand_on(c, in, n_in, vec_size, off.data(), total, din.p, doff.p, dout.p, down.p, dsrc.p, out, out_owner,
                     out_src));
    *n_out = total;
    return PASTAR_OK;
}

int pastar_gpu_expand_noalloc(pastar_ctx *c, const pastar_node *in, int n_in, int vec_size, pastar_node *out,
                              int32_t *out_owner, int32_t *out_src, int64_t *n_out)
{
    if (!c || (!in && n_in) || n_in < 0 || !n_out || vec_size < 1)
        return fail(PASTAR_EINVAL, "invalid arguments");
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    *n_out = 0;
    if (n_in == 0)
        return PASTAR_OK;
    if (n_in > PASTAR_NOALLOC_MAX_IN)
        return fail(PASTAR_EINVAL, "pastar_gpu_expand_noalloc: %d input nodes exceed the scratch's %d", n_in,
                    PASTAR_NOALLOC_MAX_IN);
    if (!c->scratch)
        return fail(PASTAR_ESTATE, "device scratch address not resolved");
    int64_t off[PASTAR_NOALLOC_MAX_IN];  // (stack: no host allocation either)
    int64_t total = 0;
    PA_TRY(expand_offsets(c, in, n_in, off, &total));
    if (total > PASTAR_NOALLOC_MAX_OUT)
        return fail(PASTAR_EINVAL, "pastar_gpu_expand_noalloc: %lld neighbours exceed the scratch's %d",
                    (long long)total, PASTAR_NOALLOC_MAX_OUT);
    HIP_TRY(hipSetDevice(c->device));
    PA_TRY(ensure_hc(c));
    // the device's scratch array, carved at fixed offsets; the kernel writes
    // every output it is asked for, so nothing has to start at zero
    unsigned char *s = c->scratch;
    pastar_node *din = reinterpret_cast<pastar_node *>(s + kScrIn);
    int64_t *doff = reinterpret_cast<int64_t *>(s + kScrOff);
    pastar_node *dout = reinterpret_cast<pastar_node *>(s + kScrOut);
    int32_t *down = reinterpret_cast<int32_t *>(s + kScrOwner);
    int32_t *dsrc = reinterpret_cast<int32_t *>(s + kScrSrc);
    PA_TRY(expand_on(c, in, n_in, vec_size, off, total, din, doff, dout, down, dsrc, out, out_owner, out_src));
    *n_out = total;
    return PASTAR_OK;
}

}  // extern "C"

// ===========================================================================
// Search
// ===========================================================================
namespace {

struct SearchCfg {
    unsigned long long kmax, kmin, pool_entries, subqueue_entries, outbox_cap;
    unsigned long long xblock_recs;  // records per destination one step's exchange carries
    int xlag;                        // steps the select may run ahead of the insert of received records (0, 1)
    int table_log2;
    int verbose, profile, eager, depth;
    int partial_k;  // partial expansion window in buckets (negative: off)
    int64_t max_steps;
    int64_t band;
};

unsigned long long maxch_of(const SearchCfg &cfg) { return (cfg.subqueue_entries + kChunk - 1) / kChunk; }
unsigned long long pool_chunks_of(const SearchCfg &cfg) { return (cfg.pool_entries + kChunk - 1) / kChunk; }

// The device address of pinned host memory (hipHostMalloc, the base of the
// allocation), for kernels that write their results straight to the host.
template <typename T, typename U>
int host_alias(T *h, U **d)
{
    void *p = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&p, (void *)h, 0));
    *d = reinterpret_cast<U *>(p);
    return PASTAR_OK;
}

int alloc_search(pastar_ctx *c, const SearchCfg &cfg)
{
    const int sw = slot_words_rt(c->kw);
    const unsigned long long maxch = maxch_of(cfg), chunks = pool_chunks_of(cfg);
    // buffers are kept across searches and only ever grow: a search sized
    // smaller than the last one (learned_log2) uses the front of the same
    // table and pool, so its device addresses, and the step graphs captured
    // for them, stay valid
    const size_t table_words = ((size_t)1 << cfg.table_log2) * sw;
    if (c->table.n < table_words) {
        c->table.reset();  // free before allocating the larger one
        PA_TRY(c->table.alloc(table_words));
    }
    c->nslots = 1ull << cfg.table_log2;
    if (c->pool.n < (size_t)chunks * kChunk) {
        c->pool.reset();
        PA_TRY(c->pool.alloc((size_t)chunks * kChunk));
    }
    if (!c->chunk_tab.p || c->cap_maxch != maxch) {  // the chunk table's row stride is maxch
        c->chunk_tab.reset();
        PA_TRY(c->chunk_tab.alloc((size_t)kBuckets * kSub * maxch));
        c->queues_clean_known = false;
    }
    if (!c->queues.p) {
        PA_TRY(c->queues.alloc(1));
        PA_TRY(c->stats.alloc(1));
        PA_TRY(c->stamps.alloc(kArrive));
        PA_TRY(c->goal.alloc(1));
        c->queues_clean_known = false;
    }
    if (c->tr) {
        const size_t rb = remote_bytes(c->kw);
        const size_t bytes = (size_t)c->n_shards * cfg.outbox_cap * rb;
        if (c->outbox.n < bytes) {
            c->outbox.reset();
            PA_TRY(c->outbox.alloc(bytes));
        }
        c->xblock_recs_max = cfg.xblock_recs;
        const size_t area = (size_t)c->n_shards * ((sizeof(XHdr) + cfg.xblock_recs * rb + 255) & ~(size_t)255);
        c->xarea = area;
        if (c->xsend.n < 2 * area) {
            c->xsend.reset();
            c->xrecv.reset();
            PA_TRY(c->xsend.alloc(2 * area));
            PA_TRY(c->xrecv.alloc(area));
        }
        if (!c->xstate.p) {
            PA_TRY(c->xstate.alloc(1));
            PA_TRY(c->stats_b.alloc(1));
        }
    }
    c->cap_log2 = cfg.table_log2;
    c->cap_kmax = cfg.kmax;
    c->cap_pool = chunks;
    c->cap_maxch = maxch;
    c->cap_outbox = cfg.outbox_cap;
    if (!c->census.p)
        PA_TRY(c->census.alloc(5));  // entries left; debug: live, live below the goal, min f, min bucket
    return PASTAR_OK;
}

// A search's device setup, stream-ordered: the table, the used chunk-table
// entries and cursors, the statistics, stamps, goal and census, and the
// control block (+ origin record) from the pinned staging area c->h_stage,
// `stage_bytes` of it (the host fills it before this call): one launch.
int init_search(pastar_ctx *c, const SearchCfg &cfg, size_t stage_bytes, bool seed_taken = false)
{
    const int sw = slot_words_rt(c->kw);
    const unsigned long long maxch = maxch_of(cfg);
    bool reset_queues = true;
    if (!c->queues_clean_known) {
        // fresh buffers: clear everything once
        HIP_TRY(hipMemsetAsync(c->queues.p, 0, sizeof(Queues), c->stream));
        HIP_TRY(hipMemsetAsync(c->chunk_tab.p, 0, sizeof(uint32_t) * c->chunk_tab.n, c->stream));
        c->queues_clean_known = true;
        reset_queues = false;
    }
    uint32_t *stage = nullptr;
    PA_TRY(host_alias(c->h_stage, &stage));
    uint32_t *ctl_dst = reinterpret_cast<uint32_t *>(c->ctl.p);
    const int words = (int)(stage_bytes / 4);
    const int blocks = (int)std::max<uint64_t>(
        (kBuckets * kSub + kBlock - 1) / kBlock, std::min<uint64_t>(8192, (c->nslots + kBlock - 1) / kBlock));
    if (sw == 4)
        hipLaunchKernelGGL((search_init_kernel<4>), dim3(blocks), dim3(kBlock), 0, c->stream, c->table.p, c->nslots,
                           c->kw, c->queues.p, c->chunk_tab.p, maxch, reset_queues ? 1 : 0, c->stats.p, c->stamps.p,
                           c->goal.p, c->census.p, stage, ctl_dst, words, seed_taken ? 1 : 0);
    else
        hipLaunchKernelGGL((search_init_kernel<8>), dim3(blocks), dim3(kBlock), 0, c->stream, c->table.p, c->nslots,
                           c->kw, c->queues.p, c->chunk_tab.p, maxch, reset_queues ? 1 : 0, c->stats.p, c->stamps.p,
                           c->goal.p, c->census.p, stage, ctl_dst, words, seed_taken ? 1 : 0);
    PA_TRY(check_launch());
    return PASTAR_OK;
}

int allreduce_i64(pastar_ctx *c, int64_t *vals, int count, RedOp op)
{
    return c->tr->allreduce(c, vals, count, op);
}

// Bucket width (the band of f one step expands).  Default: about a third of
// the mean f increase of one expansion of the origin, rounded to a power of
// two, so that a node is rarely expanded before a cheaper path to it has been
// settled (work inflation stays near the serial count) while a step still
// holds a whole f-layer of the frontier (tools/tune.py sweeps it).
int estimate_band_log2(pastar_ctx *c, int h0, int64_t band_opt, int *w_out)
{
    int64_t band = band_opt;
    if (band <= 0) {
        pastar_node origin{};
        origin.g = 0;
        origin.f = h0;
        origin.parent_mask = (1 << c->n) - 1;
        const int masks = (1 << c->n) - 1;
        std::vector<pastar_node> kids((size_t)masks);
        int64_t cnt = 0;
        PA_TRY(pastar_gpu_expand(c, &origin, 1, 1, kids.data(), nullptr, nullptr, &cnt));
        int64_t sum = 0;
        for (int64_t k = 0; k < cnt; k++)
            sum += (int64_t)kids[(size_t)k].f - h0;
        // an eighth of the mean f increase of the origin's children up to
        // N = 6, a quarter beyond: the best or tied-best width on every
        // workload (profiles/r1_tune_*.txt: kinase 30 -> 21 ms, syn4x200
        // 1.9 -> 1.5 ms with fewer expansions, PF08184 61 expansions for 60
        // serial; syn8x400 tied at 1/8 and 1/4, syn8x100 24.5 ms at 1/4
        // against 29 at 1/8)
        int div = c->n >= 7 ? 4 : 8;
        if (const char *e = std::getenv("PASTAR_BAND_DIV"))  // tuning override
            div = std::max(1, std::atoi(e));
        band = cnt ? std::max<int64_t>(1, sum / cnt / div) : 1;
    }
    int w = 0;
    while ((2ll << w) <= band * 4 / 3 && w < 24)  // nearest power of two
        w++;
    *w_out = w;
    return PASTAR_OK;
}

// Backtrace walk buffers (device and pinned host), allocated once per
// context and grown with the path length.
int ensure_walk_buffers(pastar_ctx *c, int total_len)
{
    if (!c->walk_key.p)
        PA_TRY(c->walk_key.alloc(4));
    if (!c->walk_last.p)
        PA_TRY(c->walk_last.alloc(4));
    if (!c->walk_info.p)
        PA_TRY(c->walk_info.alloc(2));
    if (c->walk_masks.n < (size_t)total_len + 1)
        PA_TRY(c->walk_masks.alloc((size_t)total_len + 1));
    if (!c->h_walk)
        HIP_TRY(hipHostMalloc((void **)&c->h_walk, 64, hipHostMallocDefault));
    if (c->h_walk_masks_n < (size_t)total_len + 1) {
        if (c->h_walk_masks)
            (void)hipHostFree(c->h_walk_masks);
        c->h_walk_masks = nullptr;
        c->h_walk_masks_n = 0;
        HIP_TRY(hipHostMalloc((void **)&c->h_walk_masks, 4 * ((size_t)total_len + 1), hipHostMallocDefault));
        c->h_walk_masks_n = (size_t)total_len + 1;
    }
    return PASTAR_OK;
}

// Enqueue one walk stretch from coordinate pos (stream-ordered; the caller
// synchronizes): key upload, walk kernel, info and masks back to pinned host
// memory (h_walk[4..5] and h_walk_masks).
int enqueue_walk(pastar_ctx *c, const uint16_t *pos, int total_len, bool local_only)
{
    const Ops ops = ops_for(c);
    pack_key(c, pos, c->h_walk);
    HIP_TRY(hipMemcpyAsync(c->walk_key.p, c->h_walk, 32, hipMemcpyHostToDevice, c->stream));
    if (c->solo_active)  // a solo search walks its own chain (solo.hpp)
        return fail(PASTAR_ESTATE, "no node table walk after an LDS-resident search");
    ops.walk(c->stream, c->dP.p, c->table.p, c->nslots - 1, c->walk_key.p, total_len + 1, local_only ? 1 : 0,
             c->walk_masks.p, c->walk_last.p, c->walk_info.p, nullptr);
    PA_TRY(check_launch());
    return PASTAR_OK;
}

// h of the origin and the automatic bucket width, once per context.
int ensure_origin(pastar_ctx *c)
{
    if (c->origin_ready)
        return PASTAR_OK;
    uint16_t zero[PASTAR_MAX_SEQ] = {0};
    DevBuf<uint16_t> dpos;
    DevBuf<int32_t> dh;
    PA_TRY(dpos.alloc(PASTAR_MAX_SEQ));
    PA_TRY(dh.alloc(1));
    HIP_TRY(hipMemcpy(dpos.p, zero, sizeof(zero), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(h_kernel, dim3(1), dim3(64), 0, c->stream, c->dP.p, dpos.p, 1, dh.p);
    PA_TRY(check_launch());
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(&c->h0, dh.p, 4, hipMemcpyDeviceToHost));
    PA_TRY(estimate_band_log2(c, c->h0, 0, &c->auto_band_log2));
    c->origin_ready = true;
    return PASTAR_OK;
}

template <int KWv>
int search_impl(pastar_ctx *c, const SearchCfg &cfg, pastar_result *res)
{
    constexpr int KW = KWv;
    const Ops ops = ops_for(c);
    const int G = c->n_shards;
    PA_TRY(ensure_hc(c));
    c->solo_active = false;
    PA_TRY(alloc_search(c, cfg));
    const int lpn = std::min(64, 1 << c->n);
    const int per_block = kWaves * (64 / lpn);
    const size_t rb = remote_bytes(KW);

    // h of the origin and the bucket width (once per context)
    uint16_t zero[PASTAR_MAX_SEQ] = {0};
    PA_TRY(ensure_origin(c));
    const int32_t h0 = c->h0;
    int w = c->auto_band_log2;
    if (cfg.band > 0)
        PA_TRY(estimate_band_log2(c, h0, cfg.band, &w));

    Ctl hc{};
    hc.band_log2 = w;
    hc.f0 = h0;
    hc.n_shards = G;
    hc.kmax = cfg.kmax;
    hc.kmin = cfg.kmin;
    hc.pool_chunks = c->pool.n / kChunk;  // the allocation (>= the request): stable across searches
    hc.maxch = maxch_of(cfg);
    hc.table_slots = c->nslots;
    hc.max_steps = cfg.max_steps;
    hc.k_start = ~0ull;
    hc.timing = 0;
    if (cfg.profile) {  // bits: 1 expand launch timing (default), 2 select phases, 4 expand phases (diagnostics, PASTAR_TIMING_MASK=7)
        const char *e = std::getenv("PASTAR_TIMING_MASK");
        hc.timing = e && *e ? std::atoi(e) : 1;
    }
    const bool sharded = c->tr != nullptr;  // the step protocol with an exchange
    hc.fuse = sharded ? 0 : 1;  // one shard: select runs in the tail of expand
    hc.depth = cfg.depth;
    {
        const char *e = std::getenv("PASTAR_DEBUG");
        hc.debug = e && *e ? std::atoi(e) : 0;
    }
    {
        // block-local continuation pays where an expansion is cheap (few
        // children, a narrow frontier: PF08184 2x, syn4x200 1.4x; kinase 8%
        // at 1 round with the 1/8 band) and costs where the fan-out is wide
        // (syn8x400 1.25x slower at any setting): the minimum rounds a level
        // must be allowed before a launch continues, by N
        // (profiles/r1_depth_sweep.txt, profiles/r1_rounds_sweep.txt)
        const char *e = std::getenv("PASTAR_DEEP_ROUNDS");  // tuning override
        hc.deep_rounds = e && *e ? std::max(1, std::atoi(e)) : (c->n <= 6 ? 1 : (1 << 30));
    }
    hc.batch_nb = 1;
    hc.prune_f = kIntMax;
    if (const char *e = std::getenv("PASTAR_PRUNE_F"))  // diagnostics: a known upper bound of the optimum
        hc.prune_f = std::atoi(e) + 1;                  // (what a bound of that quality would be worth)
    // partial expansion (N >= 7; tools/gpu/partial_probe.py): a window of one
    // bucket past the batch, the parent queued in the bucket of its first
    // waiting child, every child it has left generated when it comes up again
    hc.partial_k = cfg.partial_k;
    if (const char *e = std::getenv("PASTAR_PARTIAL_K"))  // tuning overrides
        hc.partial_k = std::atoi(e);
    if (const char *e = std::getenv("PASTAR_PARTIAL_AHEAD"))
        hc.partial_ahead = std::max(0, std::atoi(e));
    hc.partial_two = 1;
    if (const char *e = std::getenv("PASTAR_PARTIAL_TWO"))
        hc.partial_two = std::atoi(e);
    hc.spin_limit = c->spin_limit;
    hc.low_b = kBuckets;
    // (kinase at 8 shards: 147 steps at 4 buckets, 124 at 8; syn8x400: 10.9 M
    // expansions at 4, 19 M at 8; tools/gpu/probe_shards.py)
    hc.xwindow = c->n <= 6 ? 2 * kWide : kWide;
    if (const char *e = std::getenv("PASTAR_XCHG_WINDOW"))  // tuning override
        hc.xwindow = std::max(1, std::atoi(e));
    const bool seed_batch = c->tr == nullptr;
    if (seed_batch) {
        // one shard: the first batch is the origin alone, staged as select
        // would cut it (bucket 0 = bucket(h0), sub-queue 0 of the one-block
        // insert, position 0; the next kWide buckets included), so the first
        // launch expands instead of only selecting
        hc.n_batch = 1;
        hc.batch_b = 0;
        hc.batch_nb = kWide;
        hc.cur_b = 0;
        hc.has_work = 1;
        hc.steps = 1;
        hc.b_prefix[0] = 0;
        for (int r = 1; r <= kRanges; r++)
            hc.b_prefix[r] = 1;
    }
    {
        const char *e = std::getenv("PASTAR_DEEP_BLOCKS");  // tuning override
        hc.deep_blocks = e && *e ? std::max(1, std::atoi(e)) : kDeepBlocks;
    }
    // staged with the origin record below; the setup launch copies both to
    // the device, stream-ordered (no host round trip before the first step)
    std::memcpy(c->h_stage, &hc, sizeof(Ctl));

    SearchArgs a{};
    a.P = c->dP.p;
    a.ctl = c->ctl.p;
    a.stamps = c->stamps.p;
    DevBuf<int> trace;
    a.trace = nullptr;
    if (hc.debug) {
        PA_TRY(trace.alloc((size_t)kTraceSteps * 8));
        std::vector<int> init((size_t)kTraceSteps * 8, 0);
        for (int k = 0; k < kTraceSteps; k++)
            init[(size_t)k * 8 + 6] = kBuckets;
        HIP_TRY(hipMemcpy(trace.p, init.data(), init.size() * 4, hipMemcpyHostToDevice));
        a.trace = trace.p;
    }
    a.table = c->table.p;
    a.cap_mask = c->nslots - 1;
    a.q = c->queues.p;
    a.chunk_tab = c->chunk_tab.p;
    a.pool = c->pool.p;
    a.stats = c->stats.p;
    a.goal_g = c->goal.p;
    a.outbox = c->outbox.p;
    a.outbox_cap = cfg.outbox_cap;
    a.lower = &c->ctl.p->cur_b;
    a.x = c->tr ? c->xstate.p : nullptr;
    a.step = 0;
    a.maxch = maxch_of(cfg);
    a.pool_chunks = c->pool.n / kChunk;

    const dim3 blk(kBlock);
    // about one resident wave of blocks: a block then walks several chunks
    // of a large batch (pipelined) and pays its setup and final flush once
    int n_cu = 256;
    HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device));
    unsigned long long max_blocks =
        std::min<unsigned long long>(kMaxExpandBlocks, (unsigned long long)n_cu * expand_waves_per_eu(c->n, KW));
    if (const char *e = std::getenv("PASTAR_EXPAND_BLOCKS"))  // tuning probe
        max_blocks = std::max(1ull, std::strtoull(e, nullptr, 10));
    const dim3 expand_grid((unsigned)std::min<unsigned long long>(max_blocks, (cfg.kmax + per_block - 1) / per_block));

    // seed: the origin (Sequences::get_initial_node, Sequences.cpp:70-77) on
    // its owner shard, through the same relax path as remote records
    const int origin_owner = G > 1 ? owner_of(c->n, zero, G, c->hp.hash_type, c->hp.hash_shift) : 0;
    uint8_t *drec = reinterpret_cast<uint8_t *>(c->ctl.p + 1);
    {
        std::vector<uint8_t> rec(rb, 0);
        uint64_t key[4];
        pack_key(c, zero, key);
        std::memcpy(rec.data(), key, 8 * KW);
        int32_t tail[4] = {0, h0, (1 << c->n) - 1, 0};
        std::memcpy(rec.data() + 8 * KW, tail, 16);
        std::memcpy(c->h_stage + sizeof(Ctl), rec.data(), rb);
        PA_TRY(init_search(c, cfg, sizeof(Ctl) + rb, seed_batch));
    }
    if (c->shard == origin_owner) {
        ops.insert_remote(dim3(1), blk, c->stream, a, drec, 1);
        PA_TRY(check_launch());
    }
    if (sharded) {
        HIP_TRY(hipMemsetAsync(c->xstate.p, 0, sizeof(XState), c->stream));
        HIP_TRY(hipMemsetAsync(c->stats_b.p, 0, sizeof(StepStats), c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        PA_TRY(c->tr->xchg_setup(c));
    }

    double expand_ms = 0;
    int64_t launches = 0, exchanged = 0, xchg_backlog_steps = 0, xchg_backlog_max = 0, host_waits = 0;
    Ctl h{};
    c->graph_used = false;
    const double t0 = now_s();
    if (!sharded) {
        // one launch per step: expand the batch, and the last block to
        // finish cuts the next one (the first launch, with an empty batch,
        // only selects).  Runs of S steps are captured once and replayed
        // until select reports termination; with profiling the expand kernel
        // times itself on the device clock (event nodes inside a graph cost
        // several microseconds per step)
        // runs of steps captured as graphs of 4, 8, 16 and 32 launches: a
        // replay takes the shortest run that covers the steps the previous
        // search on this context predicts are left (32 with no prediction), so
        // a repeated search usually ends in one replay and few launches run
        // after termination (each would only read `status` and leave)
        constexpr int kRuns = 4;
        constexpr int kStepRuns[kRuns] = {4, 8, 16, 32};
        auto enqueue_steps = [&](int S) -> hipError_t {
            for (int k = 0; k < S; k++)
                ops.expand_one_shard(expand_grid, blk, c->stream, a);
            return hipGetLastError();
        };
        long long steps_before = 0;
        int rc = PASTAR_OK;
        // the end-of-search work rides behind every replay, gated on the
        // device-side status (queue_census_kernel, walk_kernel): the replay
        // that finishes the search is followed by the census of the open
        // list and the backtrace walk from the goal in the same stream, and
        // the one host round trip returns all of it
        int total_len = 0;
        uint16_t goal_pos[PASTAR_MAX_SEQ] = {0};
        for (int i = 0; i < c->n; i++) {
            total_len += c->hp.len[i];
            goal_pos[i] = (uint16_t)c->hp.len[i];
        }
        PA_TRY(ensure_walk_buffers(c, total_len));
        if (!c->walk_goal.p) {  // the goal key, once per context (census zeroed by search_init_kernel)
            PA_TRY(c->walk_goal.alloc(4));
            pack_key(c, goal_pos, c->h_walk);
            HIP_TRY(hipMemcpyAsync(c->walk_goal.p, c->h_walk, 32, hipMemcpyHostToDevice, c->stream));
        }
        // pinned host memory the tail writes into, by its device addresses
        unsigned long long *d_cz_tail = nullptr;
        int32_t *d_goal_tail = nullptr, *d_info = nullptr, *d_masks = nullptr;
        Ctl *d_ctl = nullptr;
        PA_TRY(host_alias(c->h_stage, &d_cz_tail));
        d_goal_tail = reinterpret_cast<int32_t *>(reinterpret_cast<unsigned char *>(d_cz_tail) + 128);
        PA_TRY(host_alias(c->h_ctl, &d_ctl));
        PA_TRY(host_alias(c->h_walk, &d_info));
        d_info += 8;  // h_walk[4..5]
        PA_TRY(host_alias(c->h_walk_masks, &d_masks));
        if (!c->tail_arrive.p) {
            PA_TRY(c->tail_arrive.alloc(2));  // arrival counter, ticket counter
            HIP_TRY(hipMemsetAsync(c->tail_arrive.p, 0, 2 * sizeof(unsigned), c->stream));
            c->tail_ticket = 0;
        }
        TailArgs ta{};
        ta.P = c->dP.p;
        ta.table = c->table.p;
        ta.cap_mask = c->nslots - 1;
        ta.goal_key = c->walk_goal.p;
        ta.max = total_len + 1;
        ta.masks = c->walk_masks.p;
        ta.last_key = c->walk_last.p;
        ta.info = c->walk_info.p;
        ta.q = c->queues.p;
        ta.census = c->census.p;
        ta.ctl = c->ctl.p;
        ta.goal = c->goal.p;
        ta.arrive = c->tail_arrive.p;
        ta.h_ctl = d_ctl;
        ta.h_goal = d_goal_tail;
        ta.h_census = d_cz_tail;
        ta.h_info = d_info;
        ta.h_masks = d_masks;
        // the completion word after the Ctl copy in h_ctl's pinned scratch
        volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(reinterpret_cast<unsigned char *>(c->h_ctl) +
                                                                        sizeof(Ctl) + 32);
        ta.h_done = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(d_ctl) + sizeof(Ctl) + 32);
        // (the ticket is counted on the device, in the word behind the arrival
        // counter, one per tail launch like the host's: the launch's arguments
        // never change, so a captured replay can hold it)
        uint32_t ticket = 0;
        auto expect_tail = [&]() {
            ticket = ++c->tail_ticket;
            *done = 0;
        };
        auto enqueue_tail = [&]() -> hipError_t {
            ops.tail(c->stream, ta);
            return hipGetLastError();
        };
        bool use_graph = !cfg.eager;
        std::vector<unsigned char> key(sizeof(SearchArgs) + 3 * sizeof(int) + sizeof(TailArgs));
        {
            std::memcpy(key.data(), &a, sizeof(SearchArgs));
            const int extra[3] = {(int)expand_grid.x, c->n, KW};
            std::memcpy(key.data() + sizeof(SearchArgs), extra, sizeof(extra));
            std::memcpy(key.data() + sizeof(SearchArgs) + sizeof(extra), &ta, sizeof(TailArgs));
        }
        if (use_graph && c->step_key != key) {  // new arguments: drop the runs captured for the old ones
            for (int gi = 0; gi < kRuns; gi++) {
                if (c->step_exec[gi])
                    (void)hipGraphExecDestroy(c->step_exec[gi]);
                if (c->step_graph[gi])
                    (void)hipGraphDestroy(c->step_graph[gi]);
                c->step_exec[gi] = nullptr;
                c->step_graph[gi] = nullptr;
            }
            c->step_key = key;
        }
        // a run is captured the first time it is needed
        auto run_exec = [&](int gi) -> hipGraphExec_t {
            if (!use_graph || c->step_exec[gi])
                return c->step_exec[gi];
            hipGraph_t graph = nullptr;
            hipGraphExec_t exec = nullptr;
            hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
            hipError_t e2 = e == hipSuccess ? enqueue_steps(kStepRuns[gi]) : e;
            if (e2 == hipSuccess) {  // the replay's tail is its last node (no gap between the last step and it)
                ops.tail(c->stream, ta);
                e2 = hipGetLastError();
            }
            hipError_t e3 = e == hipSuccess ? hipStreamEndCapture(c->stream, &graph) : e;
            if (e2 == hipSuccess && e3 == hipSuccess)
                e3 = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
            if (e2 != hipSuccess || e3 != hipSuccess) {
                if (exec)
                    (void)hipGraphExecDestroy(exec);
                if (graph)
                    (void)hipGraphDestroy(graph);
                (void)hipGetLastError();
                use_graph = false;
                if (cfg.verbose)
                    std::fprintf(stderr, "[pastar] graph capture refused (%s); eager launches\n",
                                 hipGetErrorString(e2 != hipSuccess ? e2 : e3));
                return nullptr;
            }
            c->step_graph[gi] = graph;
            c->step_exec[gi] = exec;
            return exec;
        };

        // wait for a replay by watching the tail's completion word (its last
        // store) rather than for the stream's completion signal; the stream is
        // polled too, so a failure ends the wait with its error
        bool wait_timed_out = false;
        auto wait_tail = [&]() -> hipError_t {
            const double t_wait = now_s();
            for (unsigned spin = 1; *done != ticket; spin++) {
                if ((spin & 255) == 0) {
                    if ((spin & 0xfffff) == 0 && now_s() - t_wait > host_wait_limit_s()) {
                        wait_timed_out = true;
                        return hipErrorNotReady;
                    }
                    const hipError_t q = hipStreamQuery(c->stream);
                    if (q == hipSuccess && *done == ticket)
                        break;
                    if (q != hipErrorNotReady) {
                        const hipError_t e = hipStreamSynchronize(c->stream);
                        if (e != hipSuccess)
                            return e;
                        return *done == ticket ? hipSuccess : hipErrorUnknown;
                    }
                }
            }
            return hipSuccess;
        };
        for (;;) {
            // a launch past the end exits at once (a few us), a replay costs
            // a host round trip (~20 us): the shortest run covering the
            // predicted remainder, the longest beyond it
            int gi = kRuns - 1;
            if (c->last_steps > 0) {
                const long long left = c->last_steps - steps_before;
                gi = 0;
                while (gi < kRuns - 1 && kStepRuns[gi] < left)
                    gi++;
            }
            hipGraphExec_t ex = run_exec(gi);
            expect_tail();
            hipError_t e = ex ? hipGraphLaunch(ex, c->stream) : enqueue_steps(kStepRuns[gi]);
            if (e == hipSuccess && !ex)
                e = enqueue_tail();
            if (e != hipSuccess)
                c->tail_ticket--;  // (no tail was enqueued: the device's count stays where it was)
            if (e == hipSuccess)
                e = wait_tail();
            if (e != hipSuccess) {
                if (wait_timed_out)
                    rc = fail(PASTAR_EDEVWAIT, "the device did not report a replay's end within %.0f s "
                              "(PASTAR_WAIT_TIMEOUT_S); the launch is abandoned", host_wait_limit_s());
                else
                    rc = fail(PASTAR_ENODEV, "search steps failed: %s", hipGetErrorString(e));
                break;
            }
            h = *c->h_ctl;
            const long long ran = h.steps - steps_before;
            launches += ran;
            steps_before = h.steps;
            if (h.status)
                break;
            if (cfg.verbose)
                std::fprintf(stderr, "[pastar] step %lld expanded %llu bucket %d batch %llu pool %llu chunks\n",
                             h.steps, h.expanded, h.cur_b, h.n_batch, h.pool_top);
        }
        if (h.status == 1)
            c->last_steps = h.steps;
        else if (rc == PASTAR_OK)  // a failed search may be retried on regrown buffers: drain first
            HIP_TRY(hipStreamSynchronize(c->stream));
        if (wait_timed_out)
            return rc;  // (nothing below may wait for the stream)
        c->graph_used = use_graph;
        PA_TRY(rc);
    } else {
        // The sharded step protocol, device-driven: the host only enqueues.
        //   main stream   [wait: insert of step i - 1 - lag]  select(i), expand(i)
        //   side stream   [wait: expand(i)]  pack(i), all-to-all(i), insert(i)
        // Every per-step value (record counts, goals, had-work and failure
        // flags) travels in the block headers and is consumed on the device,
        // so the host waits once per round of S steps, for the control block.
        // lag 0: the next select sees this step's received records; lag 1: it
        // runs beside their exchange and insert (they reach the select after).
        const int lag = cfg.xlag;
        if (lag) {
            // the staging arrays of the inserts that run beside a select
            const size_t cap = (size_t)G * (size_t)c->xblock_recs_max;
            if (c->xstage_cap < cap) {
                c->xstage.reset();
                PA_TRY(c->xstage.alloc(2 * cap));
                c->xstage_cap = cap;
            }
            if (!c->xstage_n.p) {
                PA_TRY(c->xstage_n.alloc(2));
                PA_TRY(c->xdrain_arrive.alloc(1));
            }
            HIP_TRY(hipMemsetAsync(c->xstage_n.p, 0, 2 * sizeof(unsigned long long), c->stream));
            HIP_TRY(hipMemsetAsync(c->xdrain_arrive.p, 0, sizeof(unsigned), c->stream));
        }
        XArgs t{};
        t.x = c->xstate.p;
        t.ctl = c->ctl.p;
        t.stats_b = c->stats_b.p;
        t.goal_g = c->goal.p;
        t.outbox = c->outbox.p;
        t.outbox_cap = cfg.outbox_cap;
        t.recv = c->xrecv.p;
        t.n_shards = G;
        t.shard = c->shard;
        t.lag = lag;
        SearchArgs ab = a;  // the insert kernel's arguments: its own statistics, the low_b word
        ab.stats = c->stats_b.p;
        ab.lower = &c->ctl.p->low_b;
        // the block of a round: a power of two of records, sized from the
        // most any shard had to send in a step of the round before (every
        // shard folds the same headers, so every shard picks the same size)
        auto set_block = [&](unsigned long long recs) {
            recs = std::max<unsigned long long>(1, std::min(recs, c->xblock_recs_max));
            c->xblock_recs = recs;
            c->xblock_bytes = (sizeof(XHdr) + recs * rb + 255) & ~(unsigned long long)255;
            t.block_recs = recs;
            t.block_bytes = c->xblock_bytes;
        };
        // (the first round starts from the size the last search on this
        // context ended with)
        set_block(c->xblock_learned ? c->xblock_learned : std::min<unsigned long long>(8192, c->xblock_recs_max));
        if (std::getenv("PASTAR_XCHG_FIXED"))
            set_block(c->xblock_recs_max);
        long long step = 0;
        int rounds = 0;
        bool resized = true;
        for (;;) {
            const unsigned pack_y =
                (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>(32, (c->xblock_recs + 4095) / 4096));
            const unsigned ins_blocks = (unsigned)std::max<unsigned long long>(
                1, std::min<unsigned long long>(1024, ((unsigned long long)G * c->xblock_recs + kBlock - 1) / kBlock));
            // steps this round: what the last search on this context predicts
            // is left (every shard counts the same steps), 16 without one
            // (short rounds while the block size is still following the demand)
            int S = resized ? 8 : 16;
            if (c->last_steps > 0)
                S = (int)std::min<long long>(64, std::max<long long>(4, c->last_steps + 1 - step));
            if (const char *e = std::getenv("PASTAR_XCHG_ROUND"))
                S = std::max(1, std::atoi(e));
            for (int k = 0; k < S; k++, step++) {
                const int ring = (int)(step % kEvRing);
                if (step - 1 - lag >= 0)
                    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_b[(step - 1 - lag) % kEvRing], 0));
                if (lag && step - 2 >= 0) {
                    // the entries insert(step - 2) staged (same parity as this step), into the
                    // open list on this stream, before this step's select
                    SearchArgs ad = a;
                    ad.lower = &c->ctl.p->low_b;
                    hipLaunchKernelGGL(xdrain_kernel, dim3(64), blk, 0, c->stream, ad,
                                       c->xstage.p + (size_t)(step & 1) * c->xstage_cap, c->xstage_n.p + (step & 1),
                                       (unsigned long long)c->xstage_cap, c->xdrain_arrive.p);
                    PA_TRY(check_launch());
                }
                a.step = (int)(step & 0x3fffffff);
                hipLaunchKernelGGL(select_kernel, dim3(1), blk, 0, c->stream, a);
                ops.expand(expand_grid, blk, c->stream, a);
                PA_TRY(check_launch());
                HIP_TRY(hipEventRecord(c->ev_a[ring], c->stream));
                HIP_TRY(hipStreamWaitEvent(c->stream_b, c->ev_a[ring], 0));
                t.step = a.step;
                t.send = c->xsend.p + (size_t)(step & 1) * c->xarea;
                if (lag) {
                    t.stage = c->xstage.p + (size_t)(step & 1) * c->xstage_cap;
                    t.stage_n = c->xstage_n.p + (step & 1);
                    t.stage_cap = (unsigned long long)c->xstage_cap;
                }
                ops.xpack(dim3((unsigned)G, pack_y), blk, c->stream_b, t);
                PA_TRY(check_launch());
                PA_TRY(c->tr->xchg(c, (int)(step & 0x3fffffff)));
                ops.xinsert(dim3(ins_blocks), blk, c->stream_b, ab, t);
                PA_TRY(check_launch());
                HIP_TRY(hipEventRecord(c->ev_b[ring], c->stream_b));
            }
            // the round's one host wait: the control block as the last insert left it
            HIP_TRY(hipMemcpyAsync(c->h_ctl, c->ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream_b));
            {
                const double t_wait = now_s();
                hipError_t q;
                unsigned spin = 0;
                while ((q = hipStreamQuery(c->stream_b)) == hipErrorNotReady) {
                    if ((++spin & 15) == 0 && now_s() - t_wait > host_wait_limit_s()) {
                        const hipError_t qa = hipStreamQuery(c->stream);
                        return fail(PASTAR_EDEVWAIT, "shard %d: the side stream did not finish the round ending at step "
                                    "%lld within %.0f s (main stream: %s); the launches are abandoned", c->shard, step,
                                    host_wait_limit_s(), hipGetErrorString(qa));
                    }
                }
                if (q != hipSuccess)
                    return fail(PASTAR_ENODEV, "sharded steps failed: %s", hipGetErrorString(q));
            }
            rounds++;
            h = *c->h_ctl;
            if (h.status)
                break;
            {
                // next round's block: 1.25 x the largest demand of one
                // (sender, destination) pair, between 4096 records and the allocation
                unsigned long long demand = 0;
                HIP_TRY(hipMemcpy(&demand, &c->xstate.p->demand_max, sizeof(demand), hipMemcpyDeviceToHost));
                HIP_TRY(hipMemsetAsync(&c->xstate.p->demand_max, 0, sizeof(demand), c->stream_b));
                const unsigned long long want = demand * 5 / 4;
                unsigned long long recs = 4096;
                while (recs < want && recs < c->xblock_recs_max)
                    recs <<= 1;
                // (shrinks only by one size a round: a quiet round between two busy ones keeps most of the block)
                if (recs < c->xblock_recs / 2)
                    recs = c->xblock_recs / 2;
                if (std::getenv("PASTAR_XCHG_FIXED"))  // tuning probe: always the largest block
                    recs = c->xblock_recs_max;
                resized = recs != c->xblock_recs;
                set_block(recs);
            }
            if (cfg.verbose)
                std::fprintf(stderr, "[pastar %d/%d] step %lld expanded %llu bucket %d status %d (%.3f s)\n", c->shard, G,
                             step, h.expanded, h.cur_b, h.status, now_s() - t0);
        }
        if (cfg.verbose)
            std::fprintf(stderr, "[pastar %d/%d] loop ends at step %lld: status %d fail mask 0x%x (%.3f s)\n", c->shard, G,
                         step, h.status, h.fail_mask, now_s() - t0);
        // the main stream may still hold steps enqueued past the end (they
        // leave at once); then the totals as both streams left them
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(c->h_ctl, c->ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost));
        h = *c->h_ctl;
        XState xs;
        HIP_TRY(hipMemcpy(&xs, c->xstate.p, sizeof(XState), hipMemcpyDeviceToHost));
        exchanged = (int64_t)xs.sent;
        xchg_backlog_steps = (int64_t)xs.backlog_steps;
        xchg_backlog_max = (int64_t)xs.backlog_max;
        host_waits = rounds;
        h.claimed += xs.claimed_b;
        if (h.status == 1) {
            h.steps = (long long)xs.steps_done;  // the same on every shard
            c->last_steps = h.steps;
            c->xblock_learned = c->xblock_recs;
        }
        if (h.status == 2 && !(h.fail_mask & 0xfff)) {
            // only another shard ran out of capacity
            c->last_fail_mask = 0;
            return fail(PASTAR_ENOMEM, "another shard exhausted its device capacity");
        }
        h.fail_mask &= 0xfff;
    }
    const double t1 = now_s();
    if (h.status == 2) {
        c->last_fail_mask = h.fail_mask;
        return fail(PASTAR_ENOMEM, "device capacity exhausted (mask %d: pool %llu entries, sub-queue %llu entries, "
                    "table 2^%d, outbox %llu)", h.fail_mask, cfg.pool_entries, cfg.subqueue_entries, cfg.table_log2,
                    cfg.outbox_cap);
    }
    if (h.status == 3)
        return fail(PASTAR_ESTATE, "step limit %lld reached", (long long)cfg.max_steps);
    if (h.status == 4) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        return report_fault(c, h.fault_sites);
    }
    // the goal and the open-list census (current entries left in the
    // queues; the table needs none: every claimed slot is a distinct node,
    // every first closing of a node is an expansion that is not a
    // reopening) in one host round trip
    if (!c->census.p)
        PA_TRY(c->census.alloc(5));  // entries left; debug: live, live below the goal, min f, min bucket
    unsigned long long *cnt = c->census.p;
    unsigned long long *cz = reinterpret_cast<unsigned long long *>(c->h_stage);  // pinned
    int32_t *h_goal_end = reinterpret_cast<int32_t *>(c->h_stage + 128);
    c->walk_ready = false;
    if (sharded) {  // (census zeroed by search_init_kernel)
        hipLaunchKernelGGL(queue_census_kernel, dim3(64), blk, 0, c->stream, c->queues.p, cnt, nullptr);
        PA_TRY(check_launch());
        HIP_TRY(hipMemcpyAsync(h_goal_end, c->goal.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(cz, cnt, 40, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    } else {
        // the census, the goal and the backtrace walk came back with the
        // last replay (the walk ran only if the goal was reached):
        // pastar_gpu_alignment needs no launch and no wait of its own
        c->walk_ready = h.status == 1;
    }
    int goal_g = *h_goal_end;
    if (sharded) {
        int64_t mn[1] = {goal_g};
        PA_TRY(allreduce_i64(c, mn, 1, kRedMin));
        goal_g = (int)mn[0];
    }
    if (goal_g == kIntMax)
        return fail(PASTAR_ENOTFOUND, "search exhausted without reaching the goal");
    if (hc.debug) {  // walks every entry left: debug only
        hipLaunchKernelGGL(open_census_kernel<KW>, dim3(256), blk, 0, c->stream, a, goal_g, cnt + 1);
        PA_TRY(check_launch());
        HIP_TRY(hipMemcpyAsync(cz, cnt, 40, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    const unsigned long long open_left = cz[0];
    const unsigned long long census[4] = {cz[1], cz[2], cz[3], cz[4]};
    if (census[1]) {
        Ctl cc;
        HIP_TRY(hipMemcpy(&cc, c->ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[pastar %d/%d] warning: %llu open nodes below the goal %d at termination (min f %llu bucket "
                     "%llu; cur_b %d batch_b %d band 2^%d f0 %d steps %lld)\n",
                     c->shard, G, census[1], goal_g, census[2], census[3], cc.cur_b, cc.batch_b, cc.band_log2, cc.f0,
                     cc.steps);
    }

    c->last_pool_chunks = h.pool_top;
    std::memset(res, 0, sizeof(*res));
    res->score = goal_g;
    res->expansions = (int64_t)h.expanded;
    res->reopen = (int64_t)h.reopen;
    res->generated = (int64_t)h.generated;
    res->open_size = (int64_t)open_left;
    res->closed_size = (int64_t)(h.expanded - h.reopen);
    res->table_used = (int64_t)h.claimed;
    res->steps = h.steps;
    res->exchanged = exchanged;
    res->xchg_backlog_steps = xchg_backlog_steps;
    res->xchg_backlog_max = xchg_backlog_max;
    res->host_waits = host_waits;
    res->seconds = t1 - t0;
    {
        const unsigned long long ticks = h.expand_ticks, timed = h.timed_launches;
        expand_ms = (double)ticks * 1e-5;  // 100 MHz device clock
        launches = h.timing ? (int64_t)timed : (int64_t)h.steps;
    }
    res->expand_ms = expand_ms;
    res->select_ms = (double)h.select_ticks * 1e-5;
    if (cfg.verbose && h.partial_k >= 0 && (c->n >= 7 || h.part_queued))
        std::fprintf(stderr, "[pastar] partial expansion (window %d buckets): %llu parents queued again, %llu taken again, "
                     "%llu entries dropped\n", h.partial_k, h.part_queued, h.part_taken, h.dropped);
    if (cfg.verbose && cfg.profile) {
        std::fprintf(stderr, "[pastar] select phases (us/launch):");
        for (int k = 0; k < 4; k++)
            std::fprintf(stderr, " %.2f", (double)h.phase_ticks[k] * 1e-2 / std::max<double>(1.0, (double)h.timed_launches));
        std::fprintf(stderr, "\n[pastar] expand phases of block 0 (us/launch):");
        for (int k = 0; k < 10; k++)
            std::fprintf(stderr, " %.2f", (double)h.body_ticks[k] * 1e-2 / std::max<double>(1.0, (double)h.body_launches));
        const double nb = std::max<double>(1.0, (double)h.blk_stats[0]);
        std::fprintf(stderr, "\n[pastar] blocks %llu over %llu launches: levels mean %.1f max %llu, rounds mean %.1f max %llu, "
                     "longest block %.2f us\n", h.blk_stats[0], h.body_launches, h.blk_stats[1] / nb, h.blk_stats[2],
                     h.blk_stats[3] / nb, h.blk_stats[4], h.blk_stats[5] * 1e-2);
        std::fprintf(stderr, "[pastar] continuation levels by parents: 1: %llu, 2-4: %llu, 5-16: %llu, more: %llu\n",
                     h.blk_stats[6], h.blk_stats[7], h.blk_stats[8], h.blk_stats[9]);
        std::fprintf(stderr, "[pastar] dive phases of block 0 (us/launch): gather %.2f levels %.2f relax %.2f\n",
                     (double)h.body_ticks[12] * 1e-2 / std::max<double>(1.0, (double)h.body_launches),
                     (double)h.body_ticks[13] * 1e-2 / std::max<double>(1.0, (double)h.body_launches),
                     (double)h.body_ticks[14] * 1e-2 / std::max<double>(1.0, (double)h.body_launches));
        std::fprintf(stderr, "[pastar] dives %llu (one start node %llu, several %llu), levels %llu, by levels 0: %llu 1: %llu "
                     "2: %llu 3+: %llu, children %llu\n", h.body_ticks[10], h.phase_ticks[0], h.phase_ticks[1], h.body_ticks[11],
                     h.phase_ticks[4], h.phase_ticks[5], h.phase_ticks[6], h.phase_ticks[7], h.phase_ticks[2]);
#ifdef PASTAR_PHASE_TIMERS
        if (!sharded)
            std::fprintf(stderr, "[pastar] tail (us): walk %.2f; last block %llu: own work %.2f, arrival and fences %.2f, "
                         "copies to the host %.2f; walk's start to the copies' end %.2f\n", (double)(cz[14] - cz[13]) * 1e-2,
                         cz[12], (double)(cz[9] - cz[8]) * 1e-2, (double)(cz[10] - cz[9]) * 1e-2,
                         (double)(cz[11] - cz[10]) * 1e-2, (double)(cz[11] - cz[13]) * 1e-2);
        if (!sharded)
            std::fprintf(stderr, "[pastar] walk (us): set-up %.2f, first round trip %.2f, the other %llu %.2f, of which "
                         "%.2f from a round's start to its records' arrival\n", (double)cz[5] * 1e-2, (double)cz[6] * 1e-2,
                         cz[15] > 1 ? cz[15] - 2 : 0ull, (double)cz[7] * 1e-2, (double)cz[17] * 1e-2);
#endif
    }
    res->gap_ms = (double)h.gap_ticks * 1e-5;
    res->expand_launches = launches;
    res->expand_parents = (int64_t)h.parents;
    int64_t all[1] = {(int64_t)h.expanded};
    if (sharded)
        PA_TRY(allreduce_i64(c, all, 1, kRedSum));
    // the goal's acceptance counts as one expansion (PAStar.cpp:341)
    res->expansions_all = all[0] + 1;
    c->searched = true;
    c->score = goal_g;
    return PASTAR_OK;
}

// ---------------------------------------------------------------------------
// LDS-resident search of a small problem (solo.hpp): PairAlign, the A* and
// the backtrace in one single-workgroup launch.
// ---------------------------------------------------------------------------
struct SoloPlan {
    SoloArgs a;
    size_t lds;
};

// The LDS layout, or false when the problem does not take the solo path:
// equal gap costs, 1-word keys, one shard, 2..8 sequences, and the pair
// tables plus a node table of at least 2^kSoloMinCapLog2 slots in 160 KB.
bool solo_plan(const pastar_ctx *c, SoloPlan *pl)
{
    if (c->tr || c->kw != 1 || c->n < 2 || c->n > 8 || c->hp.gap_open != c->hp.gap_ext)
        return false;
    if (c->hp.kshift[c->n - 1] + c->hp.kbits[c->n - 1] > kSoloKeyBits)
        return false;  // coordinates in 31 bits (32-bit keys)
    auto align16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t cells = 0;
    for (int k = 0; k < c->npairs; k++)
        cells += (size_t)(c->hp.len[c->hp.pair_x[k]] + 1) * (c->hp.len[c->hp.pair_y[k]] + 1);
    SoloArgs &a = pl->a;
    std::memset(&a, 0, sizeof(a));
    size_t off = align16(cells * 8);
    a.off_prob = (int)off;
    off = align16(off + sizeof(DevProblem));
    a.off_sub = (int)off;
    off = align16(off + (size_t)c->hp.alpha * c->hp.alpha * 4);
    a.off_codes = (int)off;
    off = align16(off + c->codes_len);
    a.off_subw = (int)off;  // a pre-weighted distance table per wave
    off = align16(off + (size_t)(kSoloThreads / 64) * (c->hp.alpha * c->hp.alpha + 1) * 4);
    if (off >= (size_t)kSoloLds)
        return false;
    int lg = kSoloMaxCapLog2;
    while (lg >= kSoloMinCapLog2 && off + ((size_t)kSoloSlotBytes << lg) > (size_t)kSoloLds)
        lg--;
    if (lg < kSoloMinCapLog2)
        return false;
    const size_t C = (size_t)1 << lg;
    a.off_best = (int)off;  // 8-B arrays first
    a.off_hcl = (int)(off + 8 * C);
    a.off_open = (int)(off + 16 * C);
    a.off_batch = (int)(off + 24 * C);  // 2 x C/4 entries of 16 B
    a.off_keys = (int)(off + 32 * C);   // 4-B keys last
    a.cap_log2 = lg;
    a.hc_cells = (int)cells;
    a.codes_len = (int)c->codes_len;
    a.alpha2 = c->hp.alpha * c->hp.alpha;
    pl->lds = off + kSoloSlotBytes * C;
    return true;
}

template <int N>
const void *solo_fn()
{
    return (const void *)solo_kernel<N>;
}

const void *solo_fn_for(int n)
{
    switch (n) {
    case 2: return solo_fn<2>();
    case 3: return solo_fn<3>();
    case 4: return solo_fn<4>();
    case 5: return solo_fn<5>();
    case 6: return solo_fn<6>();
    case 7: return solo_fn<7>();
    default: return solo_fn<8>();
    }
}

template <int N>
const void *solo_many_fn()
{
    return (const void *)solo_many_kernel<N>;
}

const void *solo_many_fn_for(int n)
{
    switch (n) {
    case 2: return solo_many_fn<2>();
    case 3: return solo_many_fn<3>();
    case 4: return solo_many_fn<4>();
    case 5: return solo_many_fn<5>();
    case 6: return solo_many_fn<6>();
    case 7: return solo_many_fn<7>();
    default: return solo_many_fn<8>();
    }
}

// The kernel arguments of one LDS-resident search on context c, its result
// areas (pinned host memory, the node-table dump) made ready; *done_out is
// the host view of the completion word, cleared.
int solo_prepare(pastar_ctx *c, const SearchCfg &cfg, const SoloPlan &pl, SoloArgs *out, volatile uint32_t **done_out)
{
    int total_len = 0;
    for (int i = 0; i < c->n; i++)
        total_len += c->hp.len[i];
    // SoloOut, the path's masks, then the completion word
    const size_t done_off = (sizeof(SoloOut) + 4 * ((size_t)total_len + 1) + 63) & ~(size_t)63;
    const size_t out_bytes = done_off + 64;
    const size_t C = (size_t)1 << pl.a.cap_log2;
    if (c->solo_dump.n < 4 * C)
        PA_TRY(c->solo_dump.alloc(4 * C));
    if (c->h_solo_n < out_bytes) {
        if (c->h_solo)
            (void)hipHostFree(c->h_solo);
        c->h_solo = nullptr;
        c->h_solo_n = 0;
        HIP_TRY(hipHostMalloc((void **)&c->h_solo, out_bytes, hipHostMallocDefault));
        c->h_solo_n = out_bytes;
        c->many_cached = false;  // (a cached launch record points into the old area)
    }
    PA_TRY(ensure_walk_buffers(c, total_len));
    SoloArgs a = pl.a;
    a.P = c->dP.p;
    a.codes = c->dcodes.p;
    a.sub = c->dsub.p;
    // the result record and the path go straight to pinned host memory (no
    // copy after the launch)
    unsigned char *d_out = nullptr;
    PA_TRY(host_alias(c->h_solo, &d_out));
    a.out = reinterpret_cast<SoloOut *>(d_out);
    a.masks = reinterpret_cast<int32_t *>(d_out + sizeof(SoloOut));
    a.done = reinterpret_cast<uint32_t *>(d_out + done_off);
    a.ticket = ++c->solo_ticket;
    volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(c->h_solo + done_off);
    *done = 0;  // (a fresh allocation holds anything)
    a.dump = c->solo_dump.p;
    a.max_path = total_len + 1;
    a.max_levels = cfg.max_steps > 0 ? cfg.max_steps : (1ll << 40);
    a.band_log2 = -1;
    if (cfg.band > 0) {
        int w = 0;
        PA_TRY(estimate_band_log2(c, 0, cfg.band, &w));
        a.band_log2 = w;
    }
    *out = a;
    *done_out = done;
    return PASTAR_OK;
}

// Wait for a completion word (the kernel's last store) rather than for the
// stream's completion signal, a few microseconds later; the stream is still
// polled, so a failed launch ends the wait with its error.
int solo_wait(hipStream_t stream, volatile uint32_t *done, uint32_t ticket, double t0)
{
    for (unsigned spin = 1; *done != ticket; spin++) {
        if ((spin & 255) == 0) {
            if ((spin & 0xfffff) == 0 && now_s() - t0 > host_wait_limit_s())
                return fail(PASTAR_EDEVWAIT, "the LDS-resident search did not report its end within %.0f s "
                            "(PASTAR_WAIT_TIMEOUT_S); the launch is abandoned", host_wait_limit_s());
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess && *done == ticket)
                break;
            if (q != hipErrorNotReady) {
                HIP_TRY(hipStreamSynchronize(stream));
                if (*done != ticket)
                    return fail(PASTAR_ENODEV, "LDS-resident search ended without its result");
                break;
            }
        }
    }
    return PASTAR_OK;
}

// The result of an LDS-resident search from its pinned record.
int solo_finish(pastar_ctx *c, const SearchCfg &cfg, int cap_log2, double seconds, pastar_result *res)
{
    int total_len = 0;
    for (int i = 0; i < c->n; i++)
        total_len += c->hp.len[i];
    const size_t C = (size_t)1 << cap_log2;
    SoloOut o;
    std::memcpy(&o, c->h_solo, sizeof(o));
    if (cfg.verbose)
        std::fprintf(stderr, "[pastar solo] status %d levels %d (%llu pile cuts) cap %d: tables %.2f us, search %.2f us, tail %.2f us\n",
                     o.status, o.levels, o.pile_cuts, o.cap, (o.t_tables - o.t_start) * 1e-2, (o.t_search - o.t_tables) * 1e-2,
                     (o.t_end - o.t_search) * 1e-2);
    if (cfg.verbose && o.phase[0] + o.phase[1] + o.phase[2] + o.phase[3])
        std::fprintf(stderr, "[pastar solo] per level (core clocks): top %.0f, entry+reads %.0f, children+relax %.0f, "
                     "push+tail %.0f\n", (double)o.phase[0] / o.levels, (double)o.phase[1] / o.levels,
                     (double)o.phase[2] / o.levels, (double)o.phase[3] / o.levels);
    if (o.status == 2)
        return fail(PASTAR_ENOMEM, "LDS-resident search outgrew its %d-slot node table", o.cap);
    if (o.status == 4)
        return fail(PASTAR_ESTATE, "step limit %lld reached", (long long)cfg.max_steps);
    if (o.status != 1 || o.score == kIntMax)
        return fail(PASTAR_ENOTFOUND, "search exhausted without reaching the goal");
    // the backtrace rides on the same copy (pastar_gpu_alignment reads it)
    std::memcpy(c->h_walk_masks, c->h_solo + sizeof(SoloOut), 4 * (size_t)std::min(o.path_len, total_len + 1));
    int *h_info = reinterpret_cast<int *>(c->h_walk + 4);
    h_info[0] = o.path_len;
    h_info[1] = o.path_status;
    c->walk_ready = true;
    c->solo_active = true;
    c->solo_cap_log2 = cap_log2;
    std::memset(res, 0, sizeof(*res));
    res->score = o.score;
    res->expansions = (int64_t)o.expanded;
    res->expansions_all = (int64_t)o.expanded + 1;  // the goal's acceptance (PAStar.cpp:341)
    res->reopen = (int64_t)o.reopen;
    res->generated = (int64_t)o.generated;
    res->open_size = (int64_t)o.open_left;
    res->closed_size = (int64_t)(o.expanded - o.reopen);
    res->table_used = (int64_t)o.claimed;
    res->steps = o.levels;
    res->seconds = seconds;
    res->expand_ms = (double)(o.t_end - o.t_start) * 1e-5;
    res->expand_launches = 1;
    res->expand_parents = (int64_t)(o.expanded + o.dropped);
    res->table_slots = (int64_t)C;
    res->solo = 1;
    c->searched = true;
    c->score = o.score;
    return PASTAR_OK;
}

// Returns PASTAR_ENOMEM when the search outgrew the LDS node table (the
// caller then runs the batched engine).
int solo_search(pastar_ctx *c, const SearchCfg &cfg, SoloPlan &pl, pastar_result *res)
{
    SoloArgs a;
    volatile uint32_t *done = nullptr;
    PA_TRY(solo_prepare(c, cfg, pl, &a, &done));
    const void *fn = solo_fn_for(c->n);
    if (!(c->solo_attr_done & (1u << c->n))) {
        HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kSoloLds));
        c->solo_attr_done |= 1u << c->n;
    }
    void *args[] = {(void *)&a};
    const double t0 = now_s();
    HIP_TRY(hipLaunchKernel(fn, dim3(1), dim3(kSoloThreads), args, pl.lds, c->stream));
    PA_TRY(check_launch());
    PA_TRY(solo_wait(c->stream, done, a.ticket, t0));
    return solo_finish(c, cfg, pl.a.cap_log2, now_s() - t0, res);
}

}  // namespace

extern "C" {

int pastar_gpu_search(pastar_ctx *c, const pastar_search_opts *opts, pastar_result *res)
{
    if (!c || !res)
        return fail(PASTAR_EINVAL, "null argument");
    // a failed search must not leave an earlier search's result readable
    // (the node table then holds this search's partial state)
    c->walk_ready = false;
    c->searched = false;
    c->score = -1;
    c->lists_ready = false;  // the search reuses the list session's buffers
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    HIP_TRY(hipSetDevice(c->device));
    pastar_search_opts o{};
    if (opts)
        o = *opts;
    SearchCfg cfg;
    const unsigned long long masks = (1ull << c->n) - 1;
    // most parents per step: up to N = 6 see below; 65536 beyond (syn8x400
    // 72 ms at 65536 and at 131072)
    if (o.batch_nodes > (1ll << 30))  // batch offsets are 32-bit on the device
        return fail(PASTAR_EINVAL, "batch_nodes %lld above 2^30", (long long)o.batch_nodes);
    // (round 2: 262144 up to N = 6, kinase 16.7 -> 15.2 ms, narrower inputs
    // flat; profiles/r2_tune_batch.txt)
    cfg.kmax = o.batch_nodes > 0 ? (unsigned long long)o.batch_nodes : (c->n <= 6 ? 262144ull : 65536ull);
    // sharded: the shards together take about twice the one-shard batch per
    // step.  A fat bucket is expanded in slices, and what one slice relaxes
    // spares the next slices the nodes it improves; G full-size slices at
    // once expand those nodes too (syn8x400 at 8 shards: 10.5 M expansions at
    // 65536 a shard, 6.6 M at 16384, 5.8 M on one shard)
    if (o.batch_nodes <= 0 && c->n_shards > 1)
        cfg.kmax = std::max<unsigned long long>(4096, 2 * cfg.kmax / (unsigned long long)c->n_shards);
    cfg.kmin = o.batch_min > 0 ? std::min<unsigned long long>((unsigned long long)o.batch_min, cfg.kmax) : cfg.kmax / 8;
    // default node-table size: learned from the last search on this context
    // (a repeated search of the same problem initialises only what it
    // needs), else 2^24 slots (512 MB, cleared in ~0.1 ms: kinase's first
    // search then runs without a capacity restart; tools/gpu/cold_probe.py)
    // (an explicit size is a floor: a repeated search never restarts below
    // what the last one needed)
    // (N >= 7: 2^26, 2 GB: syn8x400's first search ran 164 ms with a
    // capacity restart from 2^24 against 73 ms warm)
    cfg.table_log2 = o.table_slots_log2 > 0 ? std::max((int)o.table_slots_log2, c->learned_log2)
                                            : (c->learned_log2 > 0 ? c->learned_log2 : (c->n >= 7 ? 26 : 24));
    if (cfg.table_log2 < 10 || cfg.table_log2 > 32)
        return fail(PASTAR_EINVAL, "table_slots_log2 %d outside [10, 32]", cfg.table_log2);
    // (the pool is never cleared: its size costs memory only, 2 GB here)
    cfg.pool_entries = o.pool_entries > 0 ? (unsigned long long)o.pool_entries : (1ull << 28);
    cfg.subqueue_entries = o.subqueue_entries > 0 ? (unsigned long long)o.subqueue_entries : (1ull << 20);
    // the ring of records for one destination shard: a power of two, at
    // least four exchange blocks (what a step cannot send waits in the ring)
    cfg.xblock_recs = o.xchg_block_records > 0 ? (unsigned long long)o.xchg_block_records : (1ull << 20);
    if (const char *e = std::getenv("PASTAR_XCHG_BLOCK"))  // tuning override
        cfg.xblock_recs = std::max(1ull, std::strtoull(e, nullptr, 10));
    if (cfg.xblock_recs > (1ull << 24))
        return fail(PASTAR_EINVAL, "xchg_block_records %llu above 2^24", cfg.xblock_recs);
    cfg.xlag = o.xchg_lag;
    if (o.partial < -1 || o.partial > 1024)
        return fail(PASTAR_EINVAL, "partial %d outside [-1, 1024]", o.partial);
    cfg.partial_k = o.partial == 0 ? 1 : o.partial - 1;  // (-1: off)
    if (const char *e = std::getenv("PASTAR_XCHG_LAG"))  // tuning override
        cfg.xlag = std::atoi(e);
    if (cfg.xlag < 0 || cfg.xlag > 1)
        return fail(PASTAR_EINVAL, "xchg_lag %d outside [0, 1]", cfg.xlag);
    cfg.outbox_cap = std::max<unsigned long long>({1ull << 16, cfg.kmax * masks / std::max(1, c->n_shards),
                                                   2 * cfg.xblock_recs});
    cfg.table_log2 = std::max(cfg.table_log2, c->grown_log2);
    cfg.pool_entries = std::max(cfg.pool_entries, c->grown_pool);
    cfg.subqueue_entries = std::max(cfg.subqueue_entries, c->grown_maxch * (unsigned long long)kChunk);
    cfg.outbox_cap = std::max(cfg.outbox_cap, c->grown_outbox);
    {
        unsigned long long p2 = 1;
        while (p2 < cfg.outbox_cap)
            p2 <<= 1;
        cfg.outbox_cap = p2;
    }
    cfg.verbose = o.verbose;
    cfg.profile = o.profile;
    cfg.eager = o.eager;
    if (o.depth < 0 || o.depth > 1024)
        return fail(PASTAR_EINVAL, "depth %d outside [0, 1024]", o.depth);
    // levels per launch: the cheaper an expansion, the deeper (PF08184 0.40
    // -> 0.22 ms at 64, 2 launches; syn4x200 1.52 -> 1.44 ms at 12 with one
    // round; profiles/r1_depth_sweep.txt)
    // (round 2, with 1024 block-rounds per continuation level: N <= 4 at
    // 128 levels is the best or tied on 4 of 5 inputs of 3..4 x 150..400,
    // syn4x200 1.48 -> 1.17 ms; N = 5, 6 at 8: kinase is best at 6..12,
    // narrower inputs at 12..32; profiles/r2_tune_depth.txt)
    cfg.depth = o.depth > 0 ? o.depth : (c->n <= 4 ? 128 : 8);
    cfg.band = o.band;
    cfg.max_steps = o.max_steps;
    if (o.mode < PASTAR_MODE_AUTO || o.mode > PASTAR_MODE_SOLO)
        return fail(PASTAR_EINVAL, "search mode %d", o.mode);
    // a small problem runs whole in one workgroup's LDS (solo.hpp); one that
    // outgrows it runs on the batched engine from then on
    {
        SoloPlan pl;
        const bool fits = solo_plan(c, &pl);
        if (o.mode == PASTAR_MODE_SOLO && !fits)
            return fail(PASTAR_EINVAL, "the problem does not fit the LDS-resident search");
        if (fits && (o.mode == PASTAR_MODE_SOLO || (o.mode == PASTAR_MODE_AUTO && !c->solo_failed))) {
            const int src = solo_search(c, cfg, pl, res);
            if (src != PASTAR_ENOMEM || o.mode == PASTAR_MODE_SOLO)
                return src;
            c->solo_failed = true;
        }
    }
    int rc = PASTAR_OK, retries = 0;
    for (;;) {
        c->last_fail_mask = 0;
        if (c->kw == 1)
            rc = search_impl<1>(c, cfg, res);
        else if (c->kw == 2)
            rc = search_impl<2>(c, cfg, res);
        else
            rc = search_impl<4>(c, cfg, res);
        if (rc != PASTAR_ENOMEM || o.no_autogrow || retries >= 8)
            break;
        int mask = c->last_fail_mask;
        if (c->tr) {  // every shard grows the same way
            int64_t bits[4] = {mask & 1, (mask >> 1) & 1, (mask >> 2) & 1, (mask >> 3) & 1};
            const std::string err = g_err;
            if (allreduce_i64(c, bits, 4, kRedSum) != PASTAR_OK)
                break;
            g_err = err;
            mask = (bits[0] ? 1 : 0) | (bits[1] ? 2 : 0) | (bits[2] ? 4 : 0) | (bits[3] ? 8 : 0);
        }
        if (!mask)
            break;
        // a restart repeats the search up to the failure: the pool (memory
        // only) grows by 16x, the table (cleared by every search) by 4x
        if (mask & kFailNear)
            cfg.pool_entries *= 16;
        if (mask & kFailFar)
            cfg.subqueue_entries *= 4;
        if (mask & kFailTable)
            cfg.table_log2 = std::min(32, cfg.table_log2 + 2);
        if (mask & kFailOut)
            cfg.outbox_cap *= 4;
        c->grown_pool = cfg.pool_entries;
        c->grown_maxch = maxch_of(cfg);
        c->grown_log2 = cfg.table_log2;
        c->grown_outbox = cfg.outbox_cap;
        retries++;
        if (cfg.verbose)
            std::fprintf(stderr, "[pastar] capacity grow (mask %d): pool %llu sub-queue %llu table 2^%d outbox %llu\n",
                         mask, cfg.pool_entries, cfg.subqueue_entries, cfg.table_log2, cfg.outbox_cap);
    }
    if (rc == PASTAR_OK) {
        // size the next search from this one's use, with headroom, so that
        // a repeated search of similar size does not restart (the table is
        // grown when 70% full) and probes stay short: load <= 25%, and 1.5x
        // the chunks used
        const unsigned long long want = (unsigned long long)((double)res->table_used / 0.25) + 1;
        int lg = 16;
        while (lg < 32 && (1ull << lg) < want)
            lg++;
        c->learned_log2 = lg;
        // a table grown past this search's need (25% load) is not kept as
        // the floor of later searches: each one clears its whole table
        c->grown_log2 = std::min(c->grown_log2, lg);
        c->grown_pool = std::max(c->grown_pool, c->last_pool_chunks * (unsigned long long)kChunk * 3 / 2);
        res->capacity_retries = retries;
        res->table_slots = (int64_t)c->nslots;
        res->pool_entries = (int64_t)cfg.pool_entries;
        res->subqueue_entries = (int64_t)cfg.subqueue_entries;
        res->graph_replay = c->graph_used ? 1 : 0;
    }
    if (rc != PASTAR_OK && rc != PASTAR_ENOMEM && c->tr)
        c->tr->abort();  // (a capacity failure is agreed on by every shard: nobody is left waiting)
    return rc;
}

int pastar_gpu_closed_lookup(pastar_ctx *c, const uint16_t *pos, pastar_node *out)
{
    if (!c || !pos || !out)
        return fail(PASTAR_EINVAL, "null argument");
    if (!c->searched)
        return fail(PASTAR_ESTATE, "no search has run on this context");
    HIP_TRY(hipSetDevice(c->device));
    uint64_t key[4];
    pack_key(c, pos, key);
    DevBuf<uint64_t> dk, dout;
    PA_TRY(dk.alloc(4));
    PA_TRY(dout.alloc(3));
    HIP_TRY(hipMemcpyAsync(dk.p, key, 32, hipMemcpyHostToDevice, c->stream));
    // the node table of the last search: the main table, or the LDS-resident
    // search's dump (same slot layout)
    if (c->solo_active)
        hipLaunchKernelGGL(solo_lookup_kernel, dim3(1), dim3(1), 0, c->stream, c->solo_dump.p, c->solo_cap_log2, dk.p,
                           dout.p);
    else
        ops_for(c).lookup(c->stream, c->table.p, c->nslots - 1, dk.p, dout.p);
    PA_TRY(check_launch());
    uint64_t r[3];
    HIP_TRY(hipMemcpyAsync(r, dout.p, 24, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!r[0])
        return fail(PASTAR_ENOTFOUND, "coordinate not in the node table of shard %d", c->shard);
    std::memset(out, 0, sizeof(*out));
    std::memcpy(out->pos, pos, sizeof(uint16_t) * c->n);
    out->g = (int32_t)(r[1] >> 32);
    out->parent_mask = (int32_t)(uint32_t)r[1];
    out->f = out->g + (int32_t)(r[2] >> 32);
    return PASTAR_OK;
}

int pastar_gpu_alignment(pastar_ctx *c, char *rows, int stride, int *cols)
{
    if (!c || !rows || !cols)
        return fail(PASTAR_EINVAL, "null argument");
    if (!c->searched)
        return fail(PASTAR_ESTATE, "no search has run on this context");
    HIP_TRY(hipSetDevice(c->device));
    int total_len = 0;
    for (int i = 0; i < c->n; i++)
        total_len += c->hp.len[i];
    if (stride < total_len + 1)
        return fail(PASTAR_EINVAL, "stride %d < %d", stride, total_len + 1);
    // walk buffers live on the context (allocated once, grown with the
    // path length): a backtrace costs no allocation
    PA_TRY(ensure_walk_buffers(c, total_len));
    int32_t *dmasks = c->walk_masks.p;
    int *dinfo = c->walk_info.p;
    int *h_info = reinterpret_cast<int *>(c->h_walk + 4);  // pinned: h_walk[0..3] is the key
    // walk from the goal towards the origin; with several shards the walk
    // hops to the owner of each parent (PAStarDistributedBacktrace.cpp:19-213)
    std::vector<uint16_t> pos(PASTAR_MAX_SEQ, 0);
    for (int i = 0; i < c->n; i++)
        pos[i] = (uint16_t)c->hp.len[i];
    std::vector<int32_t> path;  // masks from the goal backwards
    const int G = c->n_shards;
    for (int guard = 0; guard <= total_len + 1; guard++) {
        bool origin = true;
        for (int i = 0; i < c->n; i++)
            origin &= pos[i] == 0;
        if (origin)
            break;
        const int owner = G > 1 ? owner_of(c->n, pos.data(), G, c->hp.hash_type, c->hp.hash_shift) : 0;
        // one host round trip per hop: the owner walks its stretch of the
        // chain, and with several shards the stretch (status, length, masks:
        // a fixed-size copy, so nobody needs the length first) goes to all
        if (guard == 0 && c->walk_ready) {
            // walked at the end of the search, results already on the host
        } else {
            if (owner == c->shard)
                PA_TRY(enqueue_walk(c, pos.data(), total_len, G > 1));
            if (c->tr) {
                PA_TRY(c->tr->broadcast(c, dinfo, 8, owner));
                PA_TRY(c->tr->broadcast(c, dmasks, 4 * (size_t)(total_len + 1), owner));
            }
            HIP_TRY(hipMemcpyAsync(h_info, dinfo, 8, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipMemcpyAsync(c->h_walk_masks, dmasks, 4 * ((size_t)total_len + 1), hipMemcpyDeviceToHost,
                                   c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        const int info[2] = {h_info[0], h_info[1]};
        if (info[1] < 0 || info[1] == 2)
            return fail(PASTAR_ENOTFOUND, "backtrace broken at step %d (status %d, shard %d)", info[0], info[1], owner);
        if (info[0] < 0 || info[0] > total_len + 1)
            return fail(PASTAR_ENOTFOUND, "backtrace stretch of %d steps out of range", info[0]);
        const std::vector<int32_t> seg(c->h_walk_masks, c->h_walk_masks + info[0]);
        for (int32_t m : seg) {
            path.push_back(m);
            for (int i = 0; i < c->n; i++)
                pos[i] = (uint16_t)(pos[i] - ((m >> i) & 1));
        }
        if (info[0] == 0)
            return fail(PASTAR_ENOTFOUND, "backtrace made no progress");
    }
    const int L = (int)path.size();
    std::vector<int> at(c->n, 0);
    for (int k = 0; k < L; k++) {
        const int32_t m = path[(size_t)(L - 1 - k)];
        for (int i = 0; i < c->n; i++) {
            if ((m >> i) & 1)
                rows[(size_t)i * stride + k] = c->seqs[i][at[i]++];
            else
                rows[(size_t)i * stride + k] = '-';
        }
    }
    for (int i = 0; i < c->n; i++)
        rows[(size_t)i * stride + L] = '\0';
    *cols = L;
    return PASTAR_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Transport implementations
// ---------------------------------------------------------------------------
namespace {

int RcclTransport::allreduce(pastar_ctx *c, int64_t *vals, int count, RedOp op)
{
    int64_t *d = c->xred.p;  // 64 values, persistent
    HIP_TRY(hipMemcpyAsync(d, vals, sizeof(int64_t) * count, hipMemcpyHostToDevice, c->stream));
    const ncclRedOp_t nop = op == kRedSum ? ncclSum : (op == kRedMin ? ncclMin : ncclMax);
    NCCL_TRY(ncclAllReduce(d, d, (size_t)count, ncclInt64, nop, comm_, c->stream));
    HIP_TRY(hipMemcpyAsync(vals, d, sizeof(int64_t) * count, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return PASTAR_OK;
}

int RcclTransport::xchg(pastar_ctx *c, int step)
{
    const int G = c->n_shards;
    const size_t bb = c->xblock_bytes;
    unsigned char *send = c->xsend.p + (size_t)(step & 1) * c->xarea;
    ncclComm_t comm = xcomm_ ? xcomm_ : comm_;
    NCCL_TRY(ncclGroupStart());
    for (int d = 0; d < G; d++) {
        // (a one-rank communicator exchanges its own, empty, block with
        // itself, so that this path runs whatever the world size)
        if (d == c->shard && G > 1)
            continue;
        NCCL_TRY(ncclSend(send + (size_t)d * bb, bb, ncclUint8, d, comm, c->stream_b));
        NCCL_TRY(ncclRecv(c->xrecv.p + (size_t)d * bb, bb, ncclUint8, d, comm, c->stream_b));
    }
    NCCL_TRY(ncclGroupEnd());
    return PASTAR_OK;
}

int RcclTransport::broadcast(pastar_ctx *c, void *dev, size_t bytes, int root)
{
    NCCL_TRY(ncclBroadcast(dev, dev, bytes, ncclUint8, root, comm_, c->stream));
    return PASTAR_OK;
}

int LocalTransport::xchg_setup(pastar_ctx *c)
{
    if (!g_->ev_pack[rank_][0])
        for (int k = 0; k < kEvRing; k++)
            HIP_TRY(hipEventCreateWithFlags(&g_->ev_pack[rank_][k], hipEventDisableTiming));
    g_->xsend[rank_] = {c->xsend.p, c->xsend.p + c->xarea};
    g_->device[rank_] = c->device;
    return sync();  // every shard's addresses and events are published
}

int LocalTransport::xchg(pastar_ctx *c, int step)
{
    const int G = g_->G, ring = step % kEvRing, par = step & 1;
    // this shard's blocks are packed once the side stream reaches this event;
    // the host barrier orders every shard's record before any shard's wait
    HIP_TRY(hipEventRecord(g_->ev_pack[rank_][ring], c->stream_b));
    PA_TRY(sync());
    XPeers p{};
    for (int s = 0; s < G; s++) {
        p.src[s] = g_->xsend[s][par] + (size_t)rank_ * c->xblock_bytes;
        if (s != rank_)
            HIP_TRY(hipStreamWaitEvent(c->stream_b, g_->ev_pack[s][ring], 0));
    }
    const unsigned y = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>(32, (c->xblock_recs + 4095) / 4096));
    hipLaunchKernelGGL(xcopy_kernel, dim3((unsigned)G, y), dim3(kBlock), 0, c->stream_b, p, c->xrecv.p,
                       c->xblock_bytes, (unsigned long long)remote_bytes(c->kw), rank_);
    return check_launch();
}

int LocalTransport::broadcast(pastar_ctx *c, void *dev, size_t bytes, int root)
{
    HIP_TRY(hipStreamSynchronize(c->stream));
    g_->bufs[rank_] = dev;
    g_->device[rank_] = c->device;
    PA_TRY(sync());
    if (rank_ != root) {
        HIP_TRY(hipMemcpyPeerAsync(dev, c->device, g_->bufs[root], g_->device[root], bytes, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return sync();
}

}  // namespace

extern "C" {

int pastar_group_create(int n_shards, pastar_group **out)
{
    if (!out || n_shards < 1 || n_shards > 8)
        return fail(PASTAR_EINVAL, "invalid group size %d (1..8)", n_shards);
    pastar_group *g = new pastar_group();
    g->G = n_shards;
    g->vals.resize(n_shards);
    g->counts.resize(n_shards);
    g->xsend.resize(n_shards);
    g->ev_pack.resize(n_shards);
    for (auto &r : g->ev_pack)
        r.fill(nullptr);
    g->bufs.resize(n_shards, nullptr);
    g->device.resize(n_shards, 0);
    *out = g;
    return PASTAR_OK;
}

void pastar_group_destroy(pastar_group *g)
{
    if (!g)
        return;
    for (auto &r : g->ev_pack)
        for (hipEvent_t e : r)
            if (e)
                (void)hipEventDestroy(e);
    delete g;
}

int pastar_gpu_create_grouped(const pastar_problem *p, int device, pastar_group *group, int shard_rank,
                              pastar_ctx **out)
{
    if (!group || !out)
        return fail(PASTAR_EINVAL, "null argument");
    if (shard_rank < 0 || shard_rank >= group->G)
        return fail(PASTAR_EINVAL, "shard %d outside group of %d", shard_rank, group->G);
    // a context with one shard, then joined to the group
    PA_TRY(pastar_gpu_create(p, device, 1, 0, nullptr, out));
    pastar_ctx *c = *out;
    c->n_shards = group->G;
    c->shard = shard_rank;
    c->hp.n_shards = group->G;
    c->hp.shard = shard_rank;
    HIP_TRY(hipMemcpy(c->dP.p, &c->hp, sizeof(c->hp), hipMemcpyHostToDevice));
    if (group->G > 1) {
        PA_TRY(c->xred.alloc(64));
        c->tr.reset(new LocalTransport(group, shard_rank));
        group->members++;
        PA_TRY(create_side_stream(c));
        for (int d = 0; d < 8; d++) {  // peer access for the copies, where the link allows it
            int ok = 0;
            if (d != device && hipDeviceCanAccessPeer(&ok, device, d) == hipSuccess && ok)
                (void)hipDeviceEnablePeerAccess(d, 0);
        }
        (void)hipGetLastError();
    }
    return PASTAR_OK;
}

}  // extern "C"

extern "C" {

int pastar_gpu_allreduce(pastar_ctx *c, int64_t *vals, int count, int op)
{
    if (!c || !vals || count < 0 || count > 8 || op < 0 || op > 2)
        return fail(PASTAR_EINVAL, "invalid allreduce arguments");
    if (!c->tr)
        return PASTAR_OK;
    HIP_TRY(hipSetDevice(c->device));
    return c->tr->allreduce(c, vals, count, (RedOp)op);
}

int pastar_gpu_synchronize(pastar_ctx *c)
{
    if (!c)
        return fail(PASTAR_EINVAL, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    return PASTAR_OK;
}

}  // extern "C"

// ===========================================================================
// OpenList / ClosedList (lists.hpp): host-driven operations on the device
// node table and f-bucket queues.
// ===========================================================================
namespace {

int lists_check(pastar_ctx *c)
{
    if (!c)
        return fail(PASTAR_EINVAL, "null ctx");
    if (!c->lists_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_lists_reset not called (or a search ran since)");
    HIP_TRY(hipSetDevice(c->device));
    return PASTAR_OK;
}

// device scratch (lists_io) and its pinned mirror (h_lists), grown on demand
int lists_io(pastar_ctx *c, size_t bytes)
{
    if (c->lists_io.n < bytes)
        PA_TRY(c->lists_io.alloc(std::max<size_t>(bytes, 4096)));
    if (c->h_lists_n < bytes) {
        if (c->h_lists)
            (void)hipHostFree(c->h_lists);
        c->h_lists = nullptr;
        c->h_lists_n = 0;
        const size_t n = std::max<size_t>(bytes, 4096);
        HIP_TRY(hipHostMalloc((void **)&c->h_lists, n, hipHostMallocDefault));
        c->h_lists_n = n;
    }
    return PASTAR_OK;
}

int check_coord(const pastar_ctx *c, const uint16_t *pos)
{
    for (int i = 0; i < c->n; i++)
        if (pos[i] > c->hp.len[i])
            return fail(PASTAR_EINVAL, "coordinate outside the lattice");
    return PASTAR_OK;
}

}  // namespace

extern "C" {

int pastar_gpu_lists_reset(pastar_ctx *c, const pastar_search_opts *opts)
{
    if (!c)
        return fail(PASTAR_EINVAL, "null ctx");
    if (!c->heuristic_ready)
        return fail(PASTAR_ESTATE, "pastar_gpu_build_heuristic not called");
    if (c->tr)
        return fail(PASTAR_EINVAL, "the host-driven lists are single-shard");
    HIP_TRY(hipSetDevice(c->device));
    pastar_search_opts o{};
    if (opts)
        o = *opts;
    c->lists_ready = false;
    c->searched = false;
    c->walk_ready = false;
    c->solo_active = false;
    PA_TRY(ensure_hc(c));
    PA_TRY(ensure_origin(c));
    SearchCfg cfg{};
    cfg.partial_k = -1;
    cfg.kmax = cfg.kmin = 1;
    cfg.table_log2 = o.table_slots_log2 > 0 ? (int)o.table_slots_log2 : 20;
    if (cfg.table_log2 < 10 || cfg.table_log2 > 32)
        return fail(PASTAR_EINVAL, "table_slots_log2 %d outside [10, 32]", cfg.table_log2);
    cfg.pool_entries = o.pool_entries > 0 ? (unsigned long long)o.pool_entries : (1ull << 22);
    cfg.subqueue_entries = o.subqueue_entries > 0 ? (unsigned long long)o.subqueue_entries : (1ull << 18);
    cfg.outbox_cap = 1;
    cfg.xblock_recs = 1;
    cfg.xlag = 0;
    PA_TRY(alloc_search(c, cfg));
    int w = c->auto_band_log2;
    if (o.band > 0)
        PA_TRY(estimate_band_log2(c, c->h0, o.band, &w));
    Ctl hc{};
    hc.band_log2 = w;
    hc.f0 = c->h0;
    hc.n_shards = 1;
    hc.kmax = hc.kmin = 1;
    hc.pool_chunks = c->pool.n / kChunk;  // the allocation (>= the request): stable across searches
    hc.maxch = maxch_of(cfg);
    hc.table_slots = c->nslots;
    hc.cur_b = kBuckets;  // empty: appends lower it
    hc.low_b = kBuckets;
    hc.spin_limit = c->spin_limit;
    std::memcpy(c->h_stage, &hc, sizeof(Ctl));
    PA_TRY(init_search(c, cfg, sizeof(Ctl)));
    HIP_TRY(hipStreamSynchronize(c->stream));
    SearchArgs &a = c->lists_args;
    a = SearchArgs{};
    a.P = c->dP.p;
    a.ctl = c->ctl.p;
    a.stamps = c->stamps.p;
    a.table = c->table.p;
    a.cap_mask = c->nslots - 1;
    a.q = c->queues.p;
    a.chunk_tab = c->chunk_tab.p;
    a.pool = c->pool.p;
    a.stats = c->stats.p;
    a.goal_g = c->goal.p;
    a.lower = &c->ctl.p->cur_b;
    a.maxch = maxch_of(cfg);
    a.pool_chunks = c->pool.n / kChunk;
    c->lists_reopen = 0;
    c->lists_ready = true;
    return PASTAR_OK;
}

int pastar_gpu_open_enqueue(pastar_ctx *c, const pastar_node *nodes, int count, int32_t *added, int64_t *reopened)
{
    PA_TRY(lists_check(c));
    if (count < 0 || (!nodes && count))
        return fail(PASTAR_EINVAL, "invalid arguments");
    if (reopened)
        *reopened = 0;
    if (count == 0)
        return PASTAR_OK;
    for (int k = 0; k < count; k++) {
        PA_TRY(check_coord(c, nodes[k].pos));
        if (nodes[k].g < 0 || nodes[k].f < nodes[k].g)
            return fail(PASTAR_EINVAL, "node %d: g %d, f %d", k, nodes[k].g, nodes[k].f);
    }
    const size_t nb = sizeof(pastar_node) * (size_t)count, fb = 4 * (size_t)count;
    const size_t off_flags = (nb + 15) & ~(size_t)15, off_res = (off_flags + fb + 15) & ~(size_t)15;
    PA_TRY(lists_io(c, off_res + 64));
    uint8_t *d = c->lists_io.p;
    std::memcpy(c->h_lists, nodes, nb);
    HIP_TRY(hipMemcpyAsync(d, c->h_lists, nb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(d + off_res, 0, 16, c->stream));
    HIP_TRY(hipMemsetAsync(&c->stats.p->ovf_near, 0, 16, c->stream));
    const dim3 grid((unsigned)((count + kListThreads - 1) / kListThreads));
    const pastar_node *din = reinterpret_cast<const pastar_node *>(d);
    int32_t *dflags = reinterpret_cast<int32_t *>(d + off_flags);
    unsigned long long *dres = reinterpret_cast<unsigned long long *>(d + off_res);
    if (c->kw == 1)
        hipLaunchKernelGGL(lists_enqueue_kernel<1>, grid, dim3(kListThreads), 0, c->stream, c->lists_args, din, count,
                           dflags, dres);
    else if (c->kw == 2)
        hipLaunchKernelGGL(lists_enqueue_kernel<2>, grid, dim3(kListThreads), 0, c->stream, c->lists_args, din, count,
                           dflags, dres);
    else
        hipLaunchKernelGGL(lists_enqueue_kernel<4>, grid, dim3(kListThreads), 0, c->stream, c->lists_args, din, count,
                           dflags, dres);
    PA_TRY(check_launch());
    HIP_TRY(hipMemcpyAsync(c->h_lists + off_flags, dflags, fb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_lists + off_res, dres, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_lists + off_res + 16, &c->stats.p->ovf_near, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_lists + off_res + 32, &c->ctl.p->fault, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const unsigned long long *r = reinterpret_cast<const unsigned long long *>(c->h_lists + off_res);
    if (const int sites = *reinterpret_cast<const int *>(c->h_lists + off_res + 32)) {
        c->lists_ready = false;
        return report_fault(c, sites);
    }
    if (r[1] || r[2] || r[3]) {
        c->lists_ready = false;  // a node was dropped: the lists are no longer exact
        return fail(PASTAR_ENOMEM, "OpenList capacity exhausted (table %llu, pool %llu, sub-queue %llu drops); "
                    "reset with larger capacities", r[1], r[2], r[3]);
    }
    if (added)
        std::memcpy(added, c->h_lists + off_flags, fb);
    c->lists_reopen += (long long)r[0];
    if (reopened)
        *reopened = (int64_t)r[0];
    return PASTAR_OK;
}

static int lists_pop(pastar_ctx *c, pastar_node *out, int max, int peek, int res[3])
{
    PA_TRY(lists_io(c, 64 + sizeof(pastar_node) * (size_t)std::max(max, 1)));
    uint8_t *d = c->lists_io.p;
    int *dres = reinterpret_cast<int *>(d);
    pastar_node *dout = reinterpret_cast<pastar_node *>(d + 64);
    if (c->kw == 1)
        hipLaunchKernelGGL(lists_dequeue_kernel<1>, dim3(1), dim3(kListThreads), 0, c->stream, c->lists_args, dout, max,
                           peek, dres);
    else if (c->kw == 2)
        hipLaunchKernelGGL(lists_dequeue_kernel<2>, dim3(1), dim3(kListThreads), 0, c->stream, c->lists_args, dout, max,
                           peek, dres);
    else
        hipLaunchKernelGGL(lists_dequeue_kernel<4>, dim3(1), dim3(kListThreads), 0, c->stream, c->lists_args, dout, max,
                           peek, dres);
    PA_TRY(check_launch());
    const size_t ob = peek ? 0 : sizeof(pastar_node) * (size_t)max;
    HIP_TRY(hipMemcpyAsync(c->h_lists, d, 64 + ob, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::memcpy(res, c->h_lists, 12);
    if (!peek && res[0] > 0)
        std::memcpy(out, c->h_lists + 64, sizeof(pastar_node) * (size_t)res[0]);
    return PASTAR_OK;
}

int pastar_gpu_open_dequeue(pastar_ctx *c, pastar_node *out, int max, int *count)
{
    PA_TRY(lists_check(c));
    if (!out || !count || max < 1)
        return fail(PASTAR_EINVAL, "invalid arguments");
    int res[3];
    PA_TRY(lists_pop(c, out, max, 0, res));
    *count = res[0];
    c->lists_reopen += res[2];
    return PASTAR_OK;
}

int pastar_gpu_open_highest_priority(pastar_ctx *c, int32_t *f)
{
    PA_TRY(lists_check(c));
    if (!f)
        return fail(PASTAR_EINVAL, "null argument");
    int res[3];
    PA_TRY(lists_pop(c, nullptr, 1, 1, res));
    *f = res[1];
    return PASTAR_OK;
}

int pastar_gpu_lists_size(pastar_ctx *c, int64_t *open, int64_t *closed)
{
    PA_TRY(lists_check(c));
    PA_TRY(lists_io(c, 64));
    unsigned long long *d = reinterpret_cast<unsigned long long *>(c->lists_io.p);
    HIP_TRY(hipMemsetAsync(d, 0, 16, c->stream));
    const unsigned blocks = (unsigned)std::min<uint64_t>(1024, (c->nslots + kListThreads - 1) / kListThreads);
    if (c->kw == 1)
        hipLaunchKernelGGL(lists_census_kernel<1>, dim3(blocks), dim3(kListThreads), 0, c->stream, c->table.p, c->nslots, d);
    else if (c->kw == 2)
        hipLaunchKernelGGL(lists_census_kernel<2>, dim3(blocks), dim3(kListThreads), 0, c->stream, c->table.p, c->nslots, d);
    else
        hipLaunchKernelGGL(lists_census_kernel<4>, dim3(blocks), dim3(kListThreads), 0, c->stream, c->table.p, c->nslots, d);
    PA_TRY(check_launch());
    HIP_TRY(hipMemcpyAsync(c->h_lists, d, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const unsigned long long *h = reinterpret_cast<const unsigned long long *>(c->h_lists);
    if (open)
        *open = (int64_t)h[0];
    if (closed)
        *closed = (int64_t)h[1];
    return PASTAR_OK;
}

static int lists_find_erase(pastar_ctx *c, const uint16_t *pos, int erase_which, unsigned long long r[3])
{
    PA_TRY(lists_io(c, 128));
    uint8_t *d = c->lists_io.p;
    std::memset(c->h_lists + 64, 0, 2 * PASTAR_MAX_SEQ);
    std::memcpy(c->h_lists + 64, pos, sizeof(uint16_t) * (size_t)c->n);  // the caller's pos holds n coordinates
    HIP_TRY(hipMemcpyAsync(d + 64, c->h_lists + 64, 2 * PASTAR_MAX_SEQ, hipMemcpyHostToDevice, c->stream));
    const uint16_t *dpos = reinterpret_cast<const uint16_t *>(d + 64);
    unsigned long long *dres = reinterpret_cast<unsigned long long *>(d);
    if (c->kw == 1)
        hipLaunchKernelGGL(lists_find_kernel<1>, dim3(1), dim3(1), 0, c->stream, c->lists_args, dpos, erase_which, dres);
    else if (c->kw == 2)
        hipLaunchKernelGGL(lists_find_kernel<2>, dim3(1), dim3(1), 0, c->stream, c->lists_args, dpos, erase_which, dres);
    else
        hipLaunchKernelGGL(lists_find_kernel<4>, dim3(1), dim3(1), 0, c->stream, c->lists_args, dpos, erase_which, dres);
    PA_TRY(check_launch());
    HIP_TRY(hipMemcpyAsync(c->h_lists, d, 24, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::memcpy(r, c->h_lists, 24);
    return PASTAR_OK;
}

int pastar_gpu_lists_find(pastar_ctx *c, const uint16_t *pos, pastar_node *out, int *where)
{
    PA_TRY(lists_check(c));
    if (!pos || !where)
        return fail(PASTAR_EINVAL, "null argument");
    PA_TRY(check_coord(c, pos));
    unsigned long long r[3];
    PA_TRY(lists_find_erase(c, pos, 0, r));
    *where = (int)r[0];
    if (out && r[0]) {
        std::memset(out, 0, sizeof(*out));
        std::memcpy(out->pos, pos, sizeof(uint16_t) * c->n);
        out->g = (int32_t)(r[1] >> 32);
        out->parent_mask = (int32_t)(uint32_t)r[1];
        out->f = out->g + (int32_t)(r[2] >> 32);
    }
    return PASTAR_OK;
}

int pastar_gpu_lists_erase(pastar_ctx *c, const uint16_t *pos, int which, int *erased)
{
    PA_TRY(lists_check(c));
    if (!pos || (which != 1 && which != 2))
        return fail(PASTAR_EINVAL, "invalid arguments (which: 1 OpenList, 2 ClosedList)");
    PA_TRY(check_coord(c, pos));
    unsigned long long r[3];
    PA_TRY(lists_find_erase(c, pos, which, r));
    if (erased)
        *erased = (int)r[0] == which ? 1 : 0;
    return PASTAR_OK;
}

int pastar_gpu_lists_reopened(pastar_ctx *c, int64_t *reopened)
{
    PA_TRY(lists_check(c));
    if (!reopened)
        return fail(PASTAR_EINVAL, "null argument");
    *reopened = c->lists_reopen;
    return PASTAR_OK;
}

}  // extern "C"

// ===========================================================================
// Device self-tests of the open list (selftest.hpp)
// ===========================================================================
extern "C" {

int pastar_gpu_selftest_queue(pastar_ctx *c, int scenario, int64_t *info)
{
    if (!c || !info || scenario < 0 || scenario > 1)
        return fail(PASTAR_EINVAL, "invalid arguments (scenario 0 or 1)");
    info[0] = info[1] = 0;
    // fresh, empty lists on the search's own buffers
    PA_TRY(pastar_gpu_lists_reset(c, nullptr));
    c->lists_ready = false;  // the queues below are no list session's
    SearchArgs a = c->lists_args;
    const int b1 = 3, b2 = 5;
    PA_TRY(lists_io(c, 64));
    unsigned *flags = reinterpret_cast<unsigned *>(c->lists_io.p);
    unsigned long long *out = reinterpret_cast<unsigned long long *>(c->lists_io.p + 16);
    HIP_TRY(hipMemsetAsync(c->lists_io.p, 0, 64, c->stream));
    if (scenario == 0) {
        // the handshake between the two workgroups: they are co-resident on
        // an idle device, so it takes microseconds; bounded at ~1 s
        hipLaunchKernelGGL(selftest_crossed_kernel, dim3(2), dim3(64), 0, c->stream, a, b1, b2, flags, 1u << 22);
        PA_TRY(check_launch());
        hipLaunchKernelGGL(selftest_crossed_check_kernel, dim3(1), dim3(64), 0, c->stream, a, b1, b2, out);
        PA_TRY(check_launch());
        HIP_TRY(hipMemcpyAsync(c->h_lists, out, 16, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        PA_TRY(check_fault(c));
        const unsigned long long *r = reinterpret_cast<const unsigned long long *>(c->h_lists);
        info[0] = (int64_t)r[0];
        info[1] = (int64_t)r[1];
        if (r[0])
            return fail(PASTAR_ESTATE, "crossed reservations left %llu wrong entries of %llu", r[0], r[1]);
        return PASTAR_OK;
    }
    // scenario 1: a cursor moved into a chunk nobody opened, and a store wait
    // bounded at 64 polls: the stores must give up, flag the site, and the
    // call must report PASTAR_EDEVWAIT
    const unsigned long long lost = 8;
    HIP_TRY(hipMemcpyAsync(&c->queues.p->W.d[0][b1], &lost, sizeof(lost), hipMemcpyHostToDevice, c->stream));
    const unsigned few = 64;
    HIP_TRY(hipMemcpyAsync(&c->ctl.p->spin_limit, &few, sizeof(few), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(selftest_lost_opener_kernel, dim3(1), dim3(64), 0, c->stream, a, b1);
    PA_TRY(check_launch());
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->queues_clean_known = false;  // a cursor without its chunk: clear everything next time
    return check_fault(c);
}

}  // extern "C"

// ===========================================================================
// Many independent LDS-resident searches in one launch
// ===========================================================================
extern "C" {

int pastar_gpu_search_many(pastar_ctx *const *ctxs, int count, const pastar_search_opts *opts, pastar_result *results)
{
    if (!ctxs || !results || count < 1 || count > 65535)
        return fail(PASTAR_EINVAL, "invalid arguments (1..65535 contexts)");
    pastar_search_opts o{};
    if (opts)
        o = *opts;
    SearchCfg cfg{};
    cfg.partial_k = -1;
    cfg.verbose = o.verbose;
    cfg.band = o.band;
    cfg.max_steps = o.max_steps;
    pastar_ctx *c0 = ctxs[0];
    if (!c0)
        return fail(PASTAR_EINVAL, "null context");
    HIP_TRY(hipSetDevice(c0->device));
    std::vector<SoloArgs> args((size_t)count);
    size_t lds = 0;
    const uint64_t stamp = ++g_many_stamp;  // marks the contexts of this call (a context given twice is refused)
    for (int k = 0; k < count; k++) {
        pastar_ctx *c = ctxs[k];
        if (!c)
            return fail(PASTAR_EINVAL, "null context %d", k);
        if (c->many_stamp == stamp)
            return fail(PASTAR_EINVAL, "context %d given twice (each search needs its own result areas)", k);
        c->many_stamp = stamp;
        if (c->device != c0->device || c->n != c0->n)
            return fail(PASTAR_EINVAL, "context %d: every search of one launch runs on one device with one "
                        "number of sequences (device %d, N = %d)", k, c0->device, c0->n);
        if (!c->heuristic_ready)
            return fail(PASTAR_ESTATE, "context %d: pastar_gpu_build_heuristic not called", k);
        c->walk_ready = false;
        c->searched = false;
        c->score = -1;
        c->lists_ready = false;
        // a context's launch record is prepared once and reused while its
        // options stay the same: only the ticket changes
        if (!c->many_cached || c->many_band != cfg.band || c->many_max_steps != cfg.max_steps) {
            SoloPlan pl;
            if (!solo_plan(c, &pl))
                return fail(PASTAR_EINVAL, "context %d: the problem does not fit the LDS-resident search", k);
            PA_TRY(solo_prepare(c, cfg, pl, &c->many_a, &c->many_done));
            c->many_lds = pl.lds;
            c->many_band = cfg.band;
            c->many_max_steps = cfg.max_steps;
            c->many_cached = true;
        } else {
            c->many_a.ticket = ++c->solo_ticket;
            *c->many_done = 0;
        }
        args[(size_t)k] = c->many_a;
        lds = std::max(lds, c->many_lds);
    }
    // the argument records, through the first context's staging buffer
    const size_t bytes = sizeof(SoloArgs) * (size_t)count;
    if (c0->many_args.n < bytes)
        PA_TRY(c0->many_args.alloc(bytes));
    HIP_TRY(hipMemcpyAsync(c0->many_args.p, args.data(), bytes, hipMemcpyHostToDevice, c0->stream));
    const void *fn = solo_many_fn_for(c0->n);
    if (!(c0->solo_many_attr_done & (1u << c0->n))) {
        HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kSoloLds));
        c0->solo_many_attr_done |= 1u << c0->n;
    }
    const SoloArgs *dargs = reinterpret_cast<const SoloArgs *>(c0->many_args.p);
    void *kargs[] = {(void *)&dargs};
    const double t0 = now_s();
    HIP_TRY(hipLaunchKernel(fn, dim3((unsigned)count), dim3(kSoloThreads), kargs, lds, c0->stream));
    PA_TRY(check_launch());
    // every search reports its own end; the launch's end covers them all
    HIP_TRY(hipStreamSynchronize(c0->stream));
    const double seconds = now_s() - t0;
    int rc = PASTAR_OK;
    for (int k = 0; k < count; k++) {
        if (*ctxs[k]->many_done != args[(size_t)k].ticket) {
            rc = fail(PASTAR_ENODEV, "search %d ended without its result", k);
            continue;
        }
        const int r = solo_finish(ctxs[k], cfg, args[(size_t)k].cap_log2, seconds, &results[k]);
        if (r != PASTAR_OK) {
            std::memset(&results[k], 0, sizeof(results[k]));
            results[k].score = -1;
            rc = r;
        }
    }
    return rc;
}

}  // extern "C"
