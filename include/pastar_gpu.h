/*
 * pastar_gpu.h -- C-ABI of the MI355X PAStar frontier-expansion engine.
 *
 * This is the drop-in boundary for the reference's hot path
 * (Gabrielcarvfer/mpi_pastar_msa; paths relative to its root):
 *
 *   reference interface                           replaced by
 *   --------------------------------------------  -----------------------------
 *   read_fasta_file (read_fasta.cpp:43-56)         pastar_read_fasta
 *   weightAltschulsRationale2 (WeightedSP.cpp:424) pastar_compute_weights
 *   HeuristicHPair::init (HeuristicHPair.cpp:47)   pastar_gpu_build_heuristic
 *   HeuristicHPair::calculate_h (:74-86)           pastar_gpu_h
 *   PairAlign::getScore (PairAlign.cpp:174-177)    pastar_gpu_pair_table
 *   Node<N>::getNeigh (Node.cpp:206-248, Node.h:37) pastar_gpu_expand
 *   Coord<N>::get_id (CoordHash.cpp:191-245)       pastar_owner
 *   PAStar<N>::pa_star (PAStar.cpp:627-673,        pastar_gpu_search
 *     PAStar.h:117) incl. worker_inner,
 *     OpenList / ClosedList (PriorityList.h:52-82,
 *     PAStar.cpp:92), check_stop (:480-547)
 *   ClosedList[id][coord] lookups in the backtrace pastar_gpu_closed_lookup,
 *     (backtrace.cpp:47-69, PAStarDistributed-      pastar_gpu_alignment
 *      Backtrace.cpp:19-213)
 *   MPI rank bootstrap (msa_pastar_main.cpp:56-89) pastar_rccl_unique_id +
 *                                                  pastar_gpu_create(n_shards,
 *                                                  shard_rank, rccl_id)
 *
 * Conventions: plain C types only; every entry point returns an int status
 * (0 ok, < 0 error) and never throws; pastar_last_error() describes the last
 * failure of the calling thread.  The caller owns host buffers, the context
 * owns device memory.  One context per GPU, driven by one host thread.
 * A process that has no usable gfx950 device gets PASTAR_ENODEV from
 * pastar_gpu_create: there is no CPU fallback.
 */
#ifndef PASTAR_GPU_H
#define PASTAR_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PASTAR_MAX_SEQ 16
#define PASTAR_ABI_VERSION 4

/* status codes */
#define PASTAR_OK 0
#define PASTAR_EINVAL (-1)   /* bad argument                          */
#define PASTAR_ENODEV (-2)   /* no HIP device / kernel launch failure */
#define PASTAR_ENOMEM (-3)   /* device capacity exhausted             */
#define PASTAR_EIO (-4)      /* file could not be read                */
#define PASTAR_ENOTFOUND (-5)
#define PASTAR_ECOMM (-6)    /* RCCL failure                          */
#define PASTAR_ESTATE (-7)   /* call out of order                     */
#define PASTAR_EDEVWAIT (-8) /* a bounded wait ran out: a wave's wait on
                                another wave on the device, or the host's
                                wait for a launch to report its end; the
                                call's results are discarded             */

/* Coord hash types, same numbering as the reference's hashType enum
 * (Coord.h:29): HashFZorder, HashPZorder, HashFSum, HashPSum. */
#define PASTAR_HASH_FZORDER 0
#define PASTAR_HASH_PZORDER 1
#define PASTAR_HASH_FSUM 2
#define PASTAR_HASH_PSUM 3

/* A search problem.  Mirrors the reference's process-global singletons
 * Sequences (Sequences.h:15-39), Cost (Cost.h:10-50) and
 * HeuristicHPair::weightMatrix (HeuristicHPair.h:23). */
typedef struct pastar_problem {
    int n;                          /* sequences, 2..16                       */
    const int *lengths;             /* n residue counts (>= 1 each)           */
    const char *const *residues;    /* n residue strings (lengths[i] chars)   */
    const int *weights;             /* P = n(n-1)/2 pair weights, pair order
                                       (0,1),(0,2)..(n-2,n-1) = (int)weight-
                                       Matrix[x][y]; NULL: computed on the
                                       host with pastar_compute_weights       */
    const int *sub;                 /* 128*128 distance table indexed by the
                                       residue bytes, or NULL for the
                                       reference table (Cost.cpp:12-262)      */
    int gap_open, gap_ext, gap_gap; /* Cost.h:13; all 30 in the reference     */
    int hash_type, hash_shift;      /* CoordHash owner partition (FZORDER, 12)*/
} pastar_problem;

/* Node<N> (Node.h:28-49): coordinate, g, f and the parent mask `parenti`. */
typedef struct pastar_node {
    uint16_t pos[PASTAR_MAX_SEQ];
    int32_t g;
    int32_t f;
    int32_t parent_mask;
} pastar_node;

/* Tuning of the device-resident search (all zero = defaults). */
typedef struct pastar_search_opts {
    int64_t batch_nodes;      /* most open nodes expanded per step          */
    int64_t batch_min;        /* a step with fewer nodes in its band also
                                 takes the next bands (up to 4); 0 = 1/8 of
                                 batch_nodes                               */
    int64_t table_slots_log2; /* open+closed hash table capacity (log2); 0 =
                                 2^24 on a context's first search, then what
                                 the last search needed at <= 25% load; an
                                 explicit value is a floor under the latter */
    int64_t pool_entries;     /* open-list entry pool (all f buckets)       */
    int64_t subqueue_entries; /* entries one bucket sub-queue can hold      */
    int64_t max_steps;        /* safety stop (0 = unlimited)                */
    int64_t band;             /* a step expands open nodes with f below the
                                 current minimum + band (0 = auto: half the
                                 mean f increase of one expansion)         */
    int32_t profile;          /* 1: the expand kernel times each launch on
                                 the 100 MHz device clock (s_memrealtime,
                                 first block start -> last block end)      */
    int32_t verbose;
    int32_t no_autogrow;      /* 1: fail with PASTAR_ENOMEM instead of
                                 growing an exhausted capacity x4 and
                                 restarting the search                     */
    int32_t eager;            /* 1: launch every step from the host instead
                                 of replaying a captured hipGraph          */
    int32_t depth;            /* expansion levels per step: children whose f
                                 falls in the step's buckets are expanded by
                                 the same workgroup in the same launch, up to
                                 depth - 1 more levels (0 = default, at most
                                 1024)                                     */
    int32_t mode;             /* PASTAR_MODE_*: which engine runs the search */
    /* sharded search (n_shards > 1): the record exchange between shards    */
    int32_t xchg_lag;         /* 0: a step's select sees the records the
                                 shards sent in the step before (the exchange
                                 sits between two steps); 1: the exchange and
                                 the owner's insert of step i run beside the
                                 expansion of step i + 1 (side stream), and
                                 their records reach the select after        */
    int32_t partial;          /* partial expansion (PEA*: a parent's children
                                 whose f lies at or past a window beyond the
                                 step's buckets are generated only when the
                                 parent comes up again, queued under the
                                 lowest f among them; results are the same,
                                 most of a wide fan-out is never probed):
                                 0 = default (on for N >= 7, window of one
                                 bucket), n > 0: window of n - 1 buckets,
                                 -1: off; ignored for N <= 6               */
    int64_t xchg_block_records; /* most records one step carries to one shard
                                 (the all-to-all's block, a power of two of
                                 records sized per round from the demand seen,
                                 from 4096 up to this; more wait in the
                                 sender's ring); 0 = 2^20                    */
} pastar_search_opts;

/* pastar_search_opts.mode */
#define PASTAR_MODE_AUTO 0    /* the LDS-resident search when the problem fits
                                 one workgroup's LDS (pair tables plus a node
                                 table of >= 256 slots; equal gap costs,
                                 one shard), else (or once it overflows) the
                                 batched engine                             */
#define PASTAR_MODE_BATCHED 1 /* the batched multi-workgroup engine only    */
#define PASTAR_MODE_SOLO 2    /* the LDS-resident search only (PASTAR_EINVAL
                                 if the problem does not fit, PASTAR_ENOMEM
                                 if the search outgrows the node table)    */

typedef struct pastar_result {
    int64_t score;          /* optimal weighted SP score (goal g)              */
    int64_t expansions;     /* nodes expanded by this shard, incl. the goal   */
    int64_t expansions_all; /* summed over shards                             */
    int64_t reopen;         /* re-expansions with a better g (PAStar Reopen)  */
    int64_t generated;      /* neighbours produced                            */
    int64_t open_size;      /* live open entries at termination               */
    int64_t closed_size;    /* distinct expanded nodes                        */
    int64_t table_used;     /* distinct nodes stored                          */
    int64_t steps;          /* batched expansion steps                        */
    int64_t exchanged;      /* nodes sent to other shards                     */
    double seconds;         /* first expansion -> goal accepted (wall)        */
    double expand_ms;       /* sum of expand-kernel durations (profile = 1)   */
    int64_t expand_launches; /* launches with a batch (profile = 1) / steps   */
    int64_t expand_parents; /* parents handed to the expand kernel            */
    int64_t capacity_retries; /* restarts after growing an exhausted capacity */
    int64_t table_slots;    /* node table capacity used                       */
    int64_t pool_entries, subqueue_entries;
    int64_t graph_replay;   /* 1 when the steps ran as hipGraph replays       */
    double select_ms;       /* profile = 1, one shard: part of expand_ms spent
                               in the fused select tail                    */
    double gap_ms;          /* profile = 1, one shard: device idle between
                               the end of one step and the start of the next
                               (launch gaps)                               */
    int64_t solo;           /* 1 when the search ran on the LDS-resident path
                               (one launch: PairAlign, search, backtrace;
                               steps = levels, expand_ms = that launch)    */
    /* sharded search */
    int64_t xchg_backlog_steps; /* (step, destination) pairs whose records did
                               not all fit the step's exchange block        */
    int64_t xchg_backlog_max;   /* most records left waiting for one shard   */
    int64_t host_waits;         /* times the host waited for the device during
                               the step loop (one per round of steps)       */
} pastar_result;

typedef struct pastar_ctx pastar_ctx;

const char *pastar_last_error(void);
int pastar_abi_version(void);

/* ---- host-side helpers (reference file formats and precompute) ---- */

/* read_fasta_file (read_fasta.cpp:8-56): a line that is empty or starts with
 * '>' ends the current sequence; '\r' is kept.  Writes up to *n (in: capacity)
 * sequences back to back into buf (cap bytes, no separators) and their
 * lengths into lengths[]. */
int pastar_read_fasta(const char *path, char *buf, int64_t cap, int *n, int *lengths);

/* weightAltschulsRationale2 (WeightedSP.cpp:424-519): float n*n matrix. */
int pastar_compute_weights(int n, const char *const *residues, const int *lengths, float *out);

/* Cost::cost (Cost.cpp:266-270) of the reference table. */
int pastar_cost(int r, int l);

/* Coord<N>::get_id (CoordHash.cpp:191-245); -1 on an invalid shift. */
int pastar_owner(int n, const uint16_t *pos, int size, int hash_type, int shift);

/* ---- RCCL bootstrap (replaces MPI_Init + rank bookkeeping) ---- */
int pastar_rccl_unique_id(unsigned char out[128]);

/* ---- device context ---- */

/* device: HIP ordinal; n_shards >= 1; shard_rank in [0, n_shards);
 * rccl_id: 128 bytes from pastar_rccl_unique_id on rank 0 (NULL when
 * n_shards == 1). */
int pastar_gpu_create(const pastar_problem *p, int device, int n_shards, int shard_rank,
                      const void *rccl_id, pastar_ctx **out);
void pastar_gpu_destroy(pastar_ctx *ctx);

/* In-process shard group: n_shards contexts in one process, each driven by
 * its own host thread (pastar_gpu_search is collective over the group);
 * nodes move between shards by peer copies instead of RCCL.  The shards may
 * share one device (the sharded path on a single GPU) or use several. */
typedef struct pastar_group pastar_group;
int pastar_group_create(int n_shards, pastar_group **out);
void pastar_group_destroy(pastar_group *group); /* after its contexts */
int pastar_gpu_create_grouped(const pastar_problem *p, int device, pastar_group *group, int shard_rank,
                              pastar_ctx **out);

/* Element-wise reduction of count (<= 8) host int64 values over all shards
 * (op 0 sum, 1 min, 2 max); collective.  Doubles as a barrier. */
int pastar_gpu_allreduce(pastar_ctx *ctx, int64_t *vals, int count, int op);
/* Wait for all work on the context's device. */
int pastar_gpu_synchronize(pastar_ctx *ctx);

/* Phase 1: PairAlign tables by the anti-diagonal wavefront kernel. */
int pastar_gpu_build_heuristic(pastar_ctx *ctx);
int pastar_gpu_pair_table(pastar_ctx *ctx, int pair, int32_t *out);
int pastar_gpu_weights(pastar_ctx *ctx, int32_t *out);
int pastar_gpu_h(pastar_ctx *ctx, const uint16_t *pos, int count, int32_t *out);

/* Batched Node::getNeigh.  For each input node, every border-valid neighbour
 * in increasing mask order, compacted back to back (input order preserved).
 * out/out_owner/out_src need n_in * (2^n - 1) entries; out_owner receives
 * get_id(vec_size), out_src the input index. */
int pastar_gpu_expand(pastar_ctx *ctx, const pastar_node *in, int n_in, int vec_size,
                      pastar_node *out, int32_t *out_owner, int32_t *out_src, int64_t *n_out);

/* pastar_gpu_expand without any allocation.  No counterpart in the
 * reference: it is for callers that cannot allocate device memory (code
 * under HIP graph capture, tight serving loops, harnesses that forbid
 * hipMalloc).  Same arguments, results and errors as pastar_gpu_expand; the
 * staging buffers (input nodes, offsets, neighbours, owners, sources) are a
 * fixed scratch array in device memory (about 3.9 MB per GPU, held until the
 * process ends), so a call takes at most PASTAR_NOALLOC_MAX_IN nodes and
 * PASTAR_NOALLOC_MAX_OUT neighbours and fails with PASTAR_EINVAL beyond.
 * Calls no hipMalloc / hipFree.  All calls on one GPU share that GPU's
 * scratch: calls that overlap on one GPU (several contexts or threads) race. */
#define PASTAR_NOALLOC_MAX_IN 8192
#define PASTAR_NOALLOC_MAX_OUT 65536
int pastar_gpu_expand_noalloc(pastar_ctx *ctx, const pastar_node *in, int n_in, int vec_size,
                              pastar_node *out, int32_t *out_owner, int32_t *out_src, int64_t *n_out);

/* Device-resident PAStar search from the origin to the final coordinate. */
int pastar_gpu_search(pastar_ctx *ctx, const pastar_search_opts *opts, pastar_result *res);

/* Many independent searches in ONE launch (no counterpart in the reference,
 * which aligns one family per process: PAStar::pa_star over many inputs at
 * once).  Search k runs whole in one workgroup's LDS (the LDS-resident
 * engine, PASTAR_MODE_SOLO), so every problem must fit it (small families:
 * PF08184-sized) and all contexts must sit on one device and have the same
 * number of sequences; count <= 65535 distinct contexts.  results[k] is what
 * pastar_gpu_search(ctxs[k]) returns (its `seconds` is the whole launch's);
 * afterwards each context answers pastar_gpu_alignment /
 * pastar_gpu_closed_lookup for its own search.  A search that outgrows its
 * LDS node table gets score -1 in results[k] and the call returns
 * PASTAR_ENOMEM (the others are valid); opts: band, max_steps, verbose. */
int pastar_gpu_search_many(pastar_ctx *const *ctxs, int count, const pastar_search_opts *opts,
                           pastar_result *results);

/* ClosedList lookup after a search: the stored node for a coordinate owned by
 * this shard (PASTAR_ENOTFOUND if absent). */
int pastar_gpu_closed_lookup(pastar_ctx *ctx, const uint16_t *pos, pastar_node *out);

/* Backtrace (backtrace.cpp:47-69 / PAStarDistributedBacktrace.cpp:19-213):
 * the alignment rows, n rows of `stride` bytes each, NUL terminated; *cols
 * receives the alignment length.  Collective over all shards. */
int pastar_gpu_alignment(pastar_ctx *ctx, char *rows, int stride, int *cols);

/* ---- OpenList / ClosedList (PriorityList<N>, PriorityList.h:52-122; the
 * ClosedList map, PAStar.cpp:92; PAStar::enqueue, :219-237) ----
 *
 * The device search's own node table and f-bucket queues, driven one call at
 * a time from the host: a loop shaped like worker_inner (PAStar.cpp:320-401)
 * runs over these calls unchanged (include/pastar_lists.hpp wraps them as the
 * reference's classes).  One node record serves both lists, so a node is in
 * at most one of them; ties on g keep the smaller parent mask (the batched
 * engine's rule) where the reference keeps the first found.  Single shard.
 * A search (pastar_gpu_search) reuses the buffers and ends the session.
 * Deviation from PriorityList alone: pastar_gpu_open_enqueue always makes
 * PAStar::enqueue's ClosedList check (PAStar.cpp:226-232), so a node cannot
 * be put into the OpenList while a ClosedList record with g <= its g exists;
 * the reference's PriorityList::conditional_enqueue would accept it, and no
 * call site of the reference asks that (each checks or erases first). */

/* PAStar construction: empty lists (opts: table_slots_log2, pool_entries,
 * subqueue_entries, band; zeros = defaults). */
int pastar_gpu_lists_reset(pastar_ctx *ctx, const pastar_search_opts *opts);

/* PAStar::enqueue + PriorityList::conditional_enqueue for each node: a node
 * whose record (open or closed) has g <= node.g is discarded; else it
 * (re)enters the OpenList with f = node.f.  added[i] (may be NULL) = 1 when
 * node i entered; *reopened counts ClosedList nodes improved (nodes_reopen).
 * PASTAR_ENOMEM (and the session ends) if a capacity ran out. */
int pastar_gpu_open_enqueue(pastar_ctx *ctx, const pastar_node *nodes, int count, int32_t *added,
                            int64_t *reopened);

/* PriorityList::dequeue followed by the worker's ClosedList insert
 * (worker_inner :336-351): up to max nodes, all with the lowest f of the
 * OpenList (which of several ties is unspecified), move to the ClosedList
 * and are written to out; *count = 0 when the OpenList is empty. */
int pastar_gpu_open_dequeue(pastar_ctx *ctx, pastar_node *out, int max, int *count);

/* PriorityList::get_highest_priority: the lowest f, INT32_MAX when empty. */
int pastar_gpu_open_highest_priority(pastar_ctx *ctx, int32_t *f);

/* PriorityList::size and the ClosedList map's size (nodes). */
int pastar_gpu_lists_size(pastar_ctx *ctx, int64_t *open, int64_t *closed);

/* OpenList.find / ClosedList.find: *where = 1 open, 2 closed, 0 absent; out
 * (may be NULL) receives the node. */
int pastar_gpu_lists_find(pastar_ctx *ctx, const uint16_t *pos, pastar_node *out, int *where);

/* OpenList.erase (which = 1) / ClosedList.erase (which = 2): the node leaves
 * the lists if it is in that one; *erased (may be NULL) = 1 if it was. */
int pastar_gpu_lists_erase(pastar_ctx *ctx, const uint16_t *pos, int which, int *erased);

/* Reopenings since pastar_gpu_lists_reset (nodes_reopen, PAStar.cpp:232). */
int pastar_gpu_lists_reopened(pastar_ctx *ctx, int64_t *reopened);

/* ---- device self-tests (no counterpart in the reference) ----
 * The open list hands chunk ids from the lane that reserves a range to the
 * lanes that store into it (the device-side form of PAStar::enqueue's
 * inserts, PAStar.cpp:219-237, run by many workgroups at once).
 * scenario 0: two workgroups reserve ranges of two f buckets in crossed
 *   order and store first into the bucket where they came second; must end
 *   with every entry in place (info[0] = wrong entries, info[1] = checked).
 * scenario 1: a store into a chunk nobody opened, its wait bounded at 64
 *   polls from the host: the kernel ends normally and the call returns
 *   PASTAR_EDEVWAIT naming the site.
 * After pastar_gpu_build_heuristic; ends any list session. */
int pastar_gpu_selftest_queue(pastar_ctx *ctx, int scenario, int64_t *info);

/* ---- MPI-compatible wire frame -------------------------
 * The reference's inter-rank message frame, byte-identical to what its
 * pastar_lz4_en emits (lz4sup.cpp:13-43): u32 total, u32 LZ4 bound, u32
 * payload + 1, then the LZ4 block of the payload and a trailing NUL.  Host
 * code, no device needed; the record exchange of this engine stays on RCCL.
 *   pastar_lz4_en (lz4sup.cpp:13)   pastar_wire_frame_bound + _encode
 *   pastar_lz4_dec (lz4sup.cpp:45)  pastar_wire_frame_decode: writes the
 *                                   payload and its NUL (*out_len = len + 1)
 *   Node<N>::serialize (Node.h:57-64) field order, packed little-endian
 *   (12 + 2N bytes a node: g, f, pos[N], parenti)
 *                                   pastar_wire_pack_nodes / _unpack_nodes */
int pastar_wire_frame_bound(int64_t len, int64_t *bound);
int pastar_wire_frame_encode(const void *payload, int64_t len, void *out, int64_t cap, int64_t *out_len);
int pastar_wire_frame_decode(const void *frame, int64_t frame_len, void *out, int64_t cap, int64_t *out_len);
int pastar_wire_pack_nodes(const pastar_node *nodes, int count, int n, void *out, int64_t cap, int64_t *out_len);
int pastar_wire_unpack_nodes(const void *in, int64_t len, int n, pastar_node *out, int cap, int *count);

#ifdef __cplusplus
}
#endif
#endif
