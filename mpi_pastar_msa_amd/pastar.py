"""Python mirror of the reference's PAStar hot-path interface, over the C-ABI.

Reference names kept (Gabrielcarvfer/mpi_pastar_msa, paths relative to its
root):

  Sequences            pastar/include/Sequences.h:15-39  (object, not singleton)
  Node                 pastar/include/Node.h:23-66
  HeuristicHPair       pastar/include/HeuristicHPair.h:15-29 -> Engine.init(),
                       Engine.calculate_h(), Engine.weight_matrix
  Node.getNeigh        pastar/Node.cpp:206-248 -> Engine.get_neigh()
  Coord.get_id         pastar/CoordHash.cpp:191-245 -> get_id()
  PAStarOpt            pastar/include/PAStar.h:87-112
  PAStar.pa_star       pastar/PAStar.cpp:627-673 -> Engine.pa_star()

Errors follow the reference: an invalid hash shift or thread count raises
ValueError (std::invalid_argument there); a missing FASTA file raises
OSError ("Can't open file", read_fasta.cpp:17-20).
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as nat
from ._native import check, lib

MAX_SEQ = nat.MAX_SEQ
GAP_OPEN = GAP_EXTENSION = GAP_GAP = 30  # Cost.h:13


def cost(r, l):
    """Cost::cost (Cost.cpp:266-270)."""
    return lib().pastar_cost(ord(r) if isinstance(r, str) else r, ord(l) if isinstance(l, str) else l)


def get_id(coord, size, hash_type="FZORDER", hash_shift=12):
    """Coord<N>::get_id: owner of a coordinate among `size` workers/shards."""
    if not 0 <= hash_shift <= 21:
        raise ValueError("Invalid Hash Shift")
    ht = nat.HASH_TYPES[hash_type] if isinstance(hash_type, str) else int(hash_type)
    c = (ctypes.c_uint16 * MAX_SEQ)(*coord)
    return lib().pastar_owner(len(coord), c, int(size), ht, int(hash_shift))


class Sequences:
    """The sequences being aligned (Sequences.cpp:53-87)."""

    def __init__(self, seqs):
        self.seqs = [s if isinstance(s, str) else s.decode() for s in seqs]
        if not 2 <= len(self.seqs) <= MAX_SEQ:
            raise ValueError("Invalid number of sequences: %d" % len(self.seqs))

    @classmethod
    def from_fasta(cls, path):
        """read_fasta_file (read_fasta.cpp:8-56), quirks included."""
        n = ctypes.c_int(MAX_SEQ)
        lengths = (ctypes.c_int * MAX_SEQ)()
        cap = 1 << 22
        buf = ctypes.create_string_buffer(cap)
        rc = lib().pastar_read_fasta(str(path).encode(), buf, cap, ctypes.byref(n), lengths)
        if rc == nat.EIO:
            raise OSError("Can't open file %s" % path)
        check(rc)
        seqs, off = [], 0
        for i in range(n.value):
            seqs.append(buf.raw[off:off + lengths[i]].decode("latin-1"))
            off += lengths[i]
        return cls(seqs)

    def get_seq(self, i):
        return self.seqs[i]

    def get_seq_num(self):
        return len(self.seqs)

    def get_final_coord(self):
        return tuple(len(s) for s in self.seqs)

    def get_initial_coord(self):
        return tuple(0 for _ in self.seqs)

    def get_initial_node(self):
        """Origin with parenti = (1 << N) - 1 (Sequences.cpp:70-77); f is filled by the engine."""
        return Node(self.get_initial_coord(), 0, 0, (1 << len(self.seqs)) - 1)


@dataclass
class Node:
    pos: tuple
    g: int
    f: int
    parenti: int

    def get_g(self):
        return self.g

    def get_f(self):
        return self.f

    def get_h(self):
        return self.f - self.g

    def get_parenti(self):
        return self.parenti

    def get_parent(self):
        return tuple(c - ((self.parenti >> i) & 1) for i, c in enumerate(self.pos))

    def __str__(self):  # Node.cpp:41-47
        return "(%s)\tg - %d (h - %d f - %d)" % (" ".join(map(str, self.pos)), self.g, self.get_h(), self.f)


@dataclass
class PAStarOpt:
    """PAStarOpt (PAStar.h:87-112) plus the device-search knobs."""
    hash_type: str = "FZORDER"
    hash_shift: int = 12
    threads_num: int = 1
    batch_nodes: int = 0
    batch_min: int = 0
    table_slots_log2: int = 0
    pool_entries: int = 0
    subqueue_entries: int = 0
    max_steps: int = 0
    band: int = 0
    profile: bool = False
    verbose: bool = False
    autogrow: bool = True
    eager: bool = False
    depth: int = 0
    mode: str = "auto"  # "auto": LDS-resident search when the problem fits; "batched"; "solo"
    xchg_lag: int = 0   # sharded: 1 = the exchange of step i runs beside the expansion of step i + 1
    xchg_block_records: int = 0  # sharded: records one step carries to one shard (0 = default)
    partial: int = 0    # partial expansion for N >= 7: 0 = default (window of one bucket), n > 0: n - 1 buckets, -1: off

    def search_opts(self):
        return nat.pastar_search_opts(self.batch_nodes, self.batch_min, self.table_slots_log2, self.pool_entries,
                                      self.subqueue_entries, self.max_steps, self.band, int(self.profile),
                                      int(self.verbose),
                                      int(not self.autogrow), int(self.eager), int(self.depth),
                                      {"auto": 0, "batched": 1, "solo": 2}[self.mode],
                                      int(self.xchg_lag), int(self.partial), int(self.xchg_block_records))


def compute_weights(seqs):
    """weightAltschulsRationale2 on the host (float n x n matrix)."""
    n = len(seqs)
    arr = (ctypes.c_char_p * n)(*[s.encode("latin-1") for s in seqs])
    lens = (ctypes.c_int * n)(*[len(s) for s in seqs])
    out = (ctypes.c_float * (n * n))()
    check(lib().pastar_compute_weights(n, arr, lens, out))
    return np.array(out[:], dtype=np.float32).reshape(n, n)


def rccl_unique_id():
    buf = ctypes.create_string_buffer(128)
    check(lib().pastar_rccl_unique_id(buf))
    return buf.raw


@dataclass
class SearchResult:
    score: int
    expansions: int
    expansions_all: int
    reopen: int
    generated: int
    open_size: int
    closed_size: int
    table_used: int
    steps: int
    exchanged: int
    seconds: float
    expand_ms: float
    expand_launches: int
    expand_parents: int
    capacity_retries: int = 0
    table_slots: int = 0
    pool_entries: int = 0
    subqueue_entries: int = 0
    graph_replay: int = 0
    select_ms: float = 0.0
    gap_ms: float = 0.0
    solo: int = 0
    xchg_backlog_steps: int = 0
    xchg_backlog_max: int = 0
    host_waits: int = 0
    extra: dict = field(default_factory=dict)


class ShardGroup:
    """In-process shard group (pastar_group_create): several Engines driven by
    threads of one process exchange nodes by peer copies instead of RCCL."""

    def __init__(self, n_shards):
        self.n_shards = n_shards
        self._g = ctypes.c_void_p()
        check(lib().pastar_group_create(n_shards, ctypes.byref(self._g)))

    def close(self):
        if self._g:
            lib().pastar_group_destroy(self._g)
            self._g = ctypes.c_void_p()


class Engine:
    """One device context (one GPU shard).  Owns the device memory."""

    def __init__(self, sequences, device=0, n_shards=1, shard_rank=0, rccl_id=None, weights=None,
                 hash_type="FZORDER", hash_shift=12, gap_open=GAP_OPEN, gap_ext=GAP_EXTENSION,
                 gap_gap=GAP_GAP, group=None):
        if isinstance(sequences, (list, tuple)):
            sequences = Sequences(sequences)
        if not 0 <= hash_shift <= 21:
            raise ValueError("Invalid Hash Shift")
        self.sequences = sequences
        seqs = sequences.seqs
        self.n = len(seqs)
        self.n_shards = n_shards
        self.shard_rank = shard_rank
        self._keep = [s.encode("latin-1") for s in seqs]
        self._lens = (ctypes.c_int * self.n)(*[len(s) for s in seqs])
        self._res = (ctypes.c_char_p * self.n)(*self._keep)
        npairs = self.n * (self.n - 1) // 2
        self._w = (ctypes.c_int * npairs)(*weights) if weights is not None else None
        ht = nat.HASH_TYPES[hash_type] if isinstance(hash_type, str) else int(hash_type)
        self.hash_type, self.hash_shift = ht, hash_shift
        prob = nat.pastar_problem(self.n, self._lens, self._res,
                                  self._w if self._w is not None else None, None,
                                  gap_open, gap_ext, gap_gap, ht, hash_shift)
        self._ctx = ctypes.c_void_p()
        if group is not None:
            self.n_shards = group.n_shards
            check(lib().pastar_gpu_create_grouped(ctypes.byref(prob), device, group._g, shard_rank,
                                                  ctypes.byref(self._ctx)))
        else:
            check(lib().pastar_gpu_create(ctypes.byref(prob), device, n_shards, shard_rank, rccl_id,
                                          ctypes.byref(self._ctx)))
        self.npairs = npairs
        self.pairs = [(x, y) for x in range(self.n - 1) for y in range(x + 1, self.n)]
        self._ready = False
        self._result = nat.pastar_result()
        self._so, self._so_key = None, None
        self._rows_buf = None

    def close(self):
        if self._ctx:
            lib().pastar_gpu_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- collectives over the shards ----
    def allreduce(self, values, op="sum"):
        """Element-wise sum/min/max of up to 8 integers over all shards."""
        arr = (ctypes.c_int64 * len(values))(*[int(v) for v in values])
        check(lib().pastar_gpu_allreduce(self._ctx, arr, len(values), {"sum": 0, "min": 1, "max": 2}[op]))
        return list(arr)

    def barrier(self):
        self.allreduce([0])

    def synchronize(self):
        check(lib().pastar_gpu_synchronize(self._ctx))

    # ---- HeuristicHPair ----
    def init(self):
        """HeuristicHPair::init: PairAlign tables on the GPU (wavefront kernel)."""
        check(lib().pastar_gpu_build_heuristic(self._ctx))
        self._ready = True
        return self

    @property
    def weight_matrix(self):
        """(int)weightMatrix[x][y] for the pairs in row-major order."""
        out = (ctypes.c_int32 * self.npairs)()
        check(lib().pastar_gpu_weights(self._ctx, out))
        return list(out)

    def pair_table(self, k):
        """PairAlign k's full suffix table as an (L_x+1, L_y+1) int32 array."""
        x, y = self.pairs[k]
        lx, ly = len(self.sequences.seqs[x]), len(self.sequences.seqs[y])
        out = np.empty((lx + 1) * (ly + 1), dtype=np.int32)
        check(lib().pastar_gpu_pair_table(self._ctx, k, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out.reshape(lx + 1, ly + 1)

    def calculate_h(self, coords):
        """HeuristicHPair::calculate_h for one coordinate or an (m, n) array."""
        arr = np.asarray(coords, dtype=np.uint16)
        single = arr.ndim == 1
        arr = np.atleast_2d(arr)
        buf = np.zeros((arr.shape[0], MAX_SEQ), dtype=np.uint16)
        buf[:, :self.n] = arr
        out = np.empty(arr.shape[0], dtype=np.int32)
        check(lib().pastar_gpu_h(self._ctx, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), arr.shape[0],
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return int(out[0]) if single else out

    # ---- Node::getNeigh ----
    def get_neigh_batch(self, nodes, vec_size=1, noalloc=False):
        """Batched getNeigh: returns (children, owner, src) for a list of Node.
        noalloc: through pastar_gpu_expand_noalloc (fixed device scratch, no
        allocation; bounded input and output counts)."""
        n_in = len(nodes)
        arr = (nat.pastar_node * max(n_in, 1))()
        for k, nd in enumerate(nodes):
            for i, c in enumerate(nd.pos):
                arr[k].pos[i] = c
            arr[k].g, arr[k].f, arr[k].parent_mask = nd.g, nd.f, nd.parenti
        cap = max(n_in * ((1 << self.n) - 1), 1)
        out = (nat.pastar_node * cap)()
        own = (ctypes.c_int32 * cap)()
        src = (ctypes.c_int32 * cap)()
        cnt = ctypes.c_int64()
        fn = lib().pastar_gpu_expand_noalloc if noalloc else lib().pastar_gpu_expand
        check(fn(self._ctx, arr, n_in, vec_size, out, own, src, ctypes.byref(cnt)))
        kids = [Node(tuple(out[k].pos[:self.n]), out[k].g, out[k].f, out[k].parent_mask)
                for k in range(cnt.value)]
        return kids, list(own[:cnt.value]), list(src[:cnt.value])

    def get_neigh(self, node, vec_size=1):
        """Node::getNeigh(a, vec_size): neighbours bucketed by owner, mask order kept."""
        kids, owner, _ = self.get_neigh_batch([node], vec_size)
        a = [[] for _ in range(vec_size)]
        for k, o in zip(kids, owner):
            a[o].append(k)
        return a

    def initial_node(self):
        nd = self.sequences.get_initial_node()
        nd.f = self.calculate_h(nd.pos)
        return nd

    # ---- PAStar ----
    def pa_star(self, opt=None):
        """Run the device-resident search to the optimal alignment."""
        opt = opt or PAStarOpt()
        if opt.threads_num <= 0:
            raise ValueError("Invalid number of threads")
        if not self._ready:
            self.init()
        r = self._result
        # the options struct is rebuilt only when an option changed
        key = tuple(opt.__dict__.values())
        if key != self._so_key:
            self._so, self._so_key = opt.search_opts(), key
        check(lib().pastar_gpu_search(self._ctx, ctypes.byref(self._so), ctypes.byref(r)))
        return SearchResult(*r.as_tuple())

    def selftest_queue(self, scenario):
        """pastar_gpu_selftest_queue: (wrong entries, entries checked); raises
        NativeError(EDEVWAIT) when a bounded device wait ran out."""
        if not self._ready:
            self.init()
        info = (ctypes.c_int64 * 4)()
        check(lib().pastar_gpu_selftest_queue(self._ctx, int(scenario), info))
        return info[0], info[1]

    def closed_lookup(self, coord):
        c = (ctypes.c_uint16 * MAX_SEQ)(*coord)
        out = nat.pastar_node()
        rc = lib().pastar_gpu_closed_lookup(self._ctx, c, ctypes.byref(out))
        if rc == nat.ENOTFOUND:
            return None
        check(rc)
        return Node(tuple(out.pos[:self.n]), out.g, out.f, out.parent_mask)

    def alignment(self):
        """Backtrace rows (collective over shards)."""
        if self._rows_buf is None:  # one buffer per engine, reused
            stride = sum(len(s) for s in self.sequences.seqs) + 1
            self._rows_buf = (ctypes.create_string_buffer(self.n * stride), stride, ctypes.c_int())
        buf, stride, cols = self._rows_buf
        check(lib().pastar_gpu_alignment(self._ctx, buf, stride, ctypes.byref(cols)))
        raw, n = buf.raw, cols.value
        return [raw[i * stride:i * stride + n].decode("latin-1") for i in range(self.n)]


def search_many(engines, opt=None):
    """pastar_gpu_search_many: the searches of `engines` (one problem each,
    small enough for the LDS-resident engine, same device and number of
    sequences) in one launch.  Returns their SearchResults; each engine then
    answers alignment() for its own search."""
    opt = opt or PAStarOpt()
    for e in engines:
        if not e._ready:
            e.init()
    k = len(engines)
    arr = (ctypes.c_void_p * k)(*[e._ctx.value for e in engines])
    res = (nat.pastar_result * k)()
    so = opt.search_opts()
    check(lib().pastar_gpu_search_many(arr, k, ctypes.byref(so), res))
    return [SearchResult(*r.as_tuple()) for r in res]


def _c_nodes(nodes):
    arr = (nat.pastar_node * max(len(nodes), 1))()
    for k, nd in enumerate(nodes):
        for i, c in enumerate(nd.pos):
            arr[k].pos[i] = c
        arr[k].g, arr[k].f, arr[k].parent_mask = nd.g, nd.f, nd.parenti
    return arr


def lz4_en(payload):
    """pastar_lz4_en (lz4sup.cpp:13-43): the reference's wire frame of
    `payload` (bytes), byte-identical to the reference's; the trailing NUL
    of the reference's std::string is compressed with it."""
    payload = bytes(payload)
    bound = ctypes.c_int64()
    check(lib().pastar_wire_frame_bound(len(payload), ctypes.byref(bound)))
    out = ctypes.create_string_buffer(bound.value)
    n = ctypes.c_int64()
    check(lib().pastar_wire_frame_encode(payload, len(payload), out, bound.value, ctypes.byref(n)))
    return out.raw[:n.value]


def lz4_dec(frame):
    """pastar_lz4_dec (lz4sup.cpp:45-70): the frame's decoded bytes, the
    trailing NUL included (the reference returns that length too)."""
    frame = bytes(frame)
    if len(frame) < 12:
        raise nat.NativeError(-1, "frame shorter than its header")  # PASTAR_EINVAL
    total = int.from_bytes(frame[0:4], "little")
    orig = int.from_bytes(frame[8:12], "little")
    # the header is untrusted: an LZ4 block expands at most 255x, so a length
    # beyond that (or a frame shorter than it says) is rejected before any
    # buffer is sized from it
    if total > len(frame) or total < 12 or orig > 255 * (total - 12) + 16:
        raise nat.NativeError(-1, "frame header inconsistent with the frame's size")
    out = ctypes.create_string_buffer(max(orig, 1))
    n = ctypes.c_int64()
    check(lib().pastar_wire_frame_decode(frame, len(frame), out, orig, ctypes.byref(n)))
    return out.raw[:n.value]


def pack_nodes(nodes, n):
    """Node records in Node<N>::serialize field order (Node.h:57-64:
    g, f, pos[N], parenti; little-endian, 12 + 2N bytes each)."""
    arr = _c_nodes(nodes)
    cap = (12 + 2 * n) * len(nodes)
    out = ctypes.create_string_buffer(max(cap, 1))
    ln = ctypes.c_int64()
    check(lib().pastar_wire_pack_nodes(arr, len(nodes), n, out, cap, ctypes.byref(ln)))
    return out.raw[:ln.value]


def unpack_nodes(data, n):
    data = bytes(data)
    cap = len(data) // (12 + 2 * n)
    arr = (nat.pastar_node * max(cap, 1))()
    c = ctypes.c_int()
    check(lib().pastar_wire_unpack_nodes(data, len(data), n, arr, cap, ctypes.byref(c)))
    return [Node(tuple(arr[k].pos[:n]), arr[k].g, arr[k].f, arr[k].parent_mask) for k in range(c.value)]


def _c_coord(coord):
    c = (ctypes.c_uint16 * nat.MAX_SEQ)()
    for i, v in enumerate(coord):
        c[i] = v
    return c


class PriorityList:
    """The OpenList (PriorityList<N>, PriorityList.h:52-122) on the device:
    the engine's node table and f-bucket queues driven one call at a time
    (pastar_gpu_lists_reset / open_* in include/pastar_gpu.h).  Construct it
    to start an empty OpenList + ClosedList pair on the engine's context."""

    def __init__(self, engine, opt=None):
        self.engine = engine
        so = (opt or PAStarOpt()).search_opts()
        check(lib().pastar_gpu_lists_reset(engine._ctx, ctypes.byref(so)))
        self.closed = ClosedList(engine)

    def dequeue(self):
        """PriorityList::dequeue + the worker's ClosedList insert: a node of
        the lowest f, or None when the OpenList is empty."""
        got = self.dequeue_batch(1)
        return got[0] if got else None

    def dequeue_batch(self, max_nodes):
        """Up to max_nodes nodes, all of the lowest f."""
        out = (nat.pastar_node * max_nodes)()
        cnt = ctypes.c_int()
        check(lib().pastar_gpu_open_dequeue(self.engine._ctx, out, max_nodes, ctypes.byref(cnt)))
        n = self.engine.n
        return [Node(tuple(out[k].pos[:n]), out[k].g, out[k].f, out[k].parent_mask) for k in range(cnt.value)]

    def enqueue(self, nodes):
        """PAStar::enqueue (PAStar.cpp:219-237) over a batch: the ClosedList
        check, then PriorityList::conditional_enqueue.  The reference returns
        nothing; this returns which nodes are now the OpenList's record of
        their coordinate."""
        nodes = list(nodes) if not isinstance(nodes, Node) else [nodes]
        if not nodes:
            return []
        added = (ctypes.c_int32 * len(nodes))()
        reop = ctypes.c_int64()
        check(lib().pastar_gpu_open_enqueue(self.engine._ctx, _c_nodes(nodes), len(nodes), added,
                                            ctypes.byref(reop)))
        return [bool(a) for a in added]

    def conditional_enqueue(self, node):
        """PriorityList::conditional_enqueue (PriorityList.h:104-113), with
        the reference's return value: True whether the node was inserted,
        replaced a worse record or was discarded as not better (:109-110
        returns true for that too).  The ClosedList check of PAStar::enqueue
        is part of the call (one device record serves both lists); every
        call site of the reference makes that check first."""
        self.enqueue([node])
        return True

    def get_highest_priority(self):
        f = ctypes.c_int32()
        check(lib().pastar_gpu_open_highest_priority(self.engine._ctx, ctypes.byref(f)))
        return f.value

    def size(self):
        o, c = ctypes.c_int64(), ctypes.c_int64()
        check(lib().pastar_gpu_lists_size(self.engine._ctx, ctypes.byref(o), ctypes.byref(c)))
        return o.value

    def empty(self):
        return self.get_highest_priority() == 2 ** 31 - 1

    def find(self, coord):
        """The OpenList's node at coord, or None."""
        nd, where = self.closed._find(coord)
        return nd if where == 1 else None

    def erase(self, coord):
        e = ctypes.c_int()
        check(lib().pastar_gpu_lists_erase(self.engine._ctx, _c_coord(coord), 1, ctypes.byref(e)))
        return e.value

    def reopened(self):
        r = ctypes.c_int64()
        check(lib().pastar_gpu_lists_reopened(self.engine._ctx, ctypes.byref(r)))
        return r.value


class ClosedList:
    """The ClosedList (std::map<Coord<N>, Node<N>>, PAStar.cpp:92) of the same
    device session: nodes enter it through PriorityList.dequeue."""

    def __init__(self, engine):
        self.engine = engine

    def _find(self, coord):
        out = nat.pastar_node()
        where = ctypes.c_int()
        check(lib().pastar_gpu_lists_find(self.engine._ctx, _c_coord(coord), ctypes.byref(out), ctypes.byref(where)))
        if not where.value:
            return None, 0
        return Node(tuple(out.pos[:self.engine.n]), out.g, out.f, out.parent_mask), where.value

    def find(self, coord):
        nd, where = self._find(coord)
        return nd if where == 2 else None

    def erase(self, coord):
        e = ctypes.c_int()
        check(lib().pastar_gpu_lists_erase(self.engine._ctx, _c_coord(coord), 2, ctypes.byref(e)))
        return e.value

    def size(self):
        o, c = ctypes.c_int64(), ctypes.c_int64()
        check(lib().pastar_gpu_lists_size(self.engine._ctx, ctypes.byref(o), ctypes.byref(c)))
        return c.value


def sharded_search(sequences, n_shards, devices=(0,), opt=None, **engine_kw):
    """One search sharded over `n_shards` contexts of this process (one host
    thread each, ShardGroup transport); devices are used round-robin.
    Returns (per-shard SearchResult list, alignment rows)."""
    import threading
    if isinstance(sequences, (list, tuple)):
        sequences = Sequences(sequences)
    group = ShardGroup(n_shards)
    engines = [Engine(sequences, device=devices[r % len(devices)], shard_rank=r, group=group, **engine_kw)
               for r in range(n_shards)]
    results, rows, errors = [None] * n_shards, [None] * n_shards, []

    def run(r):
        try:
            results[r] = engines[r].pa_star(opt)
            rows[r] = engines[r].alignment()
        except Exception as ex:  # pragma: no cover - surfaced below
            errors.append(ex)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(n_shards)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in engines:
        e.close()
    group.close()
    if errors:
        raise errors[0]
    return results, rows[0]


def similarity(rows):
    """backtrace_print_similarity (backtrace.cpp:136-165): percent as a float32."""
    n, total, equal = len(rows), 0, 0
    for col in zip(*rows):
        for i in range(n):
            for j in range(i + 1, n):
                equal += col[i] == col[j]
                total += 1
    return float(np.float32(equal * 100) / np.float32(total))
