"""world_size-2 (and 3) CPU tests of the sharded path over torch.distributed
`gloo`.  No GPU.

The device search shards one A* by the reference's owner hash
(CoordHash.cpp / Sequences::get_id, z-order by default): every node lives on
exactly one shard, children are routed to their owner, and each step ends in
an exchange of fixed-size blocks whose headers carry what the reference's
check_stop allreduces (goal g, had work) plus the records sent and still
waiting (pastar_gpu.hip, search_impl, G > 1 branch; kernels.hpp xpack_kernel /
xinsert_kernel).
`ShardModel` below restates that protocol step for step on the CPU, with the
oracle's Node::getNeigh as the expansion and gloo as the transport, so the
protocol itself (termination rule, goal bound, reopening, owner routing,
backtrace across owners) is exercised with several ranks here; the HIP
implementation of the same protocol is covered on one GPU with 2-8 shards in
tests/test_gpu_parity.py (sharded search), and RCCL across GPUs by the
driver's multi-GPU bench.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bind as orc
from conftest import ROOT, golden

INT_MAX = 2**31 - 1


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, fn, *args):
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, val = q.get(timeout=240)
        out[rank] = val
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        if isinstance(out[r], BaseException):
            raise out[r]
    return [out[r] for r in range(world)]


def _entry(rank, world, port, fn, args, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    try:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        val = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent instead of hanging it
        val = RuntimeError("rank %d: %r" % (rank, e))
    q.put((rank, val))


class ShardModel:
    """One shard of the sharded search (search_impl, G > 1): a node table
    (pos -> best g, parent mask, closed), f-bucketed open lists of width
    2**band_log2 above f0 = h(origin), and the exchange of csrc/kernels.hpp
    (xpack / all-to-all / xinsert): a ring of records per destination shard,
    of which one step carries at most `block` per destination in a
    fixed-size block behind a header; every shard folds the same headers."""

    WINDOW = 4  # buckets above the shards' common lowest live bucket a batch may come from

    def __init__(self, o, rank, world, band_log2, batch, block=1 << 20, lag=0):
        self.o, self.rank, self.world = o, rank, world
        self.band, self.batch, self.block, self.lag = band_log2, batch, block, lag
        self.best = {}      # pos -> (g, parenti): owned nodes, and the best this shard sent of the others'
        self.closed = {}    # pos -> g it was expanded with
        self.buckets = {}   # bucket -> [(pos, g, f, parenti)]
        self.goal_pos = tuple(o.lengths)
        self.goal_g = INT_MAX
        self.f0 = o.initial_node()[2]
        self.expanded = 0
        self.sent = 0
        self.ring = [[] for _ in range(world)]  # records waiting for each destination
        self.gmin = 0        # lowest live bucket over all shards, as of their last select
        self.quiet_run = 0
        self.backlog_steps = 0
        self.pending = []    # lag 1: records received, relaxed after the next select

    def bucket(self, f):
        return max(0, (f - self.f0) >> self.band)

    def owner(self, pos):
        return orc.get_id(list(pos), self.world, 0, 12)

    def relax(self, node, owned=True):
        """relax() in device.hpp: improved iff strictly lower g.  A node of
        another shard is relaxed too (route_child's sender-side filter): it
        is sent only when this shard improved on what it sent before."""
        pos, g, f, par = node
        b = self.best.get(pos)
        if b is not None and b[0] <= g:
            return False
        self.best[pos] = (g, par)
        if pos == self.goal_pos:
            self.goal_g = min(self.goal_g, g)
            return not owned
        if owned:
            self.buckets.setdefault(self.bucket(f), []).append(node)
        return True

    def step(self):
        """select_kernel + expand_kernel: the lowest live bucket not above the
        goal's, if it lies inside the shards' common window; at most `batch`
        entries; stale entries (g no longer the best) are dropped.  Returns
        (has_work, lowest live bucket or None)."""
        limit = self.bucket(self.goal_g) if self.goal_g < INT_MAX else None
        live = sorted(b for b, v in self.buckets.items() if v and (limit is None or b <= limit))
        if not live:
            return 0, None
        b = live[0]
        if self.gmin is not None and b > self.gmin + self.WINDOW - 1:
            return 1, b  # live entries above the window: an idle step
        batch, self.buckets[b] = self.buckets[b][:self.batch], self.buckets[b][self.batch:]
        for node in batch:
            pos, g = node[0], node[1]
            if self.best[pos][0] != g:
                continue  # stale
            if self.goal_g < INT_MAX and node[2] >= self.goal_g:
                continue  # goal bound
            self.closed[pos] = g
            self.expanded += 1
            for kid, owner in self.o.get_neigh(node, self.world, 0, 12):
                if owner == self.rank:
                    self.relax(kid)
                elif self.relax(kid, owned=False):
                    self.ring[owner].append(kid)
        return 1, b

    def exchange(self, has_work, low_b):
        """xpack + the all-to-all + xinsert's header fold.  Every shard sends
        every shard one block of `block` record slots behind a header
        {n, sent_all, backlog_all, has_work, goal, low_b}; the fields other
        than n are the same in all of a sender's blocks.  Returns (records
        for this shard, headers of all shards)."""
        n, W, C = self.o.n, self.world, self.block
        width = n + 3
        take = [self.ring[d][:C] for d in range(W)]
        self.ring = [self.ring[d][C:] for d in range(W)]
        sent_all = sum(len(t) for t in take)
        backlog_all = sum(len(r) for r in self.ring)
        self.sent += sent_all
        self.backlog_steps += backlog_all > 0
        # (the model sizes its block tensor to the step's largest block: the
        # device's blocks are fixed-size, C records, mostly empty)
        cap_t = torch.tensor([max(len(t) for t in take)], dtype=torch.int64)
        dist.all_reduce(cap_t, op=dist.ReduceOp.MAX)
        cap = max(1, int(cap_t))
        area = torch.zeros((W, 6 + cap * width), dtype=torch.int64)
        for d in range(W):
            area[d, :6] = torch.tensor([len(take[d]), sent_all, backlog_all, has_work, self.goal_g,
                                        -1 if low_b is None else low_b])
            if take[d]:
                area[d, 6:6 + len(take[d]) * width] = torch.tensor(
                    [list(k[0]) + [k[1], k[2], k[3]] for k in take[d]], dtype=torch.int64).reshape(-1)
        got = [torch.zeros_like(area) for _ in range(W)]
        dist.all_gather(got, area)  # (rank s's block for this shard is got[s][self.rank])
        recs, hdrs = [], []
        for s_ in range(W):
            blk = got[s_][self.rank]
            hdrs.append([int(v) for v in blk[:6]])
            rows = blk[6:6 + int(blk[0]) * width].reshape(-1, width).tolist()
            recs += [(tuple(row[:n]), row[n], row[n + 1], row[n + 2]) for row in rows]
        return recs, hdrs

    def search(self, max_steps=100000):
        origin = self.o.initial_node()
        if self.owner(origin[0]) == self.rank:
            self.relax(origin)
        steps = 0
        while steps < max_steps:
            has_work, low_b = self.step()
            if self.lag:  # the records of the step before reach the open list after this select
                for rec in self.pending:
                    self.relax(rec)
                self.pending = []
            recs, hdrs = self.exchange(has_work, low_b)
            if self.lag:
                self.pending = recs
            else:
                for rec in recs:
                    self.relax(rec)
            steps += 1
            # xinsert's fold: only fields that are the same in all blocks of a sender
            self.goal_g = min([self.goal_g] + [h[4] for h in hdrs])
            lows = [h[5] for h in hdrs if h[5] >= 0]
            self.gmin = min(lows) if lows else None
            work = any(h[3] or h[1] for h in hdrs)
            backlog = sum(h[2] for h in hdrs)
            # termination: nobody had a batch, sent a record or keeps records
            # in its rings, for lag + 1 steps in a row (records in flight
            # under lag 1 were sent in the step before: not quiet)
            self.quiet_run = self.quiet_run + 1 if (not work and backlog == 0) else 0
            if self.quiet_run > self.lag:
                assert not self.pending and not any(self.ring)
                return steps
        raise RuntimeError("step limit")

    def walk(self):
        """walk_kernel + broadcast: the owner of the current node names its
        parent, until the origin."""
        n = self.o.n
        pos, path = self.goal_pos, [self.goal_pos]
        while any(pos):
            owner = orc.get_id(list(pos), self.world, 0, 12)
            t = torch.zeros(1, dtype=torch.int64)
            if owner == self.rank:
                t[0] = self.best[pos][1]
            dist.broadcast(t, owner)
            mask = int(t)
            pos = tuple(pos[d] - ((mask >> d) & 1) for d in range(n))
            path.append(pos)
        return path[::-1]


def rows_from_path(seqs, path):
    rows = ["" for _ in seqs]
    for a, b in zip(path, path[1:]):
        for d, s in enumerate(seqs):
            rows[d] += s[a[d]] if b[d] > a[d] else "-"
    return rows


def _sharded_search(rank, world, fasta, band_log2, batch, block=1 << 20, lag=0):
    o = orc.Oracle(fasta=fasta)
    m = ShardModel(o, rank, world, band_log2, batch, block, lag)
    steps = m.search()
    goal_owner = orc.get_id(list(m.goal_pos), world, 0, 12)
    path = m.walk()
    rows = rows_from_path(o.seqs, path)
    # every node has exactly one owner: nothing this shard expanded or queued belongs elsewhere
    foreign = sum(1 for p in m.closed if orc.get_id(list(p), world, 0, 12) != rank)
    foreign += sum(1 for v in m.buckets.values() for nd in v if orc.get_id(list(nd[0]), world, 0, 12) != rank)
    return {"goal_g": m.goal_g, "steps": steps, "expanded": m.expanded, "sent": m.sent,
            "backlog_steps": m.backlog_steps,
            "rows": rows, "cost": o.alignment_cost(rows), "foreign": foreign,
            "goal_owner_has_goal": (rank != goal_owner) or (m.goal_pos in m.best),
            "nodes": len(m.best)}


# (name, world, band_log2, batch, block records per destination and step, lag)
CASES = [("test2", 2, 4, 64, 1 << 20, 0), ("PF08184", 2, 6, 16, 1 << 20, 0), ("test", 2, 0, 1 << 20, 1 << 20, 0),
         ("test2", 3, 8, 8, 1 << 20, 0), ("syn4x200_s1", 2, 13, 4096, 1 << 20, 0),
         # blocks too small for a step's records (they wait in the rings), and the
         # exchange running beside the next step's expansion
         ("test2", 2, 4, 64, 3, 0), ("test2", 3, 8, 8, 2, 1), ("PF08184", 2, 6, 16, 1 << 20, 1),
         ("syn4x200_s1", 2, 13, 4096, 256, 1)]


@pytest.mark.parametrize("name,world,band_log2,batch,block,lag", CASES)
def test_sharded_protocol_reaches_reference_optimum(name, world, band_log2, batch, block, lag, kat):
    ref = kat["inputs"][name]
    res = run_ranks(world, _sharded_search, golden(ref["file"]), band_log2, batch, block, lag)
    assert len({r["steps"] for r in res}) == 1  # every shard stops at the same step
    if block < 100:
        assert sum(r["backlog_steps"] for r in res) > 0  # records really waited in a ring
    for r in res:
        assert r["goal_g"] == ref["score"]
        assert r["cost"] == ref["score"]
        assert r["foreign"] == 0
        assert r["goal_owner_has_goal"]
        assert r["rows"] == res[0]["rows"]
    o = orc.Oracle(fasta=golden(ref["file"]))
    assert [row.replace("-", "") for row in res[0]["rows"]] == o.seqs
    assert sum(r["sent"] for r in res) > 0  # the exchange really carried nodes
    assert all(r["expanded"] > 0 for r in res) or ref["expansions_t1"] < 30


def _owners_cover(rank, world, fasta):
    """Every child of every expansion is routed to exactly one shard in
    [0, world), and the union of what the shards receive is the whole set."""
    o = orc.Oracle(fasta=fasta)
    node = o.initial_node()
    frontier, seen = [node], []
    for _ in range(6):
        nxt = []
        for nd in frontier:
            for kid, owner in o.get_neigh(nd, world, 0, 12):
                assert 0 <= owner < world
                assert owner == orc.get_id(list(kid[0]), world, 0, 12)
                seen.append((kid[0], owner))
                nxt.append(kid)
        frontier = nxt[:50]
    mine = sorted({p for p, w in seen if w == rank})
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    allpos = sorted({p for p, _ in seen})
    return sorted(p for g in gathered for p in g) == allpos


def test_owner_partition_covers_every_node():
    assert all(run_ranks(2, _owners_cover, golden("test2.fasta")))


def _share_id(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import bench
    rid = bench.share_rccl_id(rank, world, lambda: bytes(range(128)))
    return rid


def test_bench_rccl_id_rendezvous():
    port = free_port() - 17
    res = run_ranks(2, _share_id, port)
    assert res[0] == res[1] == bytes(range(128))


def _wire_nodes(rank, n, count):
    import random
    from mpi_pastar_msa_amd import Node
    rng = random.Random(1000 + rank)
    out = []
    for _ in range(count):
        pos = tuple(rng.randrange(0, 300) for _ in range(n))
        g = sum(pos) * 30 + rng.randrange(0, 90)
        out.append(Node(pos, g, g + rng.randrange(0, 400), rng.randrange(1, 1 << n)))
    return out


def _wire_exchange(rank, world, n, count):
    """The reference's message path between ranks (PAStarSender.cpp:54-62 ->
    PAStarMessageProcesser.cpp:40-50): each rank routes its nodes to their
    owners (Coord::get_id, z-order / 12), packs every destination's nodes in
    Node::serialize field order, frames them as pastar_lz4_en does, and
    sends the frame; the owner decodes and unpacks.  gloo carries the bytes
    here in place of MPI."""
    from mpi_pastar_msa_amd import get_id, lz4_dec, lz4_en, pack_nodes, unpack_nodes
    mine = _wire_nodes(rank, n, count)
    per = {d: [x for x in mine if get_id(x.pos, world) == d] for d in range(world)}
    reqs, keep = [], []
    for d in range(world):
        if d == rank:
            continue
        frame = lz4_en(pack_nodes(per[d], n))
        t_len = torch.tensor([len(frame)], dtype=torch.int64)
        t_buf = torch.frombuffer(bytearray(frame), dtype=torch.uint8)
        keep += [t_len, t_buf]
        reqs.append(dist.isend(t_len, d))
        reqs.append(dist.isend(t_buf, d))
    got = list(per[rank])
    for s in range(world):
        if s == rank:
            continue
        t_len = torch.zeros(1, dtype=torch.int64)
        dist.recv(t_len, s)
        t_buf = torch.zeros(int(t_len.item()), dtype=torch.uint8)
        dist.recv(t_buf, s)
        raw = lz4_dec(t_buf.numpy().tobytes())
        assert raw[-1:] == b"\0"
        got += unpack_nodes(raw[:-1], n)
    for r in reqs:
        r.wait()
    assert all(get_id(x.pos, world) == rank for x in got)
    # every rank regenerates what the others sent it
    want = [x for s in range(world) for x in _wire_nodes(s, n, count) if get_id(x.pos, world) == rank]
    key = lambda x: (x.pos, x.g, x.f, x.parenti)
    assert sorted(map(key, got)) == sorted(map(key, want))
    return len(got)


@pytest.mark.parametrize("world,n", [(2, 4), (3, 8)])
def test_wire_frame_exchange_between_ranks(world, n):
    counts = run_ranks(world, _wire_exchange, n, 3000)
    assert sum(counts) == world * 3000
    assert all(c > 0 for c in counts)
