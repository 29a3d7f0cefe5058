"""GPU tests of the OpenList / ClosedList boundary (include/pastar_gpu.h
pastar_gpu_lists_* / open_*, include/pastar_lists.hpp): the reference's
serial worker loop (worker_inner, PAStar.cpp:320-401) driven one list call
at a time reaches the oracle's optimal score, and the list operations keep
PriorityList / ClosedList semantics (PriorityList.h:52-122, PAStar.cpp:219-250)."""
import os
import random
import subprocess

import pytest

import oracle_bind as orc
from conftest import ROOT, golden
from mpi_pastar_msa_amd import ClosedList, Engine, Node, PAStarOpt, PriorityList, Sequences
from mpi_pastar_msa_amd._native import ESTATE, NativeError

pytestmark = pytest.mark.gpu

DEMO = os.path.join(ROOT, "mpi_pastar_msa_amd", "bin", "pastar_lists_astar")


def worker_loop(e):
    """worker_inner at one thread over the device lists: dequeue, the final
    node's check_stop, getNeigh on the device, PAStar::enqueue."""
    open_ = PriorityList(e)
    closed = ClosedList(e)
    goal = e.sequences.get_final_coord()
    open_.enqueue([e.initial_node()])
    expansions = 0
    while True:
        cur = open_.dequeue()
        assert cur is not None, "OpenList exhausted"
        expansions += 1
        assert closed.find(cur.pos) == cur  # the worker's ClosedList insert
        if cur.pos == goal:
            if open_.get_highest_priority() < cur.f:
                closed.erase(cur.pos)
                assert open_.conditional_enqueue(cur) is True
                continue
            return cur, expansions, open_, closed
        open_.enqueue(e.get_neigh(cur)[0])


@pytest.mark.parametrize("name", ["test", "test2", "PF08184"])
def test_worker_loop_over_device_lists(name, kat):
    ref = kat["inputs"][name]
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        cur, expansions, open_, closed = worker_loop(e)
        assert cur.g == cur.f == ref["score"]
        # serial A*: the reference's -t 1 count, up to the order of f ties
        assert ref["expansions_t1"] <= expansions <= 2 * ref["expansions_t1"] + 2
        assert closed.size() == expansions - open_.reopened()
        assert open_.size() >= 0


def test_worker_loop_random_problems_match_oracle():
    rng = random.Random(3)
    for trial in range(4):
        n = 3 + trial % 3
        seqs = ["".join(rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(rng.randint(3, 9))) for _ in range(n)]
        o = orc.Oracle(seqs=seqs)
        ref = o.astar()
        with Engine(seqs).init() as e:
            cur, expansions, _, _ = worker_loop(e)
            assert cur.g == ref["score"], (seqs, cur, ref)
            assert expansions >= ref["expansions"] - 2


@pytest.mark.parametrize("name", ["test2", "PF08184"])
def test_cpp_facades_drive_the_reference_loop(name, kat):
    """include/pastar_lists.hpp from C++: the worker loop of
    csrc/lists_astar_main.cpp prints the reference's Final Score line."""
    ref = kat["inputs"][name]
    r = subprocess.run([DEMO, golden(ref["file"])], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    s = ref["score"]
    assert "\tg - %d (h - 0 f - %d)" % (s, s) in r.stdout
    exp = int(r.stdout.split("expansions ")[1].split()[0])
    assert ref["expansions_t1"] <= exp <= 2 * ref["expansions_t1"] + 2


def test_list_operations_semantics(kat):
    ref = kat["inputs"]["test2"]
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        open_ = PriorityList(e)
        closed = ClosedList(e)
        assert open_.empty() and open_.size() == 0 and closed.size() == 0
        assert open_.get_highest_priority() == 2 ** 31 - 1
        assert open_.dequeue() is None
        origin = e.initial_node()
        kids = e.get_neigh(origin)[0]
        assert open_.enqueue(kids) == [True] * len(kids)
        assert open_.size() == len(kids)
        best = min(k.f for k in kids)
        assert open_.get_highest_priority() == best
        # conditional_enqueue returns true in all three of the reference's
        # cases (PriorityList.h:104-113): an equal or larger f is discarded
        # (:109-110 returns true), a smaller one replaces the node's record
        k0 = kids[0]
        worse, same = Node(k0.pos, k0.g + 5, k0.f + 5, k0.parenti), Node(k0.pos, k0.g, k0.f, k0.parenti)
        assert open_.conditional_enqueue(worse) is True and open_.find(k0.pos) == k0
        assert open_.conditional_enqueue(same) is True and open_.find(k0.pos) == k0
        assert open_.enqueue([worse, same]) == [False, False]
        lower = Node(k0.pos, k0.g - 7, k0.f - 7, k0.parenti)
        assert open_.conditional_enqueue(lower) is True
        assert open_.find(k0.pos) == lower and open_.size() == len(kids)
        # dequeue: lowest f first, into the ClosedList
        first = open_.dequeue()
        assert first.f == min(best, lower.f)
        assert closed.find(first.pos) == first and open_.find(first.pos) is None
        assert closed.size() == 1 and open_.size() == len(kids) - 1
        # PAStar::enqueue: a closed node with a worse g is discarded, a better
        # one leaves the ClosedList and is counted as reopened once
        assert open_.enqueue([first]) == [False] and open_.reopened() == 0
        better = Node(first.pos, first.g - 1, first.f - 1, first.parenti)
        assert open_.enqueue([better]) == [True]
        assert open_.reopened() == 1 and open_.find(first.pos) == better and closed.find(first.pos) is None
        # ... and not again when the reopened node is dequeued
        again = open_.dequeue()
        assert again == better and closed.find(first.pos) == better
        assert open_.reopened() == 1
        # two improving entries of one batch reopen their node once
        b1 = Node(first.pos, better.g - 2, better.f - 2, first.parenti)
        b2 = Node(first.pos, better.g - 3, better.f - 3, first.parenti)
        open_.enqueue([b1, b2])
        assert open_.reopened() == 2 and open_.find(first.pos) == b2
        # ties: a batch of the lowest f
        t = open_.get_highest_priority()
        batch = open_.dequeue_batch(64)
        assert batch and all(b.f == t for b in batch)
        assert len({b.pos for b in batch}) == len(batch)
        # erase from either list
        some = batch[0]
        assert open_.erase(some.pos) == 0 and closed.erase(some.pos) == 1
        assert closed.find(some.pos) is None and open_.find(some.pos) is None
        left = [k for k in kids if open_.find(k.pos)]
        if left:
            assert open_.erase(left[0].pos) == 1 and open_.find(left[0].pos) is None
        # drain: f never decreases
        last = -1
        while True:
            nd = open_.dequeue()
            if nd is None:
                break
            assert nd.f >= last
            last = nd.f
        assert open_.empty()
        # a search ends the session
        e.pa_star(PAStarOpt())
        with pytest.raises(NativeError) as ex:
            open_.dequeue()
        assert ex.value.code == ESTATE
