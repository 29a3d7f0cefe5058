"""GPU test of pastar_gpu_expand_noalloc (include/pastar_gpu.h): the batched
Node::getNeigh (Node.cpp:206-248) through the entry point that allocates
nothing, against pastar_gpu_expand on the same inputs, bit for bit: two calls
in a row on one context, the second with a smaller input (the scratch keeps
the first call's contents), then the size limits."""
import ctypes
import random

import pytest

from conftest import golden
from mpi_pastar_msa_amd import Engine, Node, Sequences
from mpi_pastar_msa_amd import _native as nat

pytestmark = pytest.mark.gpu


def random_nodes(e, rng, count):
    lens = e.sequences.get_final_coord()
    nodes = []
    for _ in range(count):
        pos = tuple(rng.choice([0, L, rng.randint(0, L)]) if rng.random() < 0.3 else rng.randint(0, L) for L in lens)
        nodes.append(Node(pos, rng.randint(0, 50000), 0, rng.randint(1, (1 << e.n) - 1)))
    return nodes


def as_tuples(res):
    kids, own, src = res
    return [(k.pos, k.g, k.f, k.parenti) for k in kids], own, src


@pytest.mark.parametrize("name", ["kinase.fasta", "test.fasta"])
def test_noalloc_expand_matches_expand_twice(name):
    rng = random.Random(11)
    with Engine(Sequences.from_fasta(golden(name))).init() as e:
        per = (1 << e.n) - 1
        big = random_nodes(e, rng, min(1500, nat_max_out() // per))
        small = random_nodes(e, rng, 7)
        for nodes in (big, small):  # the second call is the smaller one
            for vec in (1, 8):
                want = as_tuples(e.get_neigh_batch(nodes, vec))
                got = as_tuples(e.get_neigh_batch(nodes, vec, noalloc=True))
                assert got == want
                assert len(got[0]) > 0


def nat_max_out():
    return 65536


def test_noalloc_expand_rejects_sizes_beyond_the_scratch():
    with Engine(Sequences.from_fasta(golden("test.fasta"))).init() as e:  # N = 8: 255 neighbours a node
        origin = e.initial_node()
        too_many_out = [origin] * (65536 // 255 + 1)
        with pytest.raises(nat.NativeError) as ei:
            e.get_neigh_batch(too_many_out, 1, noalloc=True)
        assert ei.value.code == nat.EINVAL and "exceed the scratch" in str(ei.value)
        goal = Node(e.sequences.get_final_coord(), 0, 0, 1)  # no neighbours: only the input count matters
        with pytest.raises(nat.NativeError) as ei:
            e.get_neigh_batch([goal] * 8193, 1, noalloc=True)
        assert ei.value.code == nat.EINVAL and "exceed the scratch" in str(ei.value)
        # at the limits it still runs, and an empty input is fine
        assert e.get_neigh_batch([goal] * 8192, 1, noalloc=True) == ([], [], [])
        assert e.get_neigh_batch([], 1, noalloc=True) == ([], [], [])
        ok = as_tuples(e.get_neigh_batch([origin] * 257, 4, noalloc=True))
        assert ok == as_tuples(e.get_neigh_batch([origin] * 257, 4))
