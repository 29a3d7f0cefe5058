"""GPU tests of the open list's reserve / store hand-over and of the bounded
device waits (csrc/kernels.hpp queue_reserve / queue_store; the device form
of PAStar::enqueue's inserts, PAStar.cpp:219-237, run by many workgroups at
once).  Every kernel these tests launch ends by itself: the waits they
exercise are bounded on the device."""
import pytest

from conftest import golden
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences
from mpi_pastar_msa_amd._native import EDEVWAIT, NativeError

pytestmark = pytest.mark.gpu


def test_crossed_reservations_complete():
    """Two workgroups reserve ranges of two buckets in crossed order and
    store first where they came second: every entry must land, in order."""
    with Engine(Sequences.from_fasta(golden("test2.fasta"))).init() as e:
        for _ in range(3):
            wrong, checked = e.selftest_queue(0)
            assert wrong == 0 and checked == 64


def test_lost_opener_is_reported_not_hung():
    """A store into a chunk nobody opened gives up after its poll limit, the
    call names the site, and the context still searches correctly after."""
    with Engine(Sequences.from_fasta(golden("test2.fasta"))).init() as e:
        with pytest.raises(NativeError) as ei:
            e.selftest_queue(1)
        assert ei.value.code == EDEVWAIT
        assert "queue_store" in str(ei.value)
        # the fault word was cleared: the next calls run clean
        assert e.selftest_queue(0) == (0, 64)
        r = e.pa_star(PAStarOpt(mode="batched"))
        assert r.score == 45037
