"""GPU parity of the LDS-resident search (csrc/solo.hpp): PairAlign, the A*
and the backtrace of a small problem in one single-workgroup launch, against
the oracle and the reference's known answers.  Integer work: exact."""
import hashlib
import random

import pytest

import oracle_bind as orc
from conftest import golden
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences, similarity
from mpi_pastar_msa_amd._native import EINVAL, ENOMEM, ESTATE, NativeError

pytestmark = pytest.mark.gpu

SOLO = ["test", "test2", "PF08184"]


def _md5(rows):
    return hashlib.md5("".join(r + "\n" for r in rows).encode()).hexdigest()


@pytest.mark.parametrize("name", SOLO)
def test_solo_known_answers(name, kat):
    """Score, alignment md5 and similarity the reference printed, from one
    launch; the goal is in the dumped closed list with g == score."""
    ref = kat["inputs"][name]
    o = orc.Oracle(fasta=golden(ref["file"]))
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        for _ in range(3):  # a repeated search on the context starts clean
            r = e.pa_star(PAStarOpt(mode="solo", profile=True))
            assert r.solo == 1 and r.expand_launches == 1 and r.expand_ms > 0
            assert r.score == ref["score"]
            assert r.expansions_all >= ref["expansions_t1"]
            rows = e.alignment()
            assert [row.replace("-", "") for row in rows] == e.sequences.seqs
            assert o.alignment_cost(rows) == ref["score"]
            if "alignment_md5" in ref:
                assert _md5(rows) == ref["alignment_md5"]
            assert "%.2f" % similarity(rows) == ref["similarity"]
            goal = e.closed_lookup(e.sequences.get_final_coord())
            assert goal is not None and goal.g == ref["score"] and goal.f == ref["score"]
            origin = e.closed_lookup(e.sequences.get_initial_coord())
            assert origin.g == 0 and origin.f == ref["h_origin"]


@pytest.mark.parametrize("name", SOLO)
def test_solo_matches_batched_engine(name, kat):
    """Same score and the same alignment as the batched engine on one
    context; the closed-list lookups follow the engine that ran last."""
    ref = kat["inputs"][name]
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        rs = e.pa_star(PAStarOpt(mode="solo"))
        rows_s = e.alignment()
        rb = e.pa_star(PAStarOpt(mode="batched"))
        assert rb.solo == 0
        rows_b = e.alignment()
        assert rs.score == rb.score == ref["score"]
        assert rows_s == rows_b
        assert e.closed_lookup(e.sequences.get_final_coord()).g == ref["score"]
        rs2 = e.pa_star(PAStarOpt())  # auto: solo again
        assert rs2.solo == 1 and e.alignment() == rows_s


def test_solo_random_problems_match_oracle():
    """Random 2..8-sequence problems, ragged lengths, residues the reference
    costs 0: score and a valid optimal alignment on the solo path."""
    rng = random.Random(23)
    odd = "ACDEFGHIKLMNPQRSTVWY" + "BJOUXZ" + "acdwxy"
    ran = 0
    for trial in range(24):
        n = 2 + trial % 7
        maxlen = {2: 60, 3: 24, 4: 10, 5: 6, 6: 5, 7: 4, 8: 3}[n]
        seqs = ["".join(rng.choice(odd if trial % 3 == 0 else odd[:20]) for _ in range(rng.randint(1, maxlen)))
                for _ in range(n)]
        o = orc.Oracle(seqs=seqs)
        ref = o.astar()
        with Engine(seqs).init() as e:
            try:
                r = e.pa_star(PAStarOpt(mode="solo"))
            except NativeError as ex:  # outgrew the LDS node table
                assert ex.code == ENOMEM
                continue
            ran += 1
            assert r.score == ref["score"], (seqs, r, ref)
            rows = e.alignment()
            assert [row.replace("-", "") for row in rows] == seqs
            assert o.alignment_cost(rows) == ref["score"]
    assert ran >= 16


def test_solo_overflow_falls_back_to_batched():
    """A problem whose tables fit the LDS but whose search outgrows the LDS
    node table: mode solo reports ENOMEM, auto finishes on the batched
    engine (and stays there for the context), with the optimal score."""
    rng = random.Random(5)
    aa = "ACDEFGHIKLMNPQRSTVWY"
    base = "".join(rng.choice(aa) for _ in range(59))

    def mutate(rate=0.6):  # a family around one ancestor: ~4 K nodes, LDS holds 1 K
        out = []
        for ch in base:
            r = rng.random()
            if r < rate / 3:
                continue
            out.append(rng.choice(aa) if r < 2 * rate / 3 else ch)
            if 2 * rate / 3 <= r < rate:
                out.append(rng.choice(aa))
        return "".join(out)

    seqs = [mutate() for _ in range(3)]
    o = orc.Oracle(seqs=seqs)
    ref = o.astar()
    with Engine(seqs).init() as e:
        with pytest.raises(NativeError) as ex:
            e.pa_star(PAStarOpt(mode="solo"))
        assert ex.value.code == ENOMEM
        r = e.pa_star(PAStarOpt())
        assert r.solo == 0 and r.score == ref["score"]
        assert o.alignment_cost(e.alignment()) == ref["score"]
        assert e.pa_star(PAStarOpt()).solo == 0


def test_solo_step_limit_and_mode_errors(kat):
    from mpi_pastar_msa_amd._native import ENOTFOUND  # noqa: F401
    ref = kat["inputs"]["PF08184"]
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        assert e.pa_star(PAStarOpt(mode="solo")).score == ref["score"]
        with pytest.raises(NativeError) as ex:
            e.pa_star(PAStarOpt(mode="solo", max_steps=3))
        assert ex.value.code == ESTATE
        with pytest.raises(NativeError) as ex:
            e.alignment()
        assert ex.value.code == ESTATE
        assert e.pa_star(PAStarOpt(mode="solo")).score == ref["score"]
    big = kat["inputs"]["syn4x200_s1"]
    with Engine(Sequences.from_fasta(golden(big["file"]))).init() as e:
        with pytest.raises(NativeError) as ex:  # 1.9 MB of pair tables: not an LDS problem
            e.pa_star(PAStarOpt(mode="solo"))
        assert ex.value.code == EINVAL


def test_solo_pair_tables_and_h_after_search(kat):
    """The solo search builds its pair tables in LDS only; the HBM tables the
    other entry points read are built on first use, bit-exact."""
    import numpy as np
    ref = kat["inputs"]["PF08184"]
    o = orc.Oracle(fasta=golden(ref["file"]))
    with Engine(Sequences.from_fasta(golden(ref["file"]))).init() as e:
        assert e.pa_star(PAStarOpt()).solo == 1
        assert e.initial_node().f == ref["h_origin"]
        for k in range(e.npairs):
            np.testing.assert_array_equal(e.pair_table(k), o.pair_table(k))


@pytest.mark.parametrize("length,mutate", [(64, False), (100, False), (100, True), (100, "insert")])
def test_solo_long_paths(length, mutate):
    """Backtraces of 64 and more steps, by the walk (masks leave the kernel 64
    at a time) or by pointer jumping (a path longer than 128 steps takes a
    whole top-level jump): two sequences whose alignment has at least
    `length` columns, identical (a diagonal path of exactly `length` steps),
    mutated, or the second with ~30 insertions (a path of >= 129 steps)."""
    rng = random.Random(length)
    aa = "ACDEFGHIKLMNPQRSTVWY"
    a = "".join(rng.choice(aa) for _ in range(length))
    b = a
    if mutate == "insert":
        b = "".join(ch + (rng.choice(aa) if rng.random() < 0.3 else "") for ch in a)
        assert len(b) >= 129
    elif mutate:
        b = "".join(rng.choice(aa) if rng.random() < 0.2 else ch for ch in a if rng.random() > 0.1)
    seqs = [a, b]
    o = orc.Oracle(seqs=seqs)
    ref = o.astar()
    with Engine(seqs).init() as e:
        r = e.pa_star(PAStarOpt(mode="solo"))
        assert r.solo == 1 and r.score == ref["score"]
        rows = e.alignment()
        assert [row.replace("-", "") for row in rows] == seqs
        assert o.alignment_cost(rows) == ref["score"]
        assert len(rows[0]) >= length
        if not mutate:
            assert rows == seqs
        rb = e.pa_star(PAStarOpt(mode="batched"))
        assert rb.score == r.score and e.alignment() == rows


def test_search_many_matches_single_searches(kat):
    """pastar_gpu_search_many: independent searches of different problems
    (same N) in one launch, one workgroup each, against the same searches run
    one by one and against the oracle: scores, expansion counts, alignments."""
    import random
    from mpi_pastar_msa_amd import search_many
    rng = random.Random(5)
    ref = kat["inputs"]["PF08184"]
    problems = [Sequences.from_fasta(golden(ref["file"]))]
    for _ in range(9):
        root = [rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(rng.randint(20, 50))]
        seqs = []
        for _ in range(3):
            s = [rng.choice("ACDEFGHIKLMNPQRSTVWY") if rng.random() < 0.15 else c for c in root if rng.random() > 0.05]
            seqs.append("".join(s) or "A")
        problems.append(Sequences(seqs))
    engines = [Engine(p).init() for p in problems]
    try:
        many = search_many(engines)
        rows_many = [e.alignment() for e in engines]
        for p, e, r, rows in zip(problems, engines, many, rows_many):
            o = orc.Oracle(seqs=p.seqs)
            want = o.astar()
            assert r.solo == 1 and r.score == want["score"]
            assert o.alignment_cost(rows) == r.score
            assert [row.replace("-", "") for row in rows] == p.seqs
            single = e.pa_star(PAStarOpt(mode="solo"))
            assert (single.score, single.expansions_all, single.generated) == (r.score, r.expansions_all, r.generated)
            assert e.alignment() == rows
        assert many[0].score == ref["score"] and many[0].expansions_all == ref["expansions_t1"]
        # the same batch again (the contexts' result areas are reused), and a
        # batch that repeats a context is refused
        again = search_many(engines)
        assert [r.score for r in again] == [r.score for r in many]
        with pytest.raises(NativeError) as ei:
            search_many([engines[0], engines[0]])
        assert ei.value.code == EINVAL
    finally:
        for e in engines:
            e.close()
