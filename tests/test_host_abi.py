"""CPU tests of the product's host side: the C-ABI library loads and exports
every entry point include/pastar_gpu.h declares, its host functions (FASTA
reader, Altschul weights, owner hash, cost table) agree with the oracle, the
device entry points fail loudly without a GPU, and the msa_pastar CLI keeps
the reference's options and error behaviour.  No GPU needed."""
import ctypes
import os
import random
import re
import subprocess

import numpy as np
import pytest

import oracle_bind as orc
from conftest import ROOT, golden
from mpi_pastar_msa_amd import Sequences, compute_weights, cost, get_id
from mpi_pastar_msa_amd import _native as nat

HEADER = os.path.join(ROOT, "include", "pastar_gpu.h")
CLI = os.path.join(ROOT, "mpi_pastar_msa_amd", "bin", "msa_pastar")
HAS_GPU = os.path.exists("/dev/kfd")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pastar_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = nat.lib()
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name
        assert name in nat.SIGNATURES, "binding missing for %s" % name
    out = subprocess.check_output(["nm", "-D", "--defined-only", nat.LIB_PATH], text=True)
    exported = set(re.findall(r" T (pastar_[a-z_]+)", out))
    assert set(names) <= exported


def test_abi_version():
    text = open(HEADER).read()
    version = int(re.search(r"#define PASTAR_ABI_VERSION (\d+)", text).group(1))
    assert nat.lib().pastar_abi_version() == version


def test_search_opts_layout_matches_header():
    """The ctypes mirror of pastar_search_opts has the header's fields in the
    header's order (the options travel by value across the C-ABI), and the
    Python options land in the fields of the same name."""
    from mpi_pastar_msa_amd import PAStarOpt
    text = open(HEADER).read()
    body = re.search(r"typedef struct pastar_search_opts \{(.*?)\} pastar_search_opts;", text, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    declared = re.findall(r"\b(int64_t|int32_t)\s+([a-z_0-9]+);", body)
    mirror = [(name, ctype) for name, ctype in nat.pastar_search_opts._fields_]
    assert [n for _, n in declared] == [n for n, _ in mirror]
    for (ctype_name, name), (_, ctype) in zip(declared, mirror):
        assert ctypes.sizeof(ctype) == (8 if ctype_name == "int64_t" else 4), name
    so = PAStarOpt(partial=3, xchg_lag=1, depth=7, batch_nodes=99, band=5, xchg_block_records=4096).search_opts()
    assert (so.partial, so.xchg_lag, so.depth, so.batch_nodes, so.band, so.xchg_block_records) == (3, 1, 7, 99, 5, 4096)
    assert PAStarOpt().search_opts().partial == 0  # the engine's default: partial expansion on for N >= 7


@pytest.mark.skipif(HAS_GPU, reason="a GPU is present")
def test_device_entry_points_fail_loudly_without_gpu():
    from mpi_pastar_msa_amd import Engine
    with pytest.raises(nat.NativeError) as ex:
        Engine(["ACDE", "ACE", "ADE"])
    assert ex.value.code == nat.ENODEV
    assert "no CPU fallback" in str(ex.value)


def test_cost_matches_oracle():
    for r in range(-2, 130):
        for l in range(-2, 130):
            assert cost(r, l) == orc.cost(r, l)


@pytest.mark.parametrize("size", [1, 2, 3, 7, 8, 64, 100])
@pytest.mark.parametrize("hash_type", [0, 1, 2, 3])
def test_owner_hash_matches_oracle(size, hash_type):
    rng = random.Random(size * 7 + hash_type)
    for _ in range(200):
        n = rng.choice([3, 4, 5, 8, 10, 16])
        c = [rng.randint(0, 1000) for _ in range(n)]
        shift = rng.randint(0, 21)
        assert get_id(c, size, hash_type, shift) == orc.get_id(c, size, hash_type, shift)


def test_owner_hash_invalid_shift():
    with pytest.raises(ValueError, match="Invalid Hash Shift"):
        get_id([1, 2, 3], 8, "FZORDER", 22)
    c = (ctypes.c_uint16 * 16)(1, 2, 3)
    assert nat.lib().pastar_owner(3, c, 8, 0, 22) == -1


@pytest.mark.parametrize("name", ["test", "test2", "PF08184", "kinase", "syn4x200_s1", "syn8x400_s5"])
def test_weights_bit_exact_with_oracle(name, kat):
    seqs = Sequences.from_fasta(golden(kat["inputs"][name]["file"]))
    w = compute_weights(seqs.seqs)
    ref = orc.weights(seqs.seqs)
    assert w.tobytes() == ref.tobytes()  # IEEE single, bit for bit
    n = len(seqs.seqs)
    ints = [int(w[x, y]) for x in range(n - 1) for y in range(x + 1, n)]
    if "weights" in kat["inputs"][name]:
        assert ints == kat["inputs"][name]["weights"]


def test_weights_random_sets_bit_exact():
    rng = random.Random(11)
    for _ in range(40):
        n = rng.randint(2, 9)
        seqs = ["".join(rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(rng.randint(1, 60))) for _ in range(n)]
        assert compute_weights(seqs).tobytes() == orc.weights(seqs).tobytes()


def test_weights_degenerate_families_follow_oracle():
    """Families of near-identical sequences on which the reference's weighting
    (WeightedSP.cpp:464-509) turns negative, or divides by a smallest weight
    of zero: the host pipeline gives the oracle's bits there too (the search
    over such weights has no defined optimum, in the reference either)."""
    neg = ["NTARICGENSIPVWIAHQKGPNDFYYRAFAAH", "SIPVEWIAHQHKGPGDFYYRFFAAH", "NTARICCENSIWPVEWIAHQKGGPRGDFY",
           "NTARICGENSIPVEWIAHQGPGDFYYRFFAAH"]
    nonfinite = ["EYKKIRYLAMTPHQV", "EYKKIRYLAMTPNQ", "EYKKIRYLAMWTPHQV"]
    for seqs in (neg, nonfinite):
        w, ref = compute_weights(seqs), orc.weights(seqs)
        assert w.tobytes() == ref.tobytes()
    assert (orc.weights(neg) < 0).any() and not np.isfinite(orc.weights(nonfinite)).all()


def test_fasta_reader_matches_oracle(tmp_path):
    p = tmp_path / "q.fasta"
    p.write_bytes(b">a\nACD\nEF\n\nGH\n>b\r\nKLM\r\n>c\nNP")
    assert Sequences.from_fasta(p).seqs == orc.Oracle(fasta=p).seqs == ["ACDEF", "GH", "KLM\r", "NP"]
    with pytest.raises(OSError, match="Can't open file"):
        Sequences.from_fasta(tmp_path / "missing.fasta")
    for name in ["test", "test2", "PF08184", "kinase", "syn8x400_s5"]:
        assert Sequences.from_fasta(golden(name + ".fasta")).seqs == orc.Oracle(fasta=golden(name + ".fasta")).seqs


@pytest.mark.skipif(not os.path.exists(CLI), reason="CLI not built")
class TestCli:
    def run(self, *args):
        return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=60)

    def test_version(self):
        r = self.run("-v")
        assert r.returncode == 0 and r.stdout == "msa_pastar, version 1.0\n"

    def test_help(self):
        r = self.run("-h")
        assert "Usage" in r.stdout and "--hash_type" in r.stdout

    def test_not_a_file(self):
        r = self.run("/nonexistent.fasta")
        assert "is not a regular file" in r.stdout

    def test_bad_hash_type(self):
        r = self.run("-y", "XOR", golden("test.fasta"))
        assert r.returncode != 0 and "hash_type" in r.stderr

    def test_bad_threads_and_shift(self):
        assert "Invalid number of threads" in self.run("-t", "0", golden("test.fasta")).stderr
        assert "Invalid Hash Shift" in self.run("-s", "30", golden("test.fasta")).stderr

    @pytest.mark.skipif(HAS_GPU, reason="a GPU is present")
    def test_no_gpu_is_fatal(self):
        r = self.run(golden("test.fasta"))
        assert r.returncode != 0 and "no CPU fallback" in r.stderr
