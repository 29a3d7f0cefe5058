"""Partition study of the sharded search (the reference's zorder_tests.sh /
sum_tests.sh sweep, CoordHash.cpp:28-166), run on one GPU with the in-process
shard group: for each hash type and shift, the cross-shard traffic (records
exchanged), the load balance (max / mean expansions per shard) and the step
count.  On one GPU the shards share the chip, so the wall time is not the
multi-GPU time; traffic and balance are properties of the partition.

python tools/gpu/hash_sweep.py WORKLOAD[,..] SHARDS[,..] [HASH:SHIFT,..]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import PAStarOpt, Sequences, sharded_search  # noqa: E402

KNOWN = {"syn4x200_s1": 149875, "PF08184": 24450, "kinase": 421546, "syn8x400_s5": 1318889}
names = sys.argv[1].split(",")
shards = [int(v) for v in sys.argv[2].split(",")]
hashes = [(h.split(":")[0], int(h.split(":")[1])) for h in sys.argv[3].split(",")] if len(sys.argv) > 3 else [
    ("FZORDER", 12), ("FZORDER", 6), ("FZORDER", 18), ("FSUM", 12), ("PSUM", 12), ("PZORDER", 12)]
print("%-12s %6s %-8s %5s %9s %6s %11s %11s %8s %9s" % ("workload", "shards", "hash", "shift", "score", "steps",
                                                       "expansions", "exchanged", "balance", "search_ms"))
for name in names:
    seqs = Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", name + ".fasta"))
    for g in shards:
        for ht, sh in hashes:
            t0 = time.perf_counter()
            res, rows = sharded_search(seqs, g, opt=PAStarOpt(profile=True), hash_type=ht, hash_shift=sh)
            r0 = res[0]
            exp = [r.expansions for r in res]
            bal = max(exp) / max(1e-9, sum(exp) / len(exp))
            ok = "" if r0.score == KNOWN.get(name, r0.score) else " WRONG"
            print("%-12s %6d %-8s %5d %9d %6d %11d %11d %8.2f %9.2f%s" % (
                name, g, ht, sh, r0.score, r0.steps, r0.expansions_all, sum(r.exchanged for r in res), bal,
                max(r.seconds for r in res) * 1e3, ok), flush=True)
