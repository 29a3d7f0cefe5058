"""Repeated sharded searches of one workload on the in-process shard group:
how often a configuration ends with a score other than the known optimum.
python tools/gpu/shard_repeat.py name shards lag block reps"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import PAStarOpt, Sequences, sharded_search  # noqa: E402

KNOWN = {"syn4x200_s1": 149875, "kinase": 421546, "syn8x100_s3": 703569, "syn8x400_s5": 1318889}
name, shards, lag, block, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
seqs = Sequences.from_fasta("tests/golden/%s.fasta" % name)
bad = 0
for k in range(reps):
    res, rows = sharded_search(seqs, shards, opt=PAStarOpt(xchg_lag=lag, xchg_block_records=block))
    if res[0].score != KNOWN[name] or len({r.steps for r in res}) != 1:
        bad += 1
        print("run %d: scores %s steps %s backlog steps %d retries %s exchanged %d expansions %d" % (
            k, sorted({r.score for r in res}), sorted({r.steps for r in res}), sum(r.xchg_backlog_steps for r in res),
            [r.capacity_retries for r in res], sum(r.exchanged for r in res), res[0].expansions_all), flush=True)
    elif k < 3 or k % 50 == 49:
        print("run %d ok: steps %d backlog steps %d retries %s exchanged %d expansions %d" % (
            k, res[0].steps, sum(r.xchg_backlog_steps for r in res), [r.capacity_retries for r in res],
            sum(r.exchanged for r in res), res[0].expansions_all), flush=True)
print("%s shards %d lag %d block %d: %d of %d runs wrong" % (name, shards, lag, block, bad, reps), flush=True)
