"""Time the sharded search on one GPU (in-process shard group, peer copies):
python tools/gpu/probe_shards.py WORKLOAD[,..] SHARDS[,..] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import PAStarOpt, Sequences, sharded_search  # noqa: E402

names = sys.argv[1].split(",")
shards = [int(v) for v in sys.argv[2].split(",")]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for name in names:
    seqs = Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", name + ".fasta"))
    for g in shards:
        for _ in range(reps):
            t0 = time.perf_counter()
            res, rows = sharded_search(seqs, g, opt=PAStarOpt(profile=True, depth=int(os.environ.get("DEPTH", "0")),
                                                              xchg_lag=int(os.environ.get("LAG", "0")),
                                                              batch_nodes=int(os.environ.get("BATCH", "0"))),
                                       hash_type=os.environ.get("HASH", "FZORDER"),
                                       hash_shift=int(os.environ.get("SHIFT", "12")))
            dt = time.perf_counter() - t0
            r0 = res[0]
            ex = [r.expansions for r in res]
            print("%-12s shards %d score %d exp %d steps %d search %.2f ms (call %.1f ms) exchanged %d host waits %d "
                  "backlog steps %d max %d balance %.2f" % (
                      name, g, r0.score, r0.expansions_all, r0.steps, max(r.seconds for r in res) * 1e3, dt * 1e3,
                      sum(r.exchanged for r in res), r0.host_waits, sum(r.xchg_backlog_steps for r in res),
                      max(r.xchg_backlog_max for r in res), max(ex) * len(ex) / max(1, sum(ex))), flush=True)
