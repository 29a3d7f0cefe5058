"""Median search time of FASTA inputs under several batch_nodes values.
Usage: python tools/gpu/batch_probe.py "b1,b2,..." reps file1.fasta [...]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

batches = [int(x) for x in sys.argv[1].split(",")]
reps = int(sys.argv[2])
for path in sys.argv[3:]:
    e = Engine(Sequences.from_fasta(path)).init()
    score = None
    for b in batches:
        ts, ex = [], []
        for k in range(reps + 2):
            t = time.perf_counter()
            e.init()
            r = e.pa_star(PAStarOpt(batch_nodes=b))
            e.alignment()
            if k >= 2:
                ts.append(time.perf_counter() - t)
                ex.append(r.expansions_all)
            score = r.score if score is None else score
            assert r.score == score, (path, b, r.score, score)
        print("%-28s batch %7d: %.3f ms median (%d steps, %d expansions)" % (
            os.path.basename(path), b, 1e3 * statistics.median(ts), r.steps, statistics.median(ex)), flush=True)
    e.close()
