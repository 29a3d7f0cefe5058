"""Sweep the step band / batch size of the device search on one workload.

  python tools/tune.py WORKLOAD [--mult 0.25,0.5,1,2] [--batch 8192] [--reps 2]

Prints one line per setting: expansions, steps, reopen, wall-clock.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("workload")
ap.add_argument("--mult", default="0.125,0.25,0.5,1,2")
ap.add_argument("--batch", default="65536")
ap.add_argument("--kmin", type=int, default=0)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--table-log2", type=int, default=0)
a = ap.parse_args()
seqs = Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", a.workload + ".fasta"))
e = Engine(seqs).init()
o = e.initial_node()
kids = e.get_neigh(o)[0]
mean = sum(k.f - o.f for k in kids) / len(kids)
print("workload %s  h0 %d  mean df %.1f" % (a.workload, o.f, mean), flush=True)
for b in [int(x) for x in a.batch.split(",")]:
    for m in [float(x) for x in a.mult.split(",")]:
        band = max(1, int(mean * m))
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = e.pa_star(PAStarOpt(batch_nodes=b, batch_min=a.kmin, band=band, table_slots_log2=a.table_log2))
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print("batch %6d band %7d (x%.3f): score %d exp %9d reopen %8d steps %6d wall %.4f s  call %.4f s  %.3g exp/s"
              % (b, band, m, r.score, r.expansions_all, r.reopen, r.steps, r.seconds, best,
                 r.expansions_all / r.seconds), flush=True)
