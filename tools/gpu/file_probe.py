"""Repeated searches of one FASTA file: best and median search time, expansions,
steps.  python tools/gpu/file_probe.py path [reps] [mode]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
mode = sys.argv[3] if len(sys.argv) > 3 else "batched"
e = Engine(Sequences.from_fasta(path)).init()
ts = []
for k in range(reps):
    e.init()
    t = time.perf_counter()
    r = e.pa_star(PAStarOpt(mode=mode))
    e.alignment()
    ts.append(time.perf_counter() - t)
ts = ts[2:] if len(ts) > 3 else ts
print("%-22s %s: score %d median %.3f ms best %.3f ms expansions %d steps %d" % (
    os.path.basename(path), os.environ.get("TAG", ""), r.score, statistics.median(ts) * 1e3, min(ts) * 1e3,
    r.expansions_all, r.steps), flush=True)
