"""Run one workload a few times with device-clock profiling and verbose
diagnostics (select phase split).  Usage: python tools/gpu/probe.py WORKLOAD [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = Engine(Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", name + ".fasta")))
for i in range(reps):
    r = eng.pa_star(PAStarOpt(profile=True, verbose=(i == reps - 1)))
    print("score %d exp %d steps %d wall %.2f ms expand %.1f us/launch select %.1f gap %.1f retries %d" % (
        r.score, r.expansions, r.steps, r.seconds * 1e3, 1e3 * r.expand_ms / max(1, r.expand_launches),
        1e3 * r.select_ms / max(1, r.expand_launches), 1e3 * r.gap_ms / max(1, r.expand_launches), r.capacity_retries),
        flush=True)
