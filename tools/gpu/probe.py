"""Run workloads a few times with device-clock profiling.  Usage:
python tools/gpu/probe.py WORKLOAD[,WORKLOAD..] [reps] [depth,depth..] [verbose]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

KNOWN = {"syn4x200_s1": 149875, "PF08184": 24450, "kinase": 421546, "syn8x400_s5": 1318889, "test2": 45037,
         "syn8x100_s3": 703569, "syn8x400_s11": 1309114}
names = sys.argv[1].split(",")
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
depths = [int(d) for d in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
verbose = len(sys.argv) > 4
for name in names:
    eng = Engine(Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", name + ".fasta")))
    for d in depths:
        for i in range(reps):
            r = eng.pa_star(PAStarOpt(profile=True, depth=d, verbose=verbose and i == reps - 1,
                                      table_slots_log2=int(os.environ.get("TABLE_LOG2", "0")),
                                      pool_entries=int(os.environ.get("POOL", "0"))))
            ok = "ok" if r.score == KNOWN.get(name, r.score) else "WRONG"
            print("%-12s depth %d score %d %s exp %d steps %d wall %.2f ms expand %.1f us/launch select %.1f gap %.1f "
                  "retries %d" % (name, d, r.score, ok, r.expansions, r.steps, r.seconds * 1e3,
                                  1e3 * r.expand_ms / max(1, r.expand_launches),
                                  1e3 * r.select_ms / max(1, r.expand_launches),
                                  1e3 * r.gap_ms / max(1, r.expand_launches), r.capacity_retries), flush=True)
