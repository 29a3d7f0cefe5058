"""Per-search wall time against the search loop's own time, with the sizes
each search ran at (tools/gpu, diagnostics): finds setup that lands inside
the bench's timed steps (reallocation, graph capture, restarts)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "syn8x400_s5"
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
e = Engine(Sequences.from_fasta("tests/golden/%s.fasta" % name)).init()
opt = PAStarOpt(table_slots_log2=lg, profile=True)
for k in range(reps):
    t = time.perf_counter()
    e.init()
    t1 = time.perf_counter()
    r = e.pa_star(opt)
    t2 = time.perf_counter()
    e.alignment()
    e.synchronize()
    t3 = time.perf_counter()
    print("%s #%d: step %.2f ms (init %.2f, pa_star %.2f, loop %.2f, alignment %.2f) retries %d table 2^%d pool %d "
          "used %d graph %d steps %d" % (name, k, (t3 - t) * 1e3, (t1 - t) * 1e3, (t2 - t1) * 1e3, r.seconds * 1e3,
                                         (t3 - t2) * 1e3, r.capacity_retries, r.table_slots.bit_length() - 1,
                                         r.pool_entries, r.table_used, r.graph_replay, r.steps), flush=True)
