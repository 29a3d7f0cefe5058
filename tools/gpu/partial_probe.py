"""Partial expansion (PASTAR_PARTIAL_K / PASTAR_PARTIAL_AHEAD): entries taken,
expansions, reopenings, children generated and table use of a workload's
search.  python tools/gpu/partial_probe.py [workload] [reps] [batch_nodes]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "syn8x400_s5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 0
e = Engine(Sequences.from_fasta("tests/golden/%s.fasta" % name)).init()
for k in range(reps):
    e.init()
    t = time.perf_counter()
    r = e.pa_star(PAStarOpt(profile=True, batch_nodes=batch, verbose=(k == reps - 1 and bool(os.environ.get("PROBE_VERBOSE")))))
    dt = time.perf_counter() - t
print("%s batch %d K=%s A=%s: %.2f ms score %d steps %d taken %d expanded %d reopen %d generated %.1f M table %.1f M slots 2^%d "
      "launch %.1f us" % (name, batch, os.environ.get("PASTAR_PARTIAL_K", "-"), os.environ.get("PASTAR_PARTIAL_AHEAD", "-"),
                          dt * 1e3, r.score, r.steps, r.expand_parents, r.expansions, r.reopen, r.generated / 1e6,
                          r.table_used / 1e6, r.table_slots.bit_length() - 1,
                          r.expand_ms * 1e3 / max(1, r.expand_launches)), flush=True)
