"""Child relaxations per second of the expand kernel (one table probe and at
most one device-scope atomic each) against the measured chip ceiling for
random 8-B atomics (tools/micro/atomic_rate.hip), per workload (tools/gpu,
diagnostics)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["syn4x200_s1", "kinase"]):
    e = Engine(Sequences.from_fasta("tests/golden/%s.fasta" % name)).init()
    opt = PAStarOpt(profile=True, mode="batched", table_slots_log2=26 if name.startswith("syn8") else 0)
    for k in range(3):
        e.init()
        r = e.pa_star(opt)
    print("%s: expanded %d generated %d claimed %d reopen %d, expand kernel %.3f ms over %d launches (%.1f us each): "
          "%.2f G child relaxes/s, %.2f G claims/s; table 2^%d" % (
              name, r.expansions, r.generated, r.table_used, r.reopen, r.expand_ms, r.expand_launches,
              r.expand_ms * 1e3 / max(1, r.expand_launches), r.generated / (r.expand_ms * 1e-3) * 1e-9,
              r.table_used / (r.expand_ms * 1e-3) * 1e-9, r.table_slots.bit_length() - 1), flush=True)
    e.close()
