"""Where the first search's time goes: a fresh context in a fresh process
(code-object loading included), a second fresh context of the same input
in the same process, and warm repeats (tools/gpu, diagnostics)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["PF08184", "syn4x200_s1"]
for name in names:
    seqs = Sequences.from_fasta("tests/golden/%s.fasta" % name)
    for ctx in range(2):
        t0 = time.perf_counter()
        e = Engine(seqs)
        t1 = time.perf_counter()
        e.init()
        e.synchronize()
        t2 = time.perf_counter()
        times = []
        for k in range(4):
            t = time.perf_counter()
            e.init()
            r = e.pa_star(PAStarOpt(profile=True))
            e.alignment()
            e.synchronize()
            times.append(time.perf_counter() - t)
            if k == 0:
                first = r
        print("%s context %d: create %.2f ms, init %.2f ms, searches %s ms (engine %s); table 2^%d used %d "
              "(first search: 2^%d, %d capacity restarts)" % (
                  name, ctx, (t1 - t0) * 1e3, (t2 - t1) * 1e3, " ".join("%.3f" % (x * 1e3) for x in times),
                  "solo" if r.solo else "batched", r.table_slots.bit_length() - 1, r.table_used,
                  first.table_slots.bit_length() - 1, first.capacity_retries), flush=True)
        e.close()
