"""Repeated searches of a workload under each engine mode, with the engine's
verbose summary line (tools/gpu, diagnostics)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences  # noqa: E402

KNOWN = {"syn4x200_s1": 149875, "kinase": 421546, "PF08184": 24450, "test2": 45037, "syn8x100_s3": 703569}
names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["syn4x200_s1"]
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["auto", "batched"]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
for name in names:
    for mode in modes:
        e = Engine(Sequences.from_fasta("tests/golden/%s.fasta" % name)).init()
        for k in range(reps):
            t = time.perf_counter()
            try:
                e.init()
                r = e.pa_star(PAStarOpt(mode=mode, verbose=(k == reps - 1), profile=True))
                e.alignment()
            except Exception as ex:  # noqa: BLE001
                print(name, mode, "error", ex, flush=True)
                break
            wall = time.perf_counter() - t
            print(name, mode, "score", r.score, r.score == KNOWN.get(name), "engine", r.solo, "levels/steps", r.steps,
                  "expanded", r.expansions_all, "%.3f ms step, search %.3f ms, kernel %.3f ms" %
                  (wall * 1e3, r.seconds * 1e3, r.expand_ms), flush=True)
        e.close()
