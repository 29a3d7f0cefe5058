import sys, os, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences
for name in ["PF08184", "test2", "test"]:
    e = Engine(Sequences.from_fasta("tests/golden/%s.fasta" % name)).init()
    for k in range(4):
        t = time.perf_counter()
        r = e.pa_star(PAStarOpt(verbose=(k == 3)))
        rows = e.alignment()
        print(name, r.score, r.solo, r.steps, "%.1f us wall, kernel %.1f us" % ((time.perf_counter() - t) * 1e6, r.expand_ms * 1e3),
              "parents", r.expand_parents, "expanded", r.expansions, "generated", r.generated, "nodes", r.table_used,
              "open left", r.open_size, flush=True)
