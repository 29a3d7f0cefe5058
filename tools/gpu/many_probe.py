"""Throughput of pastar_gpu_search_many: K contexts of one FASTA problem in
one launch.  python tools/gpu/many_probe.py [fasta] [K,...] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import Engine, Sequences, search_many  # noqa: E402

fasta = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "PF08184.fasta")
ks = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,64,256,512,1024").split(",")]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
seqs = Sequences.from_fasta(fasta)
t0 = time.perf_counter()
engines = [Engine(seqs).init() for _ in range(max(ks))]
print("created %d contexts in %.2f s" % (len(engines), time.perf_counter() - t0), flush=True)
for k in ks:
    es = engines[:k]
    search_many(es)
    # the C-ABI call alone (the Python mirror's result objects are built outside the timed calls)
    import ctypes
    from mpi_pastar_msa_amd import _native as nat
    arr = (ctypes.c_void_p * k)(*[e._ctx.value for e in es])
    out = (nat.pastar_result * k)()
    fn = nat.lib().pastar_gpu_search_many
    t0 = time.perf_counter()
    for _ in range(reps):
        rc = fn(arr, k, None, out)
    dt = (time.perf_counter() - t0) / reps
    assert rc == 0
    exp = sum(r.expansions_all for r in out)
    print("K %5d: %.1f us per call, %.2f us per search, %.1f M nodes/s, launch to end %.1f us, kernel %.1f us, "
          "scores ok %s" % (k, dt * 1e6, dt * 1e6 / k, exp / dt / 1e6, out[0].seconds * 1e6,
                            max(r.expand_ms for r in out) * 1e3, len({r.score for r in out}) == 1), flush=True)
