"""Diagnostic: the sharded search on one GPU (in-process shard group), one
case at a time, each printed before it starts; host waits are bounded by
PASTAR_WAIT_TIMEOUT_S.  python tools/gpu/shard_small.py name:shards[,...]"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import PAStarOpt, Sequences, sharded_search  # noqa: E402

cases = sys.argv[1].split(",") if len(sys.argv) > 1 else ["test2:2"]
for case in cases:
    name, g = case.split(":")
    print("case", name, g, flush=True)
    faulthandler.dump_traceback_later(60, exit=True)
    seqs = Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", name + ".fasta"))
    t0 = time.time()
    res, rows = sharded_search(seqs, int(g), opt=PAStarOpt(batch_nodes=int(os.environ.get("BATCH", "4096")),
                                                           verbose=bool(os.environ.get("VERBOSE"))))
    faulthandler.cancel_dump_traceback_later()
    print("ok", [(r.score, r.steps, r.exchanged, r.host_waits, r.xchg_backlog_steps) for r in res],
          "%.3f s" % (time.time() - t0), flush=True)
