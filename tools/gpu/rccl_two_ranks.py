"""Probe: does RCCL accept two ranks on ONE device on this box?

Two processes, each with a context on device 0, joined by one RCCL
communicator of world size 2.  If RCCL refuses (a duplicate-GPU check) the
child prints the error and exits; each child runs under its own time limit.
Usage: python tools/gpu/rccl_two_ranks.py [fasta]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CHILD = r"""
import sys, os
sys.path.insert(0, %r)
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences
rank = int(sys.argv[1]); idfile = sys.argv[2]; fasta = sys.argv[3]
rid = open(idfile, 'rb').read()
print('rank', rank, 'creating', flush=True)
e = Engine(Sequences.from_fasta(fasta), device=0, n_shards=2, shard_rank=rank, rccl_id=rid).init()
print('rank', rank, 'created', flush=True)
r = e.pa_star(PAStarOpt())
print('rank', rank, 'score', r.score, 'steps', r.steps, 'exchanged', r.exchanged, 'seconds', r.seconds, flush=True)
rows = e.alignment()
print('rank', rank, 'cols', len(rows[0]), flush=True)
e.close()
""" % ROOT


def main():
    from mpi_pastar_msa_amd import rccl_unique_id
    fasta = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "test2.fasta")
    idfile = "/tmp/rccl_id.bin"
    with open(idfile, "wb") as f:
        f.write(rccl_unique_id())
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-u", "-c", CHILD, str(r), idfile, fasta], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    rc = 0
    for r, p in enumerate(procs):
        try:
            out, _ = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
            out += "\n[timed out]"
        print("---- rank %d (exit %s)\n%s" % (r, p.returncode, out[-3000:]), flush=True)
        rc |= p.returncode or 0
    return rc


if __name__ == "__main__":
    sys.exit(main())
