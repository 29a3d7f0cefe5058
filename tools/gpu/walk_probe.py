"""Columns of the alignment the search returns, as parent masks from the
goal back (the order the backtrace walk meets them), and how many memory
round trips the walk's diagonal look-ahead needs for them.
python tools/gpu/walk_probe.py [workload,...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mpi_pastar_msa_amd import Engine, Sequences  # noqa: E402

for w in (sys.argv[1] if len(sys.argv) > 1 else "syn4x200_s1,kinase").split(","):
    seqs = Sequences.from_fasta(os.path.join(ROOT, "tests", "golden", w + ".fasta"))
    e = Engine(seqs).init()
    r = e.pa_star()
    rows = e.alignment()
    n = len(rows)
    full = (1 << n) - 1
    ms = [sum((rows[i][c] != "-") << i for i in range(n)) for c in range(len(rows[0]))][::-1]
    k = rounds = 0
    while k < len(ms):
        rounds += 1
        m0 = ms[k]
        k += 1
        if k >= len(ms):
            break
        m1 = ms[k]
        k += 1
        j = 2 if (m0 & m1) == full else (1 if (m0 ^ m1) == full else 0)
        while j and k < len(ms) and (full if j == 1 else (1 << n) + j - 2) <= 63:
            m = ms[k]
            k += 1
            j = j + 1 if m == full else 0
    print(w, "score", r.score, "columns", len(ms), "without a gap", sum(m == full for m in ms), "round trips", rounds,
          "two steps a trip", (len(ms) + 1) // 2, flush=True)
    print(" ".join("%x" % m for m in ms), flush=True)
