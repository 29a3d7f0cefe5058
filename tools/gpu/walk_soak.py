"""Random families of similar sequences (a common ancestor with substitutions,
insertions and deletions: long gap-free runs broken by gap columns, ragged
ends) through the batched search and its backtrace walk, against the oracle:
score, rows that spell the sequences, SP cost of the rows.
python tools/gpu/walk_soak.py [problems] [seed]"""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_bind as orc  # noqa: E402
from mpi_pastar_msa_amd import Engine, PAStarOpt  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 150
rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 5)
alphabet = "ACDEFGHIKLMNPQRSTVWY"
longest = skipped = 0
for trial in range(count):
    n = rng.choice([2, 2, 3, 3, 4, 5])
    base = "".join(rng.choice(alphabet) for _ in range(rng.randint(1, 160 if n <= 3 else 70)))
    seqs = []
    for _ in range(n):
        s = []
        for ch in base:
            u = rng.random()
            if u < 0.03:
                continue
            s.append(rng.choice(alphabet) if u < 0.08 else ch)
            if u > 0.97:
                s.append(rng.choice(alphabet))
        if rng.random() < 0.2:
            s = s[rng.randint(0, 10):]
        if rng.random() < 0.2:
            s = s[:max(1, len(s) - rng.randint(0, 10))]
        seqs.append("".join(s) or "A")
    wm = orc.weights(seqs)
    if not np.isfinite(wm).all() or (wm < 0).any():
        # (the reference's weighting turns negative, infinite or NaN on some
        # such families: h is then no lower bound, or no number at all, and
        # no two A* orders need agree)
        skipped += 1
        continue
    o = orc.Oracle(seqs=seqs)
    ref = o.astar()
    try:
        with Engine(seqs).init() as e:
            r = e.pa_star(PAStarOpt(mode="batched", eager=trial % 3 == 0))
            rows = e.alignment()
    except Exception as err:
        print("FAILED", trial, seqs, "oracle score", ref["score"], err, flush=True)
        sys.exit(1)
    ok = (r.score == ref["score"] and [x.replace("-", "") for x in rows] == seqs
          and o.alignment_cost(rows) == ref["score"])
    run = best = 0
    for c in range(len(rows[0])):
        run = run + 1 if all(x[c] != "-" for x in rows) else 0
        best = max(best, run)
    longest = max(longest, best)
    if not ok:
        print("MISMATCH", trial, seqs, r.score, ref["score"], rows, flush=True)
        sys.exit(1)
    if trial % 25 == 24:
        print("%d problems ok, longest gap-free run so far %d columns" % (trial + 1, longest), flush=True)
print("walk_soak_ok %d problems (%d more skipped: a negative or non-finite pair weight), longest gap-free run %d columns"
      % (count - skipped, skipped, longest))
