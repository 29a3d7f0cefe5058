"""Find where a sharded search loses the optimum: run it until the score is
wrong, then compare the stored g of every node on the oracle's optimal path.
python tools/gpu/debug_shards.py WORKLOAD SHARDS [attempts] [depth]"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_bind as orc  # noqa: E402
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences, ShardGroup, get_id  # noqa: E402

name, G = sys.argv[1], int(sys.argv[2])
attempts = int(sys.argv[3]) if len(sys.argv) > 3 else 10
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 1
fasta = os.path.join(ROOT, "tests", "golden", name + ".fasta")
o = orc.Oracle(fasta=fasta)
ref = o.astar()
rows = ref["rows"]
n = len(rows)
# optimal path coordinates and g along it
path, pos = [tuple([0] * n)], [0] * n
for col in range(len(rows[0])):
    pos = [pos[k] + (rows[k][col] != "-") for k in range(n)]
    path.append(tuple(pos))
node = o.initial_node()
gs = [node[1]]
for nxt in path[1:]:
    kids = {k[0]: k for k, _ in o.get_neigh(node)}
    node = kids[nxt]
    gs.append(node[1])
print("oracle score", ref["score"], "path", len(path), "g at goal", gs[-1], flush=True)
seqs = Sequences.from_fasta(fasta)
for att in range(attempts):
    group = ShardGroup(G)
    engines = [Engine(seqs, shard_rank=r, group=group) for r in range(G)]
    res = [None] * G
    errs = []

    def run(r):
        try:
            res[r] = engines[r].pa_star(PAStarOpt(depth=depth, profile=bool(int(os.environ.get("PROFILE", "0")))))
        except Exception as e:
            errs.append(e)
    th = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    [t.start() for t in th]
    [t.join() for t in th]
    if errs:
        raise errs[0]
    score = res[0].score
    print("attempt", att, "score", score, "expansions", res[0].expansions_all, flush=True)
    if score != ref["score"]:
        for idx, (pp, g) in enumerate(zip(path, gs)):
            own = get_id(list(pp), G)
            nd = engines[own].closed_lookup(pp)
            gg = nd.g if nd else None
            if gg != g:
                prev = path[idx - 1]
                po = get_id(list(prev), G)
                pn = engines[po].closed_lookup(prev)
                print("first bad node #%d %s owner %d: true g %d, gpu %s; predecessor %s owner %d true g %d gpu %s "
                      "(f %s) mask %s" % (idx, pp, own, g, gg, prev, po, gs[idx - 1], pn.g if pn else None,
                                          pn.f if pn else None, pn.parenti if pn else None))
                print("goal-f bound", score, "pred f true", gs[idx - 1] + (pn.f - pn.g if pn else 0))
                break
        for e in engines:
            e.close()
        group.close()
        break
    for e in engines:
        e.close()
    group.close()
