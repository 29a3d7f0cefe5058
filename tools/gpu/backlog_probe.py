import sys
sys.path.insert(0, "/root/repo")
from mpi_pastar_msa_amd import Sequences, PAStarOpt, sharded_search
seqs = Sequences.from_fasta("tests/golden/syn8x100_s3.fasta")
for blk in (8192, 4096):
    for k in range(4):
        res, rows = sharded_search(seqs, 8, opt=PAStarOpt(xchg_lag=1, xchg_block_records=blk))
        print(blk, [r.score for r in res][:2], "steps", res[0].steps, "backlog steps", sum(r.xchg_backlog_steps for r in res), "max", max(r.xchg_backlog_max for r in res), "exchanged", sum(r.exchanged for r in res), flush=True)
