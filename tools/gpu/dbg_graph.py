import sys, os
sys_path_root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
__import__("sys").path.insert(0, sys_path_root)
first = sys.argv[1] if len(sys.argv) > 1 else "lib"
if first == "torch":
    import torch  # noqa
from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences, _native
_native.lib()
import torch  # noqa
e = Engine(Sequences.from_fasta("tests/golden/test2.fasta")).init()
r = e.pa_star(PAStarOpt(profile=True, verbose=True))
print(first, "graph", r.graph_replay, r.expand_ms, torch.cuda.is_available(), torch.__version__)
torch.cuda.synchronize()
x = torch.ones(10, device="cuda"); print(float(x.sum()))
