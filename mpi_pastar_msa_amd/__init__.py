"""MI355X-native PAStar frontier-expansion engine.

The search hot path of Gabrielcarvfer/mpi_pastar_msa (batched getNeigh, SP g,
HPair h, dedup/relax into the Open/Closed table, owner routing between GPU
shards) runs as hand-written HIP kernels for gfx950 behind the C-ABI in
include/pastar_gpu.h.  This package is the Python host mirror of the
reference interface; see pastar.py.
"""
from .pastar import (ClosedList, Engine, Node, PriorityList, PAStarOpt, SearchResult, Sequences, compute_weights, cost, get_id,
                     lz4_dec, lz4_en, pack_nodes, unpack_nodes,
                     rccl_unique_id, search_many, sharded_search, similarity, ShardGroup)

__all__ = ["ClosedList", "Engine", "Node", "PriorityList", "PAStarOpt", "SearchResult", "Sequences", "compute_weights", "cost", "get_id",
           "lz4_dec", "lz4_en", "pack_nodes", "unpack_nodes",
           "rccl_unique_id", "search_many", "sharded_search", "similarity", "ShardGroup"]
