"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this,
and only as the checker or the timed CPU baseline.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
MAX_SEQ = 16
MAX_PAIRS = MAX_SEQ * (MAX_SEQ - 1) // 2


class orc_problem(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int),
        ("len", ctypes.c_int * MAX_SEQ),
        ("seq", ctypes.c_char_p * MAX_SEQ),
        ("weight_f", (ctypes.c_float * MAX_SEQ) * MAX_SEQ),
        ("weight", ctypes.c_int * MAX_PAIRS),
        ("pair_x", ctypes.c_int * MAX_PAIRS),
        ("pair_y", ctypes.c_int * MAX_PAIRS),
        ("npairs", ctypes.c_int),
        ("H", ctypes.POINTER(ctypes.c_int) * MAX_PAIRS),
        ("gap_open", ctypes.c_int),
        ("gap_ext", ctypes.c_int),
        ("gap_gap", ctypes.c_int),
    ]


class orc_node(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_uint16 * MAX_SEQ), ("g", ctypes.c_int32), ("f", ctypes.c_int32),
                ("parenti", ctypes.c_int32)]


class orc_result(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int64), ("expansions", ctypes.c_int64), ("reopen", ctypes.c_int64),
                ("open_size", ctypes.c_int64), ("closed_size", ctypes.c_int64), ("similarity", ctypes.c_double),
                ("seconds", ctypes.c_double), ("aln_len", ctypes.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER(orc_problem)
        L.orc_load_fasta.restype = P
        L.orc_load_fasta.argtypes = [ctypes.c_char_p]
        L.orc_from_seqs.restype = P
        L.orc_from_seqs.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        L.orc_free.argtypes = [P]
        L.orc_init_heuristic.argtypes = [P]
        L.orc_set_gaps.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_h.argtypes = [P, ctypes.POINTER(ctypes.c_uint16)]
        L.orc_get_id.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint16), ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int]
        L.orc_get_neigh.argtypes = [P, ctypes.POINTER(orc_node), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(orc_node), ctypes.POINTER(ctypes.c_int)]
        L.orc_initial_node.argtypes = [P, ctypes.POINTER(orc_node)]
        L.orc_astar.argtypes = [P, ctypes.POINTER(orc_result), ctypes.c_char_p, ctypes.c_int]
        L.orc_pastar_mt.argtypes = [P, ctypes.c_int, ctypes.POINTER(orc_result)]
        L.orc_alignment_cost.restype = ctypes.c_int64
        L.orc_alignment_cost.argtypes = [P, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.orc_cost.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_pairalign.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_weights.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float)]
        _lib = L
    return _lib


class Oracle:
    """One problem instance of the CPU oracle."""

    def __init__(self, fasta=None, seqs=None, gaps=None):
        """gaps: (gap_open, gap_ext, gap_gap) patched over Cost.h:13's 30s."""
        L = lib()
        if fasta is not None:
            self.p = L.orc_load_fasta(str(fasta).encode())
        else:
            arr = (ctypes.c_char_p * len(seqs))(*[s.encode("latin-1") for s in seqs])
            self.p = L.orc_from_seqs(len(seqs), arr)
        if not self.p:
            raise OSError("oracle could not load the input")
        if gaps is not None:
            L.orc_set_gaps(self.p, *gaps)
        if L.orc_init_heuristic(self.p) != 0:
            raise ValueError("oracle init failed")
        pr = self.p.contents
        self.n = pr.n
        self.lengths = [pr.len[i] for i in range(self.n)]
        self.seqs = [pr.seq[i].decode("latin-1") for i in range(self.n)]
        self.weights = [pr.weight[k] for k in range(pr.npairs)]
        self.pairs = [(pr.pair_x[k], pr.pair_y[k]) for k in range(pr.npairs)]

    def close(self):
        if self.p:
            lib().orc_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def pair_table(self, k):
        import numpy as np
        x, y = self.pairs[k]
        cells = (self.lengths[x] + 1) * (self.lengths[y] + 1)
        H = self.p.contents.H[k]
        return np.ctypeslib.as_array(H, shape=(cells,)).reshape(self.lengths[x] + 1, self.lengths[y] + 1).copy()

    def h(self, coord):
        c = (ctypes.c_uint16 * MAX_SEQ)(*coord)
        return lib().orc_h(self.p, c)

    def initial_node(self):
        nd = orc_node()
        lib().orc_initial_node(self.p, ctypes.byref(nd))
        return (tuple(nd.pos[:self.n]), nd.g, nd.f, nd.parenti)

    def get_neigh(self, node, vec_size=1, hash_type=0, shift=12):
        pos, g, f, parenti = node
        nd = orc_node()
        for i, c in enumerate(pos):
            nd.pos[i] = c
        nd.g, nd.f, nd.parenti = g, f, parenti
        cap = 1 << self.n
        out = (orc_node * cap)()
        own = (ctypes.c_int * cap)()
        cnt = lib().orc_get_neigh(self.p, ctypes.byref(nd), vec_size, hash_type, shift, out, own)
        return [((tuple(out[k].pos[:self.n]), out[k].g, out[k].f, out[k].parenti), own[k]) for k in range(cnt)]

    def astar(self):
        """Serial PAStar -t 1: dict with score, expansions, alignment rows, ..."""
        cap = sum(self.lengths) + 1
        buf = ctypes.create_string_buffer(self.n * cap)
        r = orc_result()
        rc = lib().orc_astar(self.p, ctypes.byref(r), buf, cap)
        if rc != 0:
            raise RuntimeError("oracle search failed (%d)" % rc)
        rows = [buf.raw[i * cap:i * cap + r.aln_len].decode("latin-1") for i in range(self.n)]
        return {"score": r.score, "expansions": r.expansions, "reopen": r.reopen, "open_size": r.open_size,
                "closed_size": r.closed_size, "similarity": r.similarity, "seconds": r.seconds, "rows": rows}

    def pastar_mt(self, threads):
        """Multithreaded PAStar -t threads (score exact, expansions vary)."""
        r = orc_result()
        rc = lib().orc_pastar_mt(self.p, int(threads), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError("oracle parallel search failed (%d)" % rc)
        return {"score": r.score, "expansions": r.expansions, "reopen": r.reopen, "seconds": r.seconds}

    def alignment_cost(self, rows):
        cols = len(rows[0])
        stride = cols + 1
        buf = b"".join(r.encode("latin-1") + b"\0" for r in rows)
        return lib().orc_alignment_cost(self.p, buf, stride, cols)


def get_id(coord, size, hash_type=0, shift=12):
    c = (ctypes.c_uint16 * MAX_SEQ)(*coord)
    return lib().orc_get_id(len(coord), c, size, hash_type, shift)


def cost(r, l):
    return lib().orc_cost(r, l)


def pairalign(s1, s2, gap_open=30, gap_ext=30):
    import numpy as np
    out = np.empty((len(s1) + 1) * (len(s2) + 1), dtype=np.int32)
    lib().orc_pairalign(s1.encode("latin-1"), len(s1), s2.encode("latin-1"), len(s2), gap_open, gap_ext,
                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return out.reshape(len(s1) + 1, len(s2) + 1)


def weights(seqs):
    import numpy as np
    n = len(seqs)
    arr = (ctypes.c_char_p * n)(*[s.encode("latin-1") for s in seqs])
    out = (ctypes.c_float * (n * n))()
    lib().orc_weights(n, arr, out)
    return np.array(out[:], dtype=np.float32).reshape(n, n)
