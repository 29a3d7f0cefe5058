"""ctypes binding of the C-ABI in include/pastar_gpu.h.

The shared library is the product: there is no Python or CPU fallback for
any kernel.  Loading fails loudly when libpastar_gpu.so has not been built.
"""
import ctypes
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpastar_gpu.so")

MAX_SEQ = 16
OK, EINVAL, ENODEV, ENOMEM, EIO, ENOTFOUND, ECOMM, ESTATE, EDEVWAIT = 0, -1, -2, -3, -4, -5, -6, -7, -8

HASH_TYPES = {"FZORDER": 0, "PZORDER": 1, "FSUM": 2, "PSUM": 3}
HASH_NAMES = {0: "Full-Zorder", 1: "Partial-Zorder", 2: "Full-Sum", 3: "Partial-Sum"}


class pastar_problem(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int),
        ("lengths", ctypes.POINTER(ctypes.c_int)),
        ("residues", ctypes.POINTER(ctypes.c_char_p)),
        ("weights", ctypes.POINTER(ctypes.c_int)),
        ("sub", ctypes.POINTER(ctypes.c_int)),
        ("gap_open", ctypes.c_int),
        ("gap_ext", ctypes.c_int),
        ("gap_gap", ctypes.c_int),
        ("hash_type", ctypes.c_int),
        ("hash_shift", ctypes.c_int),
    ]


class pastar_node(ctypes.Structure):
    _fields_ = [
        ("pos", ctypes.c_uint16 * MAX_SEQ),
        ("g", ctypes.c_int32),
        ("f", ctypes.c_int32),
        ("parent_mask", ctypes.c_int32),
    ]


class pastar_search_opts(ctypes.Structure):
    _fields_ = [
        ("batch_nodes", ctypes.c_int64),
        ("batch_min", ctypes.c_int64),
        ("table_slots_log2", ctypes.c_int64),
        ("pool_entries", ctypes.c_int64),
        ("subqueue_entries", ctypes.c_int64),
        ("max_steps", ctypes.c_int64),
        ("band", ctypes.c_int64),
        ("profile", ctypes.c_int32),
        ("verbose", ctypes.c_int32),
        ("no_autogrow", ctypes.c_int32),
        ("eager", ctypes.c_int32),
        ("depth", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("xchg_lag", ctypes.c_int32),
        ("partial", ctypes.c_int32),
        ("xchg_block_records", ctypes.c_int64),
    ]


class pastar_result(ctypes.Structure):
    _fields_ = [
        ("score", ctypes.c_int64),
        ("expansions", ctypes.c_int64),
        ("expansions_all", ctypes.c_int64),
        ("reopen", ctypes.c_int64),
        ("generated", ctypes.c_int64),
        ("open_size", ctypes.c_int64),
        ("closed_size", ctypes.c_int64),
        ("table_used", ctypes.c_int64),
        ("steps", ctypes.c_int64),
        ("exchanged", ctypes.c_int64),
        ("seconds", ctypes.c_double),
        ("expand_ms", ctypes.c_double),
        ("expand_launches", ctypes.c_int64),
        ("expand_parents", ctypes.c_int64),
        ("capacity_retries", ctypes.c_int64),
        ("table_slots", ctypes.c_int64),
        ("pool_entries", ctypes.c_int64),
        ("subqueue_entries", ctypes.c_int64),
        ("graph_replay", ctypes.c_int64),
        ("select_ms", ctypes.c_double),
        ("gap_ms", ctypes.c_double),
        ("solo", ctypes.c_int64),
        ("xchg_backlog_steps", ctypes.c_int64),
        ("xchg_backlog_max", ctypes.c_int64),
        ("host_waits", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}

    def as_tuple(self):
        """Every field in declaration order, in one unpack of the struct's
        bytes (a per-field getattr costs ~10 us per search in Python)."""
        return _RESULT_STRUCT.unpack(bytes(self))


# every pastar_result field is 8 bytes wide: native layout without padding
_RESULT_STRUCT = struct.Struct("=" + "".join("d" if t is ctypes.c_double else "q" for _, t in pastar_result._fields_))
assert _RESULT_STRUCT.size == ctypes.sizeof(pastar_result)


# name -> (restype, argtypes); every symbol include/pastar_gpu.h declares
SIGNATURES = {
    "pastar_last_error": (ctypes.c_char_p, []),
    "pastar_abi_version": (ctypes.c_int, []),
    "pastar_read_fasta": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "pastar_compute_weights": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)]),
    "pastar_cost": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "pastar_owner": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint16), ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int]),
    "pastar_rccl_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "pastar_gpu_create": (ctypes.c_int, [ctypes.POINTER(pastar_problem), ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "pastar_gpu_destroy": (None, [ctypes.c_void_p]),
    "pastar_group_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "pastar_group_destroy": (None, [ctypes.c_void_p]),
    "pastar_gpu_create_grouped": (ctypes.c_int, [ctypes.POINTER(pastar_problem), ctypes.c_int, ctypes.c_void_p,
                                                 ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "pastar_gpu_allreduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                            ctypes.c_int]),
    "pastar_gpu_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "pastar_gpu_build_heuristic": (ctypes.c_int, [ctypes.c_void_p]),
    "pastar_gpu_pair_table": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]),
    "pastar_gpu_weights": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "pastar_gpu_h": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint16), ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int32)]),
    "pastar_gpu_expand": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_node), ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(pastar_node), ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]),
    "pastar_gpu_expand_noalloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_node), ctypes.c_int,
                                                 ctypes.c_int, ctypes.POINTER(pastar_node),
                                                 ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                                 ctypes.POINTER(ctypes.c_int64)]),
    "pastar_gpu_search": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_search_opts),
                                         ctypes.POINTER(pastar_result)]),
    "pastar_gpu_search_many": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                              ctypes.POINTER(pastar_search_opts), ctypes.POINTER(pastar_result)]),
    "pastar_gpu_closed_lookup": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint16),
                                                ctypes.POINTER(pastar_node)]),
    "pastar_gpu_alignment": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]),
    # OpenList / ClosedList
    "pastar_gpu_lists_reset": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_search_opts)]),
    "pastar_gpu_open_enqueue": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_node), ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]),
    "pastar_gpu_open_dequeue": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pastar_node), ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int)]),
    "pastar_gpu_open_highest_priority": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "pastar_gpu_lists_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                             ctypes.POINTER(ctypes.c_int64)]),
    "pastar_gpu_lists_find": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint16),
                                             ctypes.POINTER(pastar_node), ctypes.POINTER(ctypes.c_int)]),
    "pastar_gpu_lists_erase": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint16), ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_int)]),
    "pastar_gpu_lists_reopened": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "pastar_gpu_selftest_queue": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    # MPI-compatible wire frame (host only)
    "pastar_wire_frame_bound": (ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "pastar_wire_frame_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.POINTER(ctypes.c_int64)]),
    "pastar_wire_frame_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.POINTER(ctypes.c_int64)]),
    "pastar_wire_pack_nodes": (ctypes.c_int, [ctypes.POINTER(pastar_node), ctypes.c_int, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "pastar_wire_unpack_nodes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                                ctypes.POINTER(pastar_node), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
}

_lib = None


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (status %d)" % (msg, code))
        self.code = code


def lib():
    """Load libpastar_gpu.so (raises if it is missing: no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libpastar_gpu.so not built (%s); run __graft_entry__.build() or "
                              "python mpi_pastar_msa_amd/build.py" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != OK:
        msg = lib().pastar_last_error()
        raise NativeError(rc, msg.decode() if msg else "error")
    return rc
