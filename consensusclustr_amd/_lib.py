"""ctypes binding of libccg.so (the HIP engine behind include/ccg.h).

There is no CPU fallback: if the shared library is missing or a symbol is
absent, loading raises.  Build it with ``python __graft_entry__.py`` or
``make -C consensusclustr_amd/csrc``.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# CCG_LIB_PATH: another build of the library (variant timing); the default is the in-tree build
LIB_PATH = os.environ.get("CCG_LIB_PATH") or os.path.join(_HERE, "libccg.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ccg.h")

# error codes (include/ccg.h)
CCG_OK = 0
CCG_EINVAL = -1
CCG_ENOMEM = -2
CCG_EHIP = -3
CCG_ECAP = -4
CCG_ENAN = -5
CCG_ERANGE = -6
CCG_SNN_NUMBER = 0
CCG_SNN_RANK = 1
CCG_MODE_ROBUST = 0
CCG_MODE_GRANULAR = 1
COCLUSTER_ROW_ALIGN = 128
GROUP_ID_BYTES = 128

_ERRNAMES = {-1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ECAP", -5: "ENAN", -6: "ERANGE"}


class CcgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ccg error {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class ccg_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("flags", ctypes.c_int)]


class ccg_knn_stats(ctypes.Structure):
    _fields_ = [("queries", ctypes.c_int64), ("fallback", ctypes.c_int64)]


_p = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64

SIGNATURES = {
    "ccg_abi_version": (_i, []),
    "ccg_last_error": (ctypes.c_char_p, []),
    "ccg_open": (_i, [_p, _p]),
    "ccg_close": (_i, [_p]),
    "ccg_synchronize": (_i, [_p]),
    "ccg_check_errors": (_i, [_p]),
    "ccg_stream": (_p, [_p]),
    "ccg_ctx_device": (_i, [_p, _p]),
    "ccg_knn_boot": (_i, [_p, _p, _i64, _i, _p, _i64, _i, _i, _p, _p, _p]),
    "ccg_gather_rows_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _p, _p]),
    "ccg_gather_rows_rm_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _p, _p]),
    "ccg_knn_rows_dev": (_i, [_p, _p, _i64, _i, _i, _p, _p, _p, _p]),
    "ccg_knn_boot_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _i, _p, _i, _p, _p, _p, _p]),
    "ccg_knn_boot_hint_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _i, _p, _i, _p, _p, _p, _p, _p]),
    "ccg_knn_table_dev": (_i, [_p, _p, _i64, _i, _i, _p, _p, _p, _p]),
    "ccg_knn_last_fallback": (_i, [_p, _p, _i64, _p]),
    "ccg_snn_multi": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p, _p]),
    "ccg_snn_graphs": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p]),
    "ccg_snn_graph_fetch": (_i, [_p, _i, _p, _p, _p, _i64]),
    "ccg_snn_graphs_cells": (_i, [_p, _p, _i64, _i, _p, _p, _i, _i, _p]),
    "ccg_snn_classes_dev": (_i, [_p, _p, _i64, _i, _p, _p, _i, _p, _p, _p, _p, _p, _p, _i64, _p, _p]),
    "ccg_silhouette_cells": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _i64, _p, _p, _p]),
    "ccg_knn_boot_segments_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _p, _p, _i, _i, _i, _p, _p, _p, _p]),
    "ccg_knn_boot_segments": (_i, [_p, _p, _i64, _i, _p, _i64, _p, _p, _i, _i, _p, _p, _p]),
    "ccg_knn_boot_table_dev": (_i, [_p, _p, _i64, _i, _p, _i64, _i, _p, _i, _p, _p, _i, _p, _p, _p, _p]),
    "ccg_knn_boots_table_dev": (_i, [_p, _i64, _i, _p, _i64, _i, _p, _p, _i, _p, _p, _i, _i, _p, _p, _p, _p]),
    "ccg_knn_segments_dev": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p]),
    "ccg_knn_segments": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p]),
    "ccg_snn": (_i, [_p, _p, _i64, _i, _i, _i, _p, _p, _p, _i64, _p]),
    "ccg_snn_dev": (_i, [_p, _p, _i64, _i, _i, _i, _p, _p, _p, _i64, _p, _p]),
    "ccg_snn_multi_dev": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p, _p, _p]),
    "ccg_snn_rows_dev": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p, _i64, _p, _p]),
    "ccg_snn_reserve": (_i, [_p, _i64]),
    "ccg_silhouette": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p]),
    "ccg_silhouette_dev": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _p, _p, _p, _p]),
    "ccg_silhouette_cells_dev": (_i, [_p, _p, _i64, _i, _p, _i, _i, _p, _i64, _p, _p, _p, _p]),
    "ccg_silhouette_segments_dev": (_i, [_p, _p, _i, _i, _p, _p, _i, _i, _p, _i64, _p, _p, _p, _p]),
    "ccg_select_mapback_dev": (_i, [_p, _i, _p, _p, _i64, _i, _i, _i64, _p, _p, _p, _i, _p, _i, _i64, _p, _p]),
    "ccg_cocluster": (_i, [_p, _p, _i, _i64, _i64, _p, _p, _p]),
    "ccg_cocluster_dev": (_i, [_p, _p, _i, _i64, _i64, _i64, _i64, _p, _p, _p, _p]),
    "ccg_consensus_knn": (_i, [_p, _p, _p, _i64, _i, _p]),
    "ccg_consensus_knn_dev": (_i, [_p, _p, _p, _i64, _i, _p, _p, _p]),
    "ccg_consensus_knn_assign": (_i, [_p, _p, _i, _i64, _i64, _i, _p]),
    "ccg_consensus_knn_assign_dev": (_i, [_p, _p, _i, _i64, _i64, _i, _i64, _i64, _p, _p, _p]),
    "ccg_cluster_block_sums": (_i, [_p, _p, _i, _i64, _i64, _p, _i, _p, _p]),
    "ccg_cluster_block_sums_dev": (_i, [_p, _p, _i, _i64, _i64, _p, _i, _p, _p, _p]),
    "ccg_cluster_block_means": (_i, [_i, _p, _p, _p]),
    "ccg_contingency": (_i, [_p, _p, _i, _i64, _i64, _p, _i, _i, _p]),
    "ccg_contingency_dev": (_i, [_p, _p, _i, _i64, _i64, _p, _i, _i, _p, _p]),
    "ccg_pairwise_rand_ratio": (_i, [_i, _i, _p, _i, _p]),
    "ccg_pca": (_i, [_p, _p, _i64, _i64, _p, _p, _i, _p, _i64, _i, _p, _p]),
    "ccg_pca_dev": (_i, [_p, _p, _i64, _i64, _p, _p, _i, _p, _i64, _i, _p, _p, _p]),
    "ccg_pca_csc": (_i, [_p, _p, _p, _p, _i64, _i64, _p, _p, _i, _p, _i64, _i, _p, _p]),
    "ccg_pca_csc_dev": (_i, [_p, _p, _p, _p, _i64, _i64, _p, _p, _i, _p, _i64, _i, _p, _p, _p]),
    "ccg_row_slabs": (_i, [_i64, _i, _p]),
    "ccg_rect_slabs": (_i, [_i64, _i, _p]),
    "ccg_boot_shard": (_i, [_i64, _i, _i, _p, _p]),
    "ccg_allgather_plan": (_i, [_i, _p, _p, _p, _p, _p]),
    "ccg_group_open": (_i, [_p, _i, _p]),
    "ccg_group_unique_id": (_i, [_p]),
    "ccg_group_open_rank": (_i, [_i, _i, _i, _p, _p]),
    "ccg_group_close": (_i, [_p]),
    "ccg_group_info": (_i, [_p, _p, _p, _p]),
    "ccg_group_ctx": (_i, [_p, _i, _p]),
    "ccg_group_synchronize": (_i, [_p]),
    "ccg_allgather_columns": (_i, [_p, _p, _p, _i64, _i, _p]),
    "ccg_cocluster_sharded_dev": (_i, [_p, _p, _i, _i64, _i64, _p, _p, _p, _p]),
    "ccg_consensus_knn_sharded_dev": (_i, [_p, _p, _i, _i64, _i64, _i, _p, _p]),
    "ccg_group_cocluster": (_i, [_p, _p, _i, _i64, _i64, _p, _p, _p]),
    "ccg_group_consensus_knn_assign": (_i, [_p, _p, _i, _i64, _i64, _i, _p]),
    "ccg_group_knn_boot": (_i, [_p, _p, _i64, _i, _p, _i64, _i, _i, _p, _p, _p]),
    "ccg_sort_pairs_dev": (_i, [_p, _p, _p, _p, _p, _i64, _i, _p]),
    "ccg_scan_i64_dev": (_i, [_p, _p, _p, _i64, _p]),
    "ccg_timing_enable": (_i, [_p, _i]),
    "ccg_host_louvain": (_i, [_i64, _i64, _p, _p, _p, ctypes.c_double, ctypes.c_uint64, _p]),
    "ccg_timing_read": (_i, [_p, _i, _p, _p]),
}
CCG_KT = {"knn_screen": 0, "knn_total": 1, "snn": 2, "silhouette": 3, "cocluster": 4, "host_ring_wait": 100}

_LIB = None


def header_symbols(path=HEADER_PATH):
    """Every function the public header declares."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|void\*)\s+(ccg_\w+)\s*\(", text, re.M)))


def load():
    """Load libccg.so once; raises if it is missing (no CPU fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libccg.so not found at {LIB_PATH}: build it with `python __graft_entry__.py` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:  # one HIP runtime per process: let torch's copy win if torch is used
        import torch  # noqa: F401
    except Exception:
        pass
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)  # AttributeError if the export is missing
        f.restype = res
        f.argtypes = args
    _LIB = lib
    return lib


def check(rc):
    if rc != CCG_OK:
        msg = load().ccg_last_error()
        raise CcgError(rc, msg.decode() if msg else "")
    return rc
