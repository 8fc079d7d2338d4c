"""consensusclustr_amd -- MI355X-native engine for consensusClust's bootstrap hot path.

The compute lives in libccg.so (hand-written HIP for gfx950, C ABI in
include/ccg.h).  This package is the host-side mirror of the reference's
interface for that path (R/consensusClust.R) plus the multi-GPU sharding.
Importing it does not touch the GPU; the library is loaded on first use and
raises if it is missing (there is no CPU fallback).
"""
from ._lib import CcgError, load  # noqa: F401
from .engine import Engine  # noqa: F401
from .consensus import (  # noqa: F401
    K_NUM, RES_RANGE, assignment_matrix, bootstrap_indices, consensus_choice, consensus_cluster,
    getClustAssignments, mapback, robust_choice, robust_scores)
from .sharding import boot_shard, row_slabs  # noqa: F401
from .pipeline import consensusClust  # noqa: F401

__all__ = ["Engine", "CcgError", "load", "getClustAssignments", "consensus_cluster", "bootstrap_indices",
           "mapback", "assignment_matrix", "robust_choice", "consensus_choice", "robust_scores", "row_slabs",
           "boot_shard", "K_NUM", "RES_RANGE", "consensusClust"]
