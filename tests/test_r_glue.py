"""Structural checks of the R binding (src/ccg_r.c + R/ccg.R), which cannot be
run here (no R): the glue type-checks against include/ccg.h and an R-API
declaration stub, every libccg function it calls is declared in ccg.h, every
.Call entry point is registered with its true arity, and every C_ symbol the
R code uses is registered with the number of arguments it passes."""
import os
import re
import shutil
import subprocess

import pytest

from consensusclustr_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "src", "ccg_r.c")
RCODE = os.path.join(ROOT, "R", "ccg.R")


def _glue():
    return open(GLUE).read()


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_glue_type_checks_against_header():
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Werror", "-Wno-cast-function-type",
                        "-I", os.path.join(ROOT, "tests", "r_stub"), "-I", os.path.join(ROOT, "include"), GLUE],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_glue_calls_only_declared_entry_points():
    declared = set(_lib.header_symbols())
    called = set(re.findall(r"\b(ccg_(?!r_)\w+)\s*\(", _glue()))
    called -= {"ccg_ctx", "ccg_group", "ccg_config", "ccg_knn_stats"}
    assert called, "no libccg calls found"
    assert called <= declared, sorted(called - declared)


def _registered():
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r'\{"(ccg_r_\w+)",\s*\(DL_FUNC\)&\1,\s*(\d+)\}', _glue())}


def test_every_call_entry_point_is_registered_with_its_arity():
    text = _glue()
    defs = {m.group(1): m.group(2) for m in re.finditer(r"^SEXP (ccg_r_\w+)\(([^)]*)\)", text, re.M)}
    reg = _registered()
    assert set(defs) == set(reg)
    for name, args in defs.items():
        n = 0 if args.strip() in ("", "void") else args.count(",") + 1
        assert reg[name] == n, name


def test_r_code_uses_registered_symbols_with_matching_arity():
    reg = _registered()
    code = open(RCODE).read()
    calls = re.findall(r"\.Call\(C_(ccg_r_\w+)((?:[^()]|\([^()]*(?:\([^()]*\)[^()]*)*\))*)\)", code)
    assert calls
    for name, rest in calls:
        assert name in reg, name
        depth, nargs = 0, 0
        for ch in rest:
            if ch in "([":
                depth += 1
            elif ch in ")]":
                depth -= 1
            elif ch == "," and depth == 0:
                nargs += 1
        assert nargs == reg[name], (name, nargs, reg[name])


def test_r_code_covers_the_replaced_seams():
    code = open(RCODE).read()
    for fn in ("getClustAssignments", "ccgConsensusCore", "ccgConsensusKNN", "ccgJaccardDist",
               "ccgClusterDistance", "ccgStabilityMatrix", "ccgSilhouetteMeans", "ccgNullStatistics",
               "ccgSubsetPCs"):
        assert re.search(rf"^{fn} <- function\(", code, re.M), fn


def test_r_bootstrap_loop_is_batched_and_keeps_the_rng_sequence():
    """ccgConsensusCore draws every bootstrap first (one bplapply pass, the
    stream state kept), searches the kNN of a batch of bootstraps in one
    ccg_r_knn_boot call (a group splits it over GPUs), then re-enters each
    stream; getClustAssignments replays findKNN's draws before every
    clustering and builds bluster's simplified graph (R/consensusClust.R:391-400,
    :650-692)."""
    code = open(RCODE).read()
    core = code[code.index("ccgConsensusCore <- function("):code.index("ccgNullStatistics <- function(")]
    draw = code[code.index(".ccg_draw_bootstraps <- function("):code.index("ccgLevelBootstrapKNN <- function(")]
    assert draw.count("bplapply(seq_len(nboots)") == 1 and ".Random.seed" in draw
    assert ".ccg_draw_bootstraps(cells, n, nboots, BPPARAM)" in core
    assert ".Random.seed" in core and "draws[[b]]$seed" in core
    assert "C_ccg_r_knn_boot" in core and "knn = if (is.null(knns))" in core
    gca = code[code.index("getClustAssignments <- function("):code.index("#' kNN(jaccardDist, k)$id")]
    assert "C_ccg_r_knn_boot" in gca and "C_ccg_r_knn_rows" not in code
    loop = gca[gca.index("for (res in resRange)"):]
    assert loop.index(".ccg_replay_findknn_draws") < loop.index(".ccg_cluster_graph")
    assert 'simplify(g, edge.attr.comb = "first")' in code
    assert 'packageVersion("BiocNeighbors") < "1.99.0"' in code


def test_r_getclustassignments_runs_the_bench_kernels():
    """The R drop-in reaches the kernels bench.py times: every kNum graph from
    ONE SNN rows pass (ccg_snn_graphs -- the kernels of ccg_snn_rows_dev --
    decoded per graph on the host by ccg_snn_graph_fetch, no device emit)
    and the silhouettes over the bootstrap's distinct cells
    (ccg_silhouette_cells, cell = the row-name match)."""
    code = open(RCODE).read()
    gca = code[code.index("getClustAssignments <- function("):code.index("#' kNN(jaccardDist, k)$id")]
    assert "C_ccg_r_snn_multi" in gca and "C_ccg_r_snn," not in gca
    assert "cell <- match(rownames(pca), unique(rownames(pca)))" in gca and "cell = cell" in gca
    assert "C_ccg_r_snn_multi, eng, knn, ks, 0L, cell)" in gca
    sil = code[code.index("ccgSilhouetteMeans <- function("):code.index("#' Drop-in for getClustAssignments")]
    assert "C_ccg_r_silhouette_cells" in sil
    glue = _glue()
    assert re.search(r"ccg_silhouette_cells\(ctx,", glue) and re.search(r"ccg_snn_graphs_cells\(ctx,", glue)
    assert "ccg_snn_graph_fetch(ctx, t," in glue and "ccg_snn_multi(" not in glue
    # any number of k values: the glue chunks them 4 per device pass
    multi = glue[glue.index("SEXP ccg_r_snn_multi("):]
    assert "c0 += 4" in multi and "nk > 4" not in multi


def test_r_level_batching_uses_the_segment_search():
    """iterate=TRUE levels (BASELINE config 5): ccgLevelBootstrapKNN draws
    each subcluster's bootstraps from the forwarded BPPARAM streams and
    searches all of them through ccg_r_knn_boot_segments; ccgConsensusCore
    consumes them (prefetched) without drawing again."""
    code = open(RCODE).read()
    lvl = code[code.index("ccgLevelBootstrapKNN <- function("):code.index("ccgConsensusCore <- function(")]
    assert "C_ccg_r_knn_boot_segments" in lvl and ".ccg_draw_bootstraps(" in lvl
    # subclusters with a bootstrap of <= kmax distinct cells stay out of the
    # segment call, and segments x stacked cells stay below 2^31 per call
    assert "length(unique(d$idx)) > kmax" in lvl and "2^31" in lvl and "pcas[grp]" in lvl
    core = code[code.index("ccgConsensusCore <- function("):code.index("ccgNullStatistics <- function(")]
    assert "prefetched$draws" in core and "prefetched$knns[bs]" in core
    assert "ccg_knn_boot_segments(ctx, cells, Ntot, d, idx, n, off, NULL" in _glue()


def test_r_findknn_replay_is_optional_and_skipped_when_k_covers_the_rows():
    """The BiocNeighbors 1.x draw replay (parity unpinned) sits behind
    options(ccg.replay_findknn): "replay" (default), "findKNN" (the installed
    findKNN for its side effects), "none"; kmeans is not run (no draw) when
    ceiling(sqrt(m)) >= m."""
    code = open(RCODE).read()
    rep = code[code.index(".ccg_replay_findknn_draws <- function("):code.index("#' mean(approxSilhouette")]
    assert 'getOption("ccg.replay_findknn", "replay")' in rep
    assert 'identical(mode, "none")' in rep and "BiocNeighbors::findKNN(x, k = k)" in rep
    assert rep.index("if (k >= m) return(invisible(NULL))") < rep.index("sample.int(m, k)")
