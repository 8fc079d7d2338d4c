# R/ccg.R -- consensusClust's bootstrap hot path on MI355X GPUs through
# libccg.so (src/ccg_r.c, include/ccg.h).  What a maintainer adds to the
# reference package; the NAMESPACE needs
#   useDynLib(consensusClustR, .registration = TRUE, .fixes = "C_")
# R is not installed where this repository is built, so this file is checked
# only structurally there (tests/test_r_glue.py); the same pipeline runs in
# Python as consensusclustr_amd.consensus and is parity-tested on the GPU.
#
# What stays in R exactly as in the reference: sample() and its RNG streams
# (bplapply with SerialParam(RNGseed = seed), R/consensusClust.R:391-400),
# cluster_leiden / cluster_louvain (:656-658, :429-439) and all decisions.
# What moves to the GPU: findKNN, neighborsToSNNGraph, approxSilhouette,
# parDist(customDist), dbscan::kNN(dist), determineHierachy's block means
# and the counting of pairwiseRand.
#
# RNG streams.  In the reference each bootstrap's stream feeds, in order,
# sample() (:394), then for every (k, res) findKNN and cluster_leiden
# (:653-658).  Up to BiocNeighbors 1.x findKNN draws too (its KMKNN index
# runs kmeans); from 1.99 (knncolle) it draws nothing.  The drop-in keeps the
# sequence: pass 1 draws every bootstrap's sample() in its own stream and
# notes the stream's state; the GPU searches the kNN of a batch of
# bootstraps at once (split over the group's GPUs); pass 2 re-enters each
# stream at that state, re-draws sample() (the same indices) and, per
# (k, res), replays findKNN's draws (.ccg_replay_findknn_draws) before
# cluster_leiden -- so Leiden reads the stream where a live reference run
# would.  The replay follows stats::kmeans and BiocNeighbors 1.x buildKmknn
# as published; neither is installed here, so it is unpinned (DESIGN.md).

.ccg <- new.env(parent = emptyenv())

#' The engine: one GPU context, or a device group when several devices are
#' given (the group spreads bootstraps and co-cluster row slabs over GPUs).
ccgEngine <- function(devices = getOption("ccg.devices", 0L)) {
  key <- paste(devices, collapse = ",")
  if (is.null(.ccg$engine) || !identical(.ccg$key, key)) {
    if (!is.null(.ccg$engine)) .Call(C_ccg_r_close, .ccg$engine)
    .ccg$engine <- if (length(devices) > 1) {
      .Call(C_ccg_r_group_open, as.integer(devices))
    } else {
      .Call(C_ccg_r_open, as.integer(devices))
    }
    .ccg$key <- key
  }
  .ccg$engine
}

# bluster's graph step for SNNGraphParam(cluster.fun = ...,
# cluster.args = list(resolution = res)) (:656-658): leiden with the
# modularity objective, louvain with the resolution.
.ccg_cluster_graph <- function(g, clusterFun, res) {
  if (clusterFun == "leiden") {
    igraph::cluster_leiden(g, objective_function = "modularity", resolution_parameter = res)$membership
  } else if (clusterFun == "louvain") {
    igraph::cluster_louvain(g, resolution = res)$membership
  } else {
    stop("clusterFun must be 'leiden' or 'louvain'")
  }
}

# neighborsToSNNGraph's graph: make_graph + weights + simplify(edge.attr.comb
# = "first") as bluster builds it (the engine's edges are already unique,
# i < j, so simplify only fixes igraph's internal edge order)
.ccg_graph <- function(e, n) {
  g <- igraph::make_graph(rbind(e$from, e$to), n = n, directed = FALSE)
  igraph::E(g)$weight <- e$weight
  igraph::simplify(g, edge.attr.comb = "first")
}

# TRUE when the installed BiocNeighbors draws random numbers inside findKNN
# (versions before 1.99: the KMKNN index is built by kmeans on every call).
.ccg_kmknn_draws <- function() {
  if (is.null(.ccg$kmknn)) {
    .ccg$kmknn <- requireNamespace("BiocNeighbors", quietly = TRUE) &&
      utils::packageVersion("BiocNeighbors") < "1.99.0"
  }
  .ccg$kmknn
}

# The random draws of one findKNN(x, k) call under BiocNeighbors 1.x, without
# the index: buildKmknn runs kmeans(x, ceiling(sqrt(nrow(x)))), whose only
# random step picks the initial centres -- sample.int(m, k), and when those
# rows repeat (bootstrap copies) sample.int(nrow(unique(x)), k) again.
# nunique() returns nrow(unique(x)) (computed at most once per bootstrap).
# options(ccg.replay_findknn = ): "replay" (default) replays the draws as
# above; "findKNN" calls the installed BiocNeighbors::findKNN itself for its
# side effects on the stream (exact whatever the installed version does, at
# the cost of the CPU search); "none" draws nothing (BiocNeighbors >= 1.99, or
# when bit-exact Leiden streams are not needed).
.ccg_replay_findknn_draws <- function(x, nunique, k = 10L) {
  mode <- getOption("ccg.replay_findknn", "replay")
  if (identical(mode, "none") || !.ccg_kmknn_draws()) return(invisible(NULL))
  if (identical(mode, "findKNN")) {
    BiocNeighbors::findKNN(x, k = k)
    return(invisible(NULL))
  }
  m <- nrow(x)
  k <- ceiling(sqrt(m))
  if (k >= m) return(invisible(NULL))
  ctr <- x[sample.int(m, k), , drop = FALSE]
  if (any(duplicated(ctr))) sample.int(nunique(), k)
  invisible(NULL)
}

#' mean(approxSilhouette(x, l)[, 3], na.rm = TRUE) for every clustering in
#' the list `labs` in one batched call (:447, :518, :664, :811).
#' cell: for a bootstrap matrix whose rows repeat cells, the 1-based cell of
#' each row (match(rownames(x), unique(rownames(x)))): widths are then
#' computed once per (cell, label) and weighted (ccg_silhouette_cells).
ccgSilhouetteMeans <- function(x, labs, eng = ccgEngine(), cell = NULL) {
  codes <- vapply(labs, function(l) as.integer(factor(l)), integer(nrow(x)))
  if (!is.matrix(codes)) codes <- matrix(codes, nrow = nrow(x))
  if (is.null(cell)) return(.Call(C_ccg_r_silhouette, eng, x, codes))
  .Call(C_ccg_r_silhouette_cells, eng, x, codes, as.integer(cell))
}

#' Drop-in for getClustAssignments (R/consensusClust.R:650-692): one exact
#' kNN at max(kNum) (the k = 10, 15 lists are its prefixes) over the
#' bootstrap's distinct cells, the SNN graphs on the GPU, host clustering in
#' the same (k, res) order with findKNN's RNG draws replayed before each
#' clustering, one batched silhouette over all candidate clusterings, the same
#' scoring rules and rank(ties.method = "first") selection, first-copy
#' map-back.  pca is the bootstrap matrix pca[sample(...), ] with its
#' duplicated row names (:394); knn, when given, is its n x max(kNum)
#' neighbour matrix already searched in a batch (ccgConsensusCore).
getClustAssignments <- function(pca, clusterFun = "leiden", resRange, kNum, mode = "robust", cellOrder, seed,
                                minSize = 0, knn = NULL, ...) {
  eng <- ccgEngine()
  if (is.null(knn)) {
    # rows -> distinct cells (copies share a row name), so the search runs
    # over the distinct cells and expands back to rows
    first <- !duplicated(rownames(pca))
    cell <- match(rownames(pca), rownames(pca)[first])
    knn <- .Call(C_ccg_r_knn_boot, eng, pca[first, , drop = FALSE], matrix(cell, ncol = 1L),
                 as.integer(max(kNum)))[[1L]]
  }
  nu <- NULL
  nunique <- function() {
    if (is.null(nu)) nu <<- nrow(unique(pca))
    nu
  }
  # every graph of kNum from one SNN pass over the max(kNum) lists, at the
  # level of the bootstrap's copies (rows sharing a row name share a class)
  ks <- sort(unique(as.integer(kNum)))
  cell <- match(rownames(pca), unique(rownames(pca)))
  graphs <- .Call(C_ccg_r_snn_multi, eng, knn, ks, 0L, cell)
  labs <- list()
  for (k in kNum) {
    g <- .ccg_graph(graphs[[match(as.integer(k), ks)]], nrow(pca))
    for (res in resRange) {
      .ccg_replay_findknn_draws(pca, nunique, k)  # the reference's findKNN for this (k, res), :656
      labs[[length(labs) + 1L]] <- .ccg_cluster_graph(g, clusterFun, res)
    }
  }
  mapback <- function(l) setNames(l, rownames(pca))[match(cellOrder, rownames(pca))]
  if (mode == "robust") {
    # copies of a cell share a row name: widths once per (cell, label)
    s <- ccgSilhouetteMeans(pca, labs, eng, cell = cell)
    score <- ifelse(s$nclust > 1 & s$minsize > minSize, s$mean, ifelse(s$minsize > minSize, 0, 0.15))
    r <- rank(score, ties.method = "first")
    return(mapback(labs[[which(r == max(r))]]))
  }
  do.call(cbind, lapply(labs, mapback))
}

#' kNN(jaccardDist, k)$id (:425) straight from the assignment matrix.
ccgConsensusKNN <- function(clustAssignments, k, eng = ccgEngine()) {
  storage.mode(clustAssignments) <- "integer"
  .Call(C_ccg_r_consensus_knn, eng, clustAssignments, as.integer(k))
}

#' 1 - parDist(clustAssignments, method = "custom", func = customDist)
#' (:410-421) as a "dist" object -- only for callers that need the matrix
#' itself; the consensus path below never builds it.
ccgJaccardDist <- function(clustAssignments, eng = ccgEngine()) {
  storage.mode(clustAssignments) <- "integer"
  d <- .Call(C_ccg_r_cocluster_dist, eng, clustAssignments)
  structure(d, Size = nrow(clustAssignments), Labels = rownames(clustAssignments), Diag = FALSE, Upper = FALSE,
            method = "custom", class = "dist")
}

#' determineHierachy(as.matrix(jaccardDist), assignments, return = "distance")
#' (:463, :699-721) from the assignment matrix.
ccgClusterDistance <- function(clustAssignments, assignments, eng = ccgEngine()) {
  u <- unique(assignments)
  storage.mode(clustAssignments) <- "integer"
  m <- .Call(C_ccg_r_block_dist, eng, clustAssignments, match(assignments, u), length(u))
  dimnames(m) <- list(u, u)
  m
}

#' determineHierachy(..., return = "dendrogram") on the co-clustering
#' distance (:585, :621): complete-linkage hclust of the cluster distances.
ccgClusterDendrogram <- function(clustAssignments, assignments, eng = ccgEngine()) {
  as.dendrogram(hclust(as.dist(ccgClusterDistance(clustAssignments, assignments, eng)), method = "complete"))
}

#' The stability matrix of :470-481: per bootstrap pairwiseRand(ratio,
#' adjusted) from GPU contingency tables, stacked and averaged as the
#' reference does (NULL where its simplify2array/apply fails).
ccgStabilityMatrix <- function(clustAssignments, finalAssignments, eng = ccgEngine()) {
  lev <- levels(factor(finalAssignments))
  storage.mode(clustAssignments) <- "integer"
  mats <- .Call(C_ccg_r_stability, eng, clustAssignments, match(as.character(finalAssignments), lev),
                length(lev), TRUE)
  tryCatch(apply(simplify2array(mats), 2, rowMeans, na.rm = TRUE), error = function(e) NULL)
}

#' The bootstrap + consensus core of consensusClust (R/consensusClust.R:388-497)
#' over the engine: call it from consensusClust in place of those lines.
#' Returns list(assignments, clustAssignments).
.ccg_serial <- function(BPPARAM) {
  if (inherits(BPPARAM, "SerialParam")) return(BPPARAM)
  # HIP cannot run in forked workers; the same RNG streams come from a
  # SerialParam with the same seed
  BiocParallel::SerialParam(RNGseed = BiocParallel::bpRNGseed(BPPARAM))
}

# pass 1 (:391-394): every bootstrap's sample() in its own stream, and the
# stream's state on entry (the global state is restored after bplapply)
.ccg_draw_bootstraps <- function(cells, n, nboots, BPPARAM) {
  BiocParallel::bplapply(seq_len(nboots), function(boot) {
    st <- get(".Random.seed", envir = globalenv())
    list(idx = match(sample(cells, n, replace = TRUE), cells), seed = st)
  }, BPPARAM = BPPARAM)
}

#' iterate=TRUE, one level at a time (BASELINE config 5): the bootstrap
#' draws of every subcluster PC matrix in `pcas` (each from the forwarded
#' BPPARAM's streams, as the recursive consensusClust call of :562-566 draws
#' them) and their kNN in batched ccg_r_knn_boot_segments calls -- every
#' subcluster's bootstraps in one set of GPU launches.  Pass element s of the
#' result as ccgConsensusCore(pcas[[s]], ..., prefetched = result[[s]]).  A
#' maintainer restructures :546-567 into three lapply passes: PCs of every
#' subcluster, ccgLevelBootstrapKNN, then each subcluster's consensus core.
ccgLevelBootstrapKNN <- function(pcas, nboots, bootSize, kNum, BPPARAM, batch = 32L) {
  eng <- ccgEngine()
  BPPARAM <- .ccg_serial(BPPARAM)
  draws <- lapply(pcas, function(p) {
    d <- .ccg_draw_bootstraps(rownames(p), bootSize * nrow(p), nboots, BPPARAM)
    list(draws = d, knns = vector("list", nboots))
  })
  kmax <- as.integer(max(kNum))
  # a segment needs kmax + 1 distinct cells in every bootstrap: other
  # subclusters are searched by their own ccgConsensusCore (prefetched knns NULL)
  ok <- which(vapply(draws, function(x) {
    all(vapply(x$draws, function(d) length(unique(d$idx)) > kmax, logical(1)))
  }, logical(1)))
  # the library's (segment, cell) keys are 31-bit: segments x stacked cells of
  # one call < 2^31.  Subclusters go into groups that fit with one bootstrap
  # each; each group's batch is cut to fit.
  groups <- list()
  cur <- integer(0)
  for (s in ok) {
    trial <- c(cur, s)
    if (length(trial) * sum(vapply(pcas[trial], nrow, integer(1))) < 2^31) {
      cur <- trial
    } else {
      if (length(cur)) groups[[length(groups) + 1L]] <- cur
      cur <- s
    }
  }
  if (length(cur)) groups[[length(groups) + 1L]] <- cur
  for (grp in groups) {
    ntot <- sum(vapply(pcas[grp], nrow, integer(1)))
    bg <- max(1L, min(batch, floor((2^31 - 1) / (ntot * length(grp)))))
    for (b0 in seq(1L, nboots, by = bg)) {
      bs <- b0:min(nboots, b0 + bg - 1L)
      boots <- lapply(draws[grp], function(x) {
        vapply(x$draws[bs], function(d) d$idx, integer(length(x$draws[[1L]]$idx)))
      })
      boots <- lapply(boots, function(b) if (is.matrix(b)) b else matrix(b, ncol = length(bs)))
      res <- tryCatch(.Call(C_ccg_r_knn_boot_segments, eng, pcas[grp], boots, kmax),
                      error = function(e) NULL)  # on failure each subcluster's core searches its own
      if (!is.null(res)) for (t in seq_along(grp)) draws[[grp[t]]]$knns[bs] <- res[[t]]
    }
  }
  draws
}

ccgConsensusCore <- function(pca, nboots, bootSize, clusterFun, resRange, kNum, mode, seed, minStability,
                             BPPARAM = BiocParallel::SerialParam(RNGseed = seed), batch = 32L,
                             prefetched = NULL) {
  eng <- ccgEngine()
  BPPARAM <- .ccg_serial(BPPARAM)
  cells <- rownames(pca)
  n <- bootSize * nrow(pca)
  draws <- if (is.null(prefetched)) .ccg_draw_bootstraps(cells, n, nboots, BPPARAM) else prefetched$draws
  after <- get0(".Random.seed", envir = globalenv(), inherits = FALSE)
  clustAssignments <- vector("list", nboots)
  for (b0 in seq(1L, nboots, by = batch)) {
    bs <- b0:min(nboots, b0 + batch - 1L)
    # the batch's kNN in one engine call: the distinct-cell search per
    # bootstrap, bootstraps split over the GPUs of a device group (or the
    # level's batched search, ccgLevelBootstrapKNN)
    knns <- if (!is.null(prefetched) && !any(vapply(prefetched$knns[bs], is.null, logical(1)))) {
      prefetched$knns[bs]
    } else {
      boot <- vapply(draws[bs], function(d) d$idx, integer(length(draws[[1L]]$idx)))
      tryCatch(.Call(C_ccg_r_knn_boot, eng, pca, matrix(boot, ncol = length(bs)), as.integer(max(kNum))),
               error = function(e) NULL)
    }
    # pass 2: re-enter each stream, re-draw sample() (the same indices: the
    # stream then stands where the reference's getClustAssignments starts)
    for (t in seq_along(bs)) {
      b <- bs[t]
      assign(".Random.seed", draws[[b]]$seed, envir = globalenv())
      clustAssignments[[b]] <- tryCatch({
        s <- sample(cells, n, replace = TRUE)
        getClustAssignments(pca[s, ], resRange = resRange, kNum = kNum, clusterFun = clusterFun,
                            cellOrder = cells, mode = mode, seed = seed, knn = if (is.null(knns)) NULL else knns[[t]])
      }, error = function(e) rep(1, length(cells)))
    }
  }
  if (is.null(after)) rm(".Random.seed", envir = globalenv()) else assign(".Random.seed", after, envir = globalenv())
  clustAssignments <- do.call(cbind, clustAssignments)
  rownames(clustAssignments) <- cells
  clustAssignments[is.na(clustAssignments)] <- -1
  storage.mode(clustAssignments) <- "integer"

  # consensus graph (:423-441): kNN on the co-clustering distance, SNN rank
  knn <- ccgConsensusKNN(clustAssignments, max(kNum), eng)
  finals <- unlist(lapply(kNum, function(k) {
    g <- .ccg_graph(.Call(C_ccg_r_snn, eng, knn[, seq_len(k), drop = FALSE], as.integer(k), 1L), nrow(pca))
    BiocParallel::bplapply(resRange, function(res) {
      if (clusterFun == "leiden") {
        igraph::cluster_leiden(g, objective_function = "modularity", resolution_parameter = res,
                               beta = 0.01, n_iterations = 2)$membership
      } else {
        igraph::cluster_louvain(g, resolution = res)$membership
      }
    }, BPPARAM = BPPARAM)
  }), recursive = FALSE)

  # consensus resolution (:445-456): silhouettes batched over the candidates
  nu <- vapply(finals, function(f) length(unique(f)), integer(1))
  scored <- which(nu > 1 & nu < nrow(pca) / 10)
  score <- ifelse(nu == nrow(pca), -1, 0.15)
  if (length(scored)) score[scored] <- ccgSilhouetteMeans(pca, finals[scored], eng)$mean
  r <- rank(score, ties.method = "last")
  finalAssignments <- finals[[which(r == max(r))]]

  if (length(unique(finalAssignments)) > 1) {
    # small clusters join their nearest cluster by co-clustering distance (:462-467)
    while (min(table(finalAssignments)) < max(kNum[1], 20)) {
      small <- names(which.min(table(finalAssignments)))
      cd <- ccgClusterDistance(clustAssignments, finalAssignments, eng)
      diag(cd) <- 1
      finalAssignments[finalAssignments == small] <- colnames(cd)[which.min(cd[small, ])]
    }
    # bootstrap stability (:470-496)
    stab <- ccgStabilityMatrix(clustAssignments, finalAssignments, eng)
    if (is.null(stab)) {
      finalAssignments <- rep(1, length(finalAssignments))
    } else {
      diag(stab) <- 1
      dimnames(stab) <- list(unique(finalAssignments), unique(finalAssignments))
      stab[is.na(stab)] <- 1
      while (min(stab) < minStability) {
        m <- as.numeric(which(stab == min(stab), arr.ind = TRUE))
        finalAssignments[finalAssignments == m[2]] <- m[1]
        clustAssignments[clustAssignments == m[2]] <- m[1]
        stab[m[1], m[2]] <- 1
        stab[m[2], m[1]] <- 1
      }
    }
  }
  list(assignments = finalAssignments, clustAssignments = clustAssignments)
}

#' generateNullStatistic's clustering (:796-813) for a list of null PC
#' matrices at once: one batched kNN over all simulations, then per
#' simulation the SNN graphs, host clustering and batched silhouettes.
ccgNullStatistics <- function(pcaNulls, kNum, clusterFun = "leiden", minSize = 5,
                              resRange = c(seq(0.01, 0.3, 0.03), seq(0.3, 2, 0.2))) {
  eng <- ccgEngine()
  ok <- which(!vapply(pcaNulls, function(p) all(is.na(p)), logical(1)))
  out <- numeric(length(pcaNulls))
  if (!length(ok)) return(out)
  knns <- .Call(C_ccg_r_knn_segments, eng, pcaNulls[ok], as.integer(max(kNum)))
  for (t in seq_along(ok)) {
    x <- pcaNulls[[ok[t]]]
    labs <- list()
    for (k in kNum) {
      g <- .ccg_graph(.Call(C_ccg_r_snn, eng, knns[[t]], as.integer(k), 0L), nrow(x))
      for (res in resRange) labs[[length(labs) + 1L]] <- .ccg_cluster_graph(g, clusterFun, res)
    }
    s <- ccgSilhouetteMeans(x, labs, eng)
    score <- ifelse(s$nclust > 1 & s$minsize > minSize, s$mean, ifelse(s$minsize > minSize, 0, 0.15))
    r <- rank(score, ties.method = "first")
    pick <- which(r == max(r))
    out[ok[t]] <- if (s$nclust[pick] < 2) 0 else s$mean[pick]
  }
  out
}

#' The PC matrix of a cell subset (:287, :337-382): log1p(counts / sf) on the
#' variable genes, prcomp_irlba with per-gene centring and scaling -- on the
#' GPU, exact (signs: each component's largest-|loading| gene positive).
#' pcNum = "find" (or > 30) takes 50 components and applies the :356 rule.
ccgSubsetPCs <- function(counts, sizeFactors, genes, cells = seq_len(ncol(counts)), pcNum = "find", pcVar = 0.2) {
  eng <- ccgEngine()
  find <- identical(pcNum, "find") || pcNum > 30
  k <- if (find) 50L else as.integer(pcNum)
  if (is.logical(genes)) genes <- which(genes)
  p <- if (inherits(counts, "dgCMatrix")) {
    # sparse counts stay sparse: the slots go to the GPU, which forms only the
    # selected genes x cells (R/consensusClust.R:273-288)
    .Call(C_ccg_r_pca_csc, eng, as.numeric(counts@x), counts@i, counts@p, nrow(counts),
          as.numeric(sizeFactors), as.integer(genes), as.integer(cells), k)
  } else {
    .Call(C_ccg_r_pca, eng, as.matrix(counts) + 0, as.numeric(sizeFactors), as.integer(genes),
          as.integer(cells), k)
  }
  if (find) k <- max(which(cumsum(p$sdev[1:50]) / sum(p$sdev[1:50]) > pcVar)[1], 5)
  x <- p$x[, seq_len(k), drop = FALSE]
  rownames(x) <- colnames(counts)[cells]
  list(pca = x, sdev = p$sdev, pcNum = k)
}
