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

.ccg_graph <- function(e, n) {
  g <- igraph::make_graph(rbind(e$from, e$to), n = n, directed = FALSE)
  igraph::E(g)$weight <- e$weight
  g
}

#' mean(approxSilhouette(x, l)[, 3], na.rm = TRUE) for every clustering in
#' the list `labs` in one batched call (:447, :518, :664, :811).
ccgSilhouetteMeans <- function(x, labs, eng = ccgEngine()) {
  codes <- vapply(labs, function(l) as.integer(factor(l)), integer(nrow(x)))
  if (!is.matrix(codes)) codes <- matrix(codes, nrow = nrow(x))
  .Call(C_ccg_r_silhouette, eng, x, codes)
}

#' Drop-in for getClustAssignments (R/consensusClust.R:650-692): one exact
#' kNN at max(kNum) (the k = 10, 15 lists are its prefixes), the SNN graphs
#' on the GPU, host clustering in the same (k, res) order, one batched
#' silhouette over all candidate clusterings, the same scoring rules and
#' rank(ties.method = "first") selection, first-copy map-back.
getClustAssignments <- function(pca, clusterFun = "leiden", resRange, kNum, mode = "robust", cellOrder, seed,
                                minSize = 0, ...) {
  eng <- ccgEngine()
  knn <- .Call(C_ccg_r_knn_rows, eng, pca, as.integer(max(kNum)))
  labs <- list()
  for (k in kNum) {
    g <- .ccg_graph(.Call(C_ccg_r_snn, eng, knn, as.integer(k), 0L), nrow(pca))
    for (res in resRange) labs[[length(labs) + 1L]] <- .ccg_cluster_graph(g, clusterFun, res)
  }
  mapback <- function(l) setNames(l, rownames(pca))[match(cellOrder, rownames(pca))]
  if (mode == "robust") {
    s <- ccgSilhouetteMeans(pca, labs, eng)
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
ccgConsensusCore <- function(pca, nboots, bootSize, clusterFun, resRange, kNum, mode, seed, minStability,
                             BPPARAM = BiocParallel::SerialParam(RNGseed = seed)) {
  eng <- ccgEngine()
  if (!inherits(BPPARAM, "SerialParam")) {
    # HIP cannot run in forked workers; the same RNG streams come from a
    # SerialParam with the same seed
    BPPARAM <- BiocParallel::SerialParam(RNGseed = BiocParallel::bpRNGseed(BPPARAM))
  }
  cells <- rownames(pca)
  clustAssignments <- BiocParallel::bplapply(seq_len(nboots), function(boot) {
    tryCatch(getClustAssignments(pca[sample(cells, bootSize * nrow(pca), replace = TRUE), ],
                                 resRange = resRange, kNum = kNum, clusterFun = clusterFun, cellOrder = cells,
                                 mode = mode, seed = seed),
             error = function(e) rep(1, length(cells)))
  }, BPPARAM = BPPARAM)
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
  p <- .Call(C_ccg_r_pca, eng, as.matrix(counts) + 0, as.numeric(sizeFactors), as.integer(genes),
             as.integer(cells), k)
  if (find) k <- max(which(cumsum(p$sdev[1:50]) / sum(p$sdev[1:50]) > pcVar)[1], 5)
  x <- p$x[, seq_len(k), drop = FALSE]
  rownames(x) <- colnames(counts)[cells]
  list(pca = x, sdev = p$sdev, pcNum = k)
}
