"""Parallel BLAS build vs the oracle's sequential
restatement of BvhBLAS::build (bvh.cpp:255-465).

The product's `surf_bvh_build` must write the reference's index permutation and
node pool exactly, for every thread count: BVH topology fixes traversal order
and therefore which of two equal-depth hits wins.  CPU only (host code)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
import surf_amd

# BvhNode words compared: leftFirst, count, bbMin.xyz, bbMax.xyz (pads skipped)
FIELDS = [0, 1, 4, 5, 6, 8, 9, 10]


def tri_records(v: np.ndarray) -> np.ndarray:
    """(n, 3, 3) vertices as stored (v0, v1, v2) -> (n, 16) Triangle records with
    the reference centroid (v0 + v1 + v2) * 0.333f (mesh.cpp:20)."""
    v = v.astype(np.float32)
    t = np.zeros((v.shape[0], 16), np.float32)
    t[:, 0:3], t[:, 4:7], t[:, 8:11] = v[:, 0], v[:, 1], v[:, 2]
    t[:, 12:15] = ((v[:, 0] + v[:, 1]) + v[:, 2]) * np.float32(0.333)
    return t


def soup(n: int, seed: int, spread: float = 10.0, size: float = 0.05) -> np.ndarray:
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (n, 1, 3))
    return tri_records(c + rng.normal(0.0, size, (n, 3, 3)))


def check(tris: np.ndarray, threads=(1, 2, 8)):
    oi, on = oracle.bvh_build(tris)
    for th in threads:
        pi, pn = surf_amd.bvh_build(tris, th)
        assert pn.shape == on.shape, f"threads={th}: nodesUsed {pn.shape[0]} != {on.shape[0]}"
        assert np.array_equal(pi, oi), f"threads={th}: index permutation differs"
        assert np.array_equal(pn.view(np.uint32)[:, FIELDS], on.view(np.uint32)[:, FIELDS]), f"threads={th}: nodes differ"


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000])
def test_small_soups(n):
    check(soup(n, n))


@pytest.mark.parametrize("n,seed", [(40_000, 1), (150_000, 2), (400_000, 3)])
def test_parallel_soups(n, seed):
    check(soup(n, seed))


def test_clustered_and_ragged():
    """Clusters of very different sizes: one-sided splits and deep chains."""
    rng = np.random.default_rng(7)
    parts = [soup(60_000, 11, spread=0.01, size=1e-4), soup(30_000, 12, spread=50.0, size=0.5),
             soup(5, 13, spread=1e4, size=1.0)]
    tris = np.concatenate(parts)
    check(tris[rng.permutation(len(tris))])


def test_identical_centroids():
    """All keys equal on every axis: the root stays one leaf (findSplitPlane
    skips every axis, bvh.cpp:305)."""
    one = soup(1, 5)
    check(np.repeat(one, 50_000, axis=0))


def test_flat_plane():
    """Zero extent on one axis (lo == hi skips it), many equal keys."""
    rng = np.random.default_rng(9)
    g = rng.integers(0, 300, (80_000, 1, 2)).astype(np.float32) * np.float32(0.1)
    v = np.zeros((80_000, 3, 3), np.float32)
    v[:, :, 0:2] = g + rng.uniform(0, 0.1, (80_000, 3, 2)).astype(np.float32)
    check(tri_records(v))


def test_non_finite_falls_back_to_sequential():
    """A NaN vertex makes min/max order-dependent: the builder must then run the
    reference's sequential order, so the result still matches."""
    t = soup(50_000, 21)
    t[123, 0] = np.nan
    t[777, 9] = np.inf
    check(t, threads=(8,))

