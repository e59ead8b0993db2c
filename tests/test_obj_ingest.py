"""OBJ ingestion at scale: the product's parallel
chunked parser against the oracle's front-to-back tinyobj restatement
(mesh.cpp:69-154).  Triangles and TriExtensions must be identical, for every
thread count, on the bundled assets and on large generated files that use
every index form (v, v/t, v//n, v/t/n; 1-based and negative), quads, n-gons,
CRLF line ends, comments and gzip.  CPU only (host code)."""
from __future__ import annotations

import gzip
import os

import numpy as np
import pytest

import oracle
import surf_amd

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(REPO, "assets")
TRI_WORDS = [0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14]
EXT_WORDS = [0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, 15, 16, 17]


def check(path, threads=(1, 3, 8)):
    ot, ox = oracle.obj_load(path)
    for th in threads:
        pt, px = surf_amd.obj_load(path, th)
        assert pt.shape == ot.shape, f"threads={th}: {pt.shape[0]} vs {ot.shape[0]} triangles"
        assert np.array_equal(pt.view(np.uint32)[:, TRI_WORDS], ot.view(np.uint32)[:, TRI_WORDS]), f"threads={th}: triangles"
        assert np.array_equal(px.view(np.uint32)[:, EXT_WORDS], ox.view(np.uint32)[:, EXT_WORDS]), f"threads={th}: extensions"
    return len(ot)


@pytest.mark.parametrize("name", ["susanne", "cube", "lens", "plane"])
def test_bundled_assets(name):
    path = os.path.join(ASSETS, name + ".obj")
    if not os.path.exists(path):
        path += ".gz"
    assert check(path) > 0


def write_lattice(path, copies, seed=0, crlf=False):
    """`copies` jittered copies of a 12-face box-like solid per cell, with every
    face/index form; vertices written with 9 significant digits."""
    rng = np.random.default_rng(seed)
    nl = "\r\n" if crlf else "\n"
    lines = ["# generated lattice", "o lattice"]
    nv = nt = nn = 0
    for c in range(copies):
        off = np.array([c % 17, (c // 17) % 13, c // 221], np.float64) * 2.5
        v = off + rng.uniform(-1, 1, (8, 3))
        for p in v:
            lines.append("v %.9g %.9g %.9g" % tuple(p))
        for _ in range(4):
            lines.append("vt %.6g %.6g" % tuple(rng.uniform(0, 1, 2)))
        for _ in range(3):
            lines.append("vn %.6g %.6g %.6g" % tuple(rng.normal(size=3)))
        b, t, n = nv + 1, nt + 1, nn + 1
        form = c % 5
        if form == 0:      # triangles, v/t/n, 1-based
            lines += [f"f {b}/{t}/{n} {b + 1}/{t + 1}/{n + 1} {b + 2}/{t + 2}/{n + 2}",
                      f"f {b + 3}/{t + 3}/{n} {b + 4}/{t}/{n + 1} {b + 5}/{t + 1}/{n + 2}"]
        elif form == 1:    # quads, v//n, negative
            lines += ["f -8//-3 -7//-2 -6//-1 -5//-3", "f -4//-1 -3//-2 -2//-3 -1//-1"]
        elif form == 2:    # pentagon + hexagon fans, v/t
            lines += [f"f {b}/{t} {b + 1}/{t + 1} {b + 2}/{t + 2} {b + 3}/{t + 3} {b + 4}/{t}",
                      f"f {b + 2}/{t} {b + 3}/{t + 1} {b + 4}/{t + 2} {b + 5}/{t + 3} {b + 6}/{t} {b + 7}/{t + 1}"]
        elif form == 3:    # plain v, tabs and extra spaces, degenerate 2-corner face skipped
            lines += [f"f\t{b} {b + 1}   {b + 2}", f"f {b + 3} {b + 4}", "  f  -1 -2 -3 -4"]
        else:              # quad with a tie-prone square layout, mixed forms
            lines += [f"f {b}/{t}/{n} {b + 1}//{n} {b + 2}/{t + 1} {b + 3}", "# comment f 1 2 3"]
        nv, nt, nn = nv + 8, nt + 4, nn + 3
    text = nl.join(lines) + nl
    if path.endswith(".gz"):
        with gzip.open(path, "wt", newline="") as f:
            f.write(text)
    else:
        with open(path, "w", newline="") as f:
            f.write(text)


@pytest.mark.parametrize("copies,suffix,crlf", [(7, ".obj", False), (40_000, ".obj", False), (25_000, ".obj", True),
                                                (30_000, ".obj.gz", False)])
def test_generated_large(tmp_path, copies, suffix, crlf):
    path = str(tmp_path / f"lattice{suffix}")
    write_lattice(path, copies, seed=copies, crlf=crlf)
    assert check(path) > copies


def test_out_of_range_index_raises(tmp_path):
    path = str(tmp_path / "bad.obj")
    with open(path, "w") as f:
        f.write("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n")
    with pytest.raises(surf_amd.SurfError):
        surf_amd.obj_load(path, 4)
