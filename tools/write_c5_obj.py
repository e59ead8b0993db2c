"""Writes the C5 lattice (648 Suzannes at translate(-8+2i,
-0.4+1.2j, -4+1.5k) * scale(0.5)) as one OBJ file, for timing OBJ ingestion at
scale (row f4): python tools/write_c5_obj.py OUT.obj[.gz]"""
import gzip
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(REPO, "assets", "susanne.obj")
opener = gzip.open if not os.path.exists(src) else open
if not os.path.exists(src):
    src += ".gz"
v, vt, vn, faces = [], [], [], []
with opener(src, "rt") as f:
    for line in f:
        if line.startswith("v "):
            v.append([float(x) for x in line.split()[1:4]])
        elif line.startswith("vt "):
            vt.append(line)
        elif line.startswith("vn "):
            vn.append(line)
        elif line.startswith("f "):
            faces.append(line.split()[1:])
v = np.array(v)
out = sys.argv[1]
w = (gzip.open if out.endswith(".gz") else open)(out, "wt")
w.write("# C5 lattice: 648 Suzannes\n")
w.writelines(vt)
w.writelines(vn)
nv = len(v)
for i in range(9):
    for j in range(8):
        for k in range(9):
            p = v * 0.5 + np.array([-8 + 2 * i, -0.4 + 1.2 * j, -4 + 1.5 * k])
            w.write("".join("v %.9g %.9g %.9g\n" % tuple(q) for q in p))
            # faces reference this copy's vertices with negative indices; uv/normal shared (1-based)
            for fc in faces:
                parts = []
                for c in fc:
                    a = c.split("/")
                    a[0] = str(int(a[0]) - nv - 1)
                    parts.append("/".join(a))
                w.write("f " + " ".join(parts) + "\n")
w.close()
