"""Instance order on the closest-hit walk (tools/inst_order_sim.cpp): BLAS node
visits per ray in TLAS order against nearest-world-box-first (exact with the
tie rule), on the C3 extension rays of 40 rows of frame 7 and on the long
drain path of tools/chainpath_rays.npz.
usage: python tools/inst_order_sim.py   (builds /tmp/inst_order_sim with g++)"""
import os, subprocess, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O


def main():
    exe = os.path.join(tempfile.gettempdir(), "inst_order_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "tools", "inst_order_sim.cpp"), "-o", exe, "-lz"], check=True)
    O.load()
    S = O.OracleScene()
    W = 1280
    (eo, ed), _ = S.record_rays(W, 720, 7, 300 * W, 340 * W, max_ext=1 << 22, max_shadow=1 << 22)
    z = np.load(os.path.join(REPO, "tools", "chainpath_rays.npz"))
    env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"))
    d = tempfile.mkdtemp()
    for name, o, dd in (("C3 extension rays", eo, ed), ("long drain path", z["eo"], z["ed"])):
        fn = os.path.join(d, "r.bin")
        with open(fn, "wb") as f:
            np.array([len(o)], np.uint32).tofile(f)
            np.concatenate([o, dd], axis=1).astype(np.float32).tofile(f)
        out = subprocess.run([exe, fn], capture_output=True, text=True, check=True, env=env).stdout
        print(name + ":", out.strip())


if __name__ == "__main__":
    main()
