"""Ray-order keys on the lock-step traversal model (tools/lockstep_sim.cpp).

Records the C3 extension rays of 40 rows of frame 7 with the oracle, orders them by
the pool key of the round-2 kernels (start instance x quadrant) and by the heavy-
instance mask x quadrant (poolKey, keyMode 1), and prints the model's visit steps
per 64 rays for each.  Measured on the GPU (profiles/r3_experiments/keys_mask/):
k_extend 186 -> 167 ms per C3 render with the mask key.

usage: python tools/lockstep_sim.py   (builds /tmp/lockstep_sim with g++)
"""
import os, subprocess, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O

def main():
    exe = os.path.join(tempfile.gettempdir(), "lockstep_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "tools", "lockstep_sim.cpp"), "-o", exe, "-lz"], check=True)
    O.load()
    S = O.OracleScene()
    W = 1280
    (eo, ed), _ = S.record_rays(W, 720, 7, 300 * W, 340 * W, max_ext=1 << 21, max_shadow=1 << 21)
    n = len(eo)
    inst = S.trace_closest(eo, ed)[3]
    primary = np.abs(eo[:, 2] + 7.0) < 0.6                    # camera rays (lens disk at z = -7)
    prev = np.concatenate([[0], inst[:-1]]).astype(np.int64)  # a continuation starts on the previous ray's hit
    quad = (eo[:, 0] >= 0) + 2 * (eo[:, 2] >= 0)
    env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"))
    d = tempfile.mkdtemp()
    def write(order, fn):
        with open(fn, "wb") as f:
            np.array([n], np.uint32).tofile(f)
            np.concatenate([eo[order], ed[order]], axis=1).astype(np.float32).tofile(f)
    pos = np.arange(n)
    old = np.where(primary, 63, np.minimum(prev, 14) * 4 + quad)
    write(np.argsort(old * n + pos, kind="stable"), os.path.join(d, "old.bin"))
    subprocess.run([exe, os.path.join(d, "old.bin"), "mask", os.path.join(d, "mask.bin")], check=True, env=env)
    m = np.fromfile(os.path.join(d, "mask.bin"), dtype=np.uint32)
    rays_old = np.argsort(old * n + pos, kind="stable")
    heavy = ((m >> 3) & 7).astype(np.int64)                    # sus0, sus1, lens: the three largest BLASes
    new = np.where(primary[rays_old], 63, heavy * 4 + quad[rays_old])
    write(rays_old[np.argsort(new * n + pos, kind="stable")], os.path.join(d, "mask_order.bin"))
    for name in ("old", "mask_order"):
        out = subprocess.run([exe, os.path.join(d, name + ".bin")], capture_output=True, text=True, check=True, env=env).stdout
        print(name, out.splitlines()[0])

if __name__ == "__main__":
    main()
