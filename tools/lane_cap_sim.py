"""Capped lane walk on the lock-step model (tools/lane_cap_sim.cpp).

Records the C3 extension rays of 40 rows of frame 7 with the oracle, orders them
as k_extend traces them (poolKey keyMode 2: heavy-instance mask descending x
origin quadrant, camera rays last) and prints, per cap on a lane's DFS steps,
the wave steps per 64 rays and how many rays a one-ray-per-wave pass would
have to finish.

usage: python tools/lane_cap_sim.py   (C5=1: the C5 lattice; builds /tmp/lane_cap_sim with g++)
"""
import os, subprocess, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O


def main():
    exe = os.path.join(tempfile.gettempdir(), "lane_cap_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "tools", "lane_cap_sim.cpp"), "-o", exe, "-lz"], check=True)
    lock = os.path.join(tempfile.gettempdir(), "lockstep_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "tools", "lockstep_sim.cpp"), "-o", lock, "-lz"], check=True)
    O.load()
    c5 = os.environ.get("C5") == "1"              # the C5 lattice (SCENE_VARIANT=1)
    S = O.OracleScene(variant=1) if c5 else O.OracleScene()
    W = 1280
    rows = int(os.environ.get("ROWS", "12" if c5 else "40"))
    r0 = 340 if c5 else 300
    (eo, ed), _ = S.record_rays(W, 720, 7, r0 * W, (r0 + rows) * W, max_ext=1 << 22, max_shadow=1 << 22)
    n = len(eo)
    primary = np.abs(eo[:, 2] + 7.0) < 0.6
    quad = (eo[:, 0] >= 0) + 2 * (eo[:, 2] >= 0)
    env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"), SCENE_VARIANT="1" if c5 else "0")
    d = tempfile.mkdtemp()

    def write(order, fn):
        with open(fn, "wb") as f:
            np.array([len(order)], np.uint32).tofile(f)
            np.concatenate([eo[order], ed[order]], axis=1).astype(np.float32).tofile(f)
    if c5:
        key = np.where(primary, 63, quad)         # no heavy instances: the origin quadrant
    else:
        write(np.arange(n), os.path.join(d, "all.bin"))
        subprocess.run([lock, os.path.join(d, "all.bin"), "mask", os.path.join(d, "mask.bin")], check=True, env=env)
        m = np.fromfile(os.path.join(d, "mask.bin"), dtype=np.uint32)
        heavy = ((m >> 3) & 7).astype(np.int64)
        key = np.where(primary, 63, (7 - heavy) * 4 + quad)
    order = np.argsort(key * n + np.arange(n), kind="stable")
    write(order, os.path.join(d, "ordered.bin"))
    print(f"{n} extension rays (rows {r0}..{r0 + rows} of frame 7, {'C5' if c5 else 'C3'}), {'quadrant' if c5 else 'keyMode 2'} order")
    out = subprocess.run([exe, os.path.join(d, "ordered.bin")], capture_output=True, text=True, check=True, env=env).stdout
    print(out, end="")


if __name__ == "__main__":
    main()
