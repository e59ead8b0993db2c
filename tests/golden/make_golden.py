"""Generates the regression fixtures under tests/golden/ from the CPU oracle.

These are NOT reference outputs (the reference cannot be built here -- see
DESIGN.md): they pin the oracle against unintended changes and give the GPU
tests small vectors that need no oracle run.  Re-run only after a deliberate,
documented oracle change:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402


def main():
    cases = []
    for seed in [0, 1, 2, 3, 1799, 65535, 123456789, 0xFFFFFFF0]:
        init = oracle.init_seed(seed)
        cases.append({"seed": seed, "init": init, "stream": oracle.random_u32_stream(init, 64)})
    with open(os.path.join(HERE, "rng.json"), "w") as f:
        json.dump({"source": "oracle/cpu_ref.cpp seedOf/rndU (surf_math.cpp:31-63)", "cases": cases}, f)
    s = oracle.OracleScene()
    acc, cnt, _ = s.render(32, 24, 2)
    counts = np.array([cnt[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")], np.uint64)
    np.savez_compressed(os.path.join(HERE, "oracle_32x24x2.npz"), acc=acc, counts=counts)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
