"""The glibc-exact sinf/cosf/expf the kernels use (csrc/device/surf_math.h)
against this machine's glibc, on a strided sweep of the ranges the path
tracer uses (tools/verify_libm.c does the exhaustive sweep), and through the
library's host build of the same source."""
import ctypes as C
import os
import subprocess

import numpy as np

import surf_amd

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_strided_sweep_matches_glibc(tmp_path):
    exe = tmp_path / "verify_libm"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-x", "c++", "-I", os.path.join(REPO, "surf-path-tracer_amd", "csrc"),
                    os.path.join(REPO, "tools", "verify_libm.c"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "211"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout


def test_library_host_build_matches_glibc():
    lib = surf_amd.load()
    libm = C.CDLL("libm.so.6")
    for name in ("sinf", "cosf", "expf"):
        getattr(libm, name).argtypes = [C.c_float]
        getattr(libm, name).restype = C.c_float
    rng = np.random.default_rng(0)
    th = (rng.random(3000, dtype=np.float32) * np.float32(6.2831855)).tolist()
    ex = (-rng.random(3000, dtype=np.float32) * np.float32(60.0)).tolist()
    assert all(lib.surf_ref_sinf(x) == libm.sinf(x) for x in th)
    assert all(lib.surf_ref_cosf(x) == libm.cosf(x) for x in th)
    assert all(lib.surf_ref_expf(x) == libm.expf(x) for x in ex)
