"""The C-ABI libraries load and export every symbol their headers declare:
include/surf_hip.h (libsurf_hip.so) and include/surf_mgpu.h (libsurf_mgpu.so)
(no compute calls: this runs without a GPU)."""
import os
import re
import subprocess

import surf_amd

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "surf_hip.h")
MGPU_HEADER = os.path.join(os.path.dirname(HEADER), "surf_mgpu.h")


def declared_functions(header=HEADER):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(surf_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ["surf_create", "surf_upload_scene", "surf_set_camera", "surf_render", "surf_clear_accumulator",
                 "surf_read_accumulator", "surf_finalize_rgba8", "surf_get_stats", "surf_last_error", "surf_destroy"]:
        assert must in fns


def test_library_exports_every_declared_symbol():
    lib = surf_amd.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.surf_abi_version() == 4


def test_exports_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", surf_amd.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for f in declared_functions():
        assert f in syms, f


def test_code_object_targets_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf" if os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf") else "readelf",
                          "-S", surf_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(surf_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_errors_are_returned_not_raised():
    lib = surf_amd.load()
    import ctypes as C
    h = C.c_void_p()
    # bad arguments never abort: they return SURF_ERR_INVALID
    assert lib.surf_create(0, 0, 0, 0, 0, C.byref(h)) == -1
    assert lib.surf_render(None, 1, 0, 0, 1) == -1
    assert lib.surf_scene_build_indoor(b"/nonexistent", 0, C.byref(h)) == -6


def test_mgpu_library_exports_every_declared_symbol():
    lib = surf_amd.load_mgpu()
    fns = declared_functions(MGPU_HEADER)
    assert "surf_mgpu_gather" in fns and "surf_mgpu_create_all" in fns
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", surf_amd.MGPU_LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert all(f in syms for f in fns)
    # the gather is RCCL's (rccl.h:745); the render library itself stays RCCL-free
    deps = subprocess.run(["ldd", surf_amd.MGPU_LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl" in deps
    assert "librccl" not in subprocess.run(["ldd", surf_amd.LIB_PATH], capture_output=True, text=True).stdout


def test_stats_struct_layout_matches_the_header(tmp_path):
    """surf_stats as the C compiler lays it out (include/surf_hip.h) equals the
    ctypes mirror the Python binding passes to surf_get_stats: size and every
    field's offset."""
    import ctypes as C
    fields = [f[0] for f in surf_amd.Stats._fields_]
    src = tmp_path / "layout.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"surf_hip.h\"\nint main(void) {\n"
                   "  printf(\"size %zu\\n\", sizeof(surf_stats));\n" +
                   "".join(f"  printf(\"{f} %zu\\n\", offsetof(surf_stats, {f}));\n" for f in fields) + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    assert int(got["size"]) == C.sizeof(surf_amd.Stats)
    for f in fields:
        assert int(got[f]) == getattr(surf_amd.Stats, f).offset, f
