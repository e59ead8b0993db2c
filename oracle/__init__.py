"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  Parity status:
UNPINNED against a run of the reference (see oracle/cpu_ref.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
BENCH_BIN = os.path.join(HERE, "cpu_ref_bench")
ASSETS_DIR = os.path.join(os.path.dirname(HERE), "assets")


def build():
    subprocess.run(["make", "-s", "-C", HERE, "-j4"], check=True)


class Counters(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("n_ext", C.c_uint64), ("n_hit", C.c_uint64), ("n_cont", C.c_uint64),
                ("n_shadow", C.c_uint64), ("n_acc", C.c_uint64), ("n_unocc", C.c_uint64), ("max_segments", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P, U32, I32, F, D = C.c_void_p, C.c_uint32, C.c_int, C.c_float, C.c_double
    sig = {
        "orc_scene_create": ([C.c_char_p, I32], P), "orc_scene_destroy": ([P], None),
        "orc_scene_mesh_tris": ([P, P, I32], I32),
        "orc_scene_instance_count": ([P], U32), "orc_scene_light_count": ([P], U32),
        "orc_scene_set_camera": ([P, U32, U32], None), "orc_camera_ubo": ([P, P], None),
        "orc_scene_export": ([P, I32, P], C.c_uint64),
        "orc_render": ([P, U32, U32, U32, U32, U32, U32, U32, I32, P, C.POINTER(Counters)], D),
        "orc_render_spp": ([P, U32, U32, U32, U32, U32, U32, U32, U32, I32, P, C.POINTER(Counters)], D),
        "orc_trace_closest": ([P, U32, P, P, P, P, P, P, P], None),
        "orc_trace_any": ([P, U32, P, P, P, P], None),
        "orc_trace_brute": ([P, U32, P, P, P, P, P], None),
        "orc_trace_visits": ([P, U32, P, P, P, P], None),
        "orc_path_lengths": ([P, U32, U32, U32, P], None),
        "orc_scene_update": ([P, F], None),
        "orc_record_rays": ([P, U32, U32, U32, U32, U32, U32, P, P, P, U32, P, P, P, P], None),
        "orc_bvh_depths": ([P, C.POINTER(U32), C.POINTER(U32)], None),
        "orc_init_seed": ([U32], U32), "orc_random_u32": ([C.POINTER(U32)], U32),
        "orc_random_f32": ([C.POINTER(U32)], F),
        "orc_finalize_rgba8": ([P, U32, F, P], None),
        "orc_set_zero_cutoff": ([I32], None),
        "orc_bvh_build": ([P, U32, P, P], U32),
        "orc_obj_load": ([C.c_char_p, P, P, C.c_uint64], C.c_long),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data


EXPORT_ORDER = ["triangles", "tri_ext", "blas_indices", "blas_nodes", "materials", "instances",
                "tlas_indices", "tlas_nodes", "lights", "background"]


class OracleScene:
    def __init__(self, assets_dir: str = ASSETS_DIR, variant: int = 0):
        lib = load()
        self._h = lib.orc_scene_create(assets_dir.encode(), variant)
        if not self._h:
            raise RuntimeError(f"oracle could not load the scene from {assets_dir}")

    def mesh_tris(self):
        out = np.zeros(8, np.uint32)
        n = load().orc_scene_mesh_tris(self._h, _p(out), 8)
        return [int(x) for x in out[:n]]

    def instance_count(self):
        return load().orc_scene_instance_count(self._h)

    def light_count(self):
        return load().orc_scene_light_count(self._h)

    def camera_ubo(self, width, height) -> bytes:
        load().orc_scene_set_camera(self._h, width, height)
        buf = (C.c_uint8 * 128)()
        load().orc_camera_ubo(self._h, buf)
        return bytes(buf)

    def export(self) -> dict[str, bytes]:
        out = {}
        for i, k in enumerate(EXPORT_ORDER):
            n = load().orc_scene_export(self._h, i, None)
            buf = (C.c_uint8 * max(int(n), 1))()
            load().orc_scene_export(self._h, i, buf)
            out[k] = bytes(buf)[: int(n)]
        return out

    def render(self, width, height, frames, first_frame=0, rows=None, max_segments=0, threads=0, spp=1):
        """`frames` frames of `spp` samples per pixel (Renderer::render with
        samplesPerFrame = spp); first_frame is the sample count before the first
        frame (the accumulator's totalSamples; the frame index when spp = 1)."""
        r0, r1 = (0, height) if rows is None else rows
        acc = np.zeros((r1 - r0, width, 4), np.float32)
        cnt = Counters()
        secs = load().orc_render_spp(self._h, width, height, r0, r1, first_frame, frames, spp, max_segments, threads,
                                     _p(acc), C.byref(cnt))
        return acc, cnt.as_dict(), secs

    def trace_closest(self, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        inst, prim = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        load().orc_trace_closest(self._h, n, _p(o), _p(d), _p(t), _p(u), _p(v), _p(inst), _p(prim))
        return t, u, v, inst, prim

    def trace_any(self, o, d, tmax):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        tmax = np.ascontiguousarray(tmax, np.float32)
        occ = np.zeros(len(o), np.uint8)
        load().orc_trace_any(self._h, len(o), _p(o), _p(d), _p(tmax), _p(occ))
        return occ

    def trace_brute(self, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        t = np.zeros(n, np.float32)
        inst, prim = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        load().orc_trace_brute(self._h, n, _p(o), _p(d), _p(t), _p(inst), _p(prim))
        return t, inst, prim

    def trace_visits(self, o, d):
        """Per ray and instance: BLAS node visits and triangle tests of the closest-hit traversal."""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        ni = self.instance_count()
        nodes, tris = np.zeros((len(o), ni), np.uint32), np.zeros((len(o), ni), np.uint32)
        load().orc_trace_visits(self._h, len(o), _p(o), _p(d), _p(nodes), _p(tris))
        return nodes, tris

    def update(self, dt: float):
        """GPUScene::update: rotate instance 3 by dt radians about +y, refit the TLAS."""
        load().orc_scene_update(self._h, dt)

    def path_lengths(self, width, height, frame):
        """Extension rays per pixel path of one frame (diagnostics)."""
        out = np.zeros(width * height, np.uint32)
        load().orc_path_lengths(self._h, width, height, frame, _p(out))
        return out.reshape(height, width)

    def record_rays(self, width, height, frame, pix_begin, pix_end, max_ext=1 << 20, max_shadow=1 << 20):
        eo, ed = np.zeros((max_ext, 3), np.float32), np.zeros((max_ext, 3), np.float32)
        so, sd = np.zeros((max_shadow, 3), np.float32), np.zeros((max_shadow, 3), np.float32)
        st = np.zeros(max_shadow, np.float32)
        ne, ns = C.c_uint32(), C.c_uint32()
        load().orc_record_rays(self._h, width, height, frame, pix_begin, pix_end, max_ext, _p(eo), _p(ed), C.byref(ne),
                               max_shadow, _p(so), _p(sd), _p(st), C.byref(ns))
        return (eo[: ne.value], ed[: ne.value]), (so[: ns.value], sd[: ns.value], st[: ns.value])

    def bvh_depths(self):
        t, b = C.c_uint32(), C.c_uint32()
        load().orc_bvh_depths(self._h, C.byref(t), C.byref(b))
        return t.value, b.value

    def close(self):
        if self._h:
            load().orc_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def set_zero_cutoff(on: bool):
    """Radiance-neutral early end of zero-throughput paths (default off = reference)."""
    load().orc_set_zero_cutoff(1 if on else 0)


def init_seed(s: int) -> int:
    return load().orc_init_seed(s)


def random_u32_stream(seed: int, n: int) -> list[int]:
    s = C.c_uint32(seed)
    return [load().orc_random_u32(C.byref(s)) for _ in range(n)]


def finalize_rgba8(acc: np.ndarray, inv_samples: float) -> np.ndarray:
    acc = np.ascontiguousarray(acc, np.float32).reshape(-1, 4)
    out = np.zeros(len(acc), np.uint32)
    load().orc_finalize_rgba8(_p(acc), len(acc), inv_samples, _p(out))
    return out


def bvh_build(tris: np.ndarray):
    """Sequential reference BLAS build over (n, 16) float32 Triangle records
    (v0, v1, v2, centroid at 16-B strides).  Returns (indices (n,) u32,
    nodes (used, 12) float32 view of the 48-B BvhNode records)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32)
    n = tris.shape[0]
    idx = np.empty(n, np.uint32)
    nodes = np.zeros((2 * n, 12), np.float32)
    used = load().orc_bvh_build(_p(tris), n, _p(idx), _p(nodes))
    return idx, nodes[:used]


def obj_load(path: str):
    """Mesh(path) with tinyobj semantics: ((n, 16) float32 Triangle records,
    (n, 20) float32 TriExtension records)."""
    n = load().orc_obj_load(path.encode(), None, None, 0)
    if n < 0:
        raise OSError(f"oracle: cannot read {path}")
    tris = np.zeros((n, 16), np.float32)
    ext = np.zeros((n, 20), np.float32)
    load().orc_obj_load(path.encode(), _p(tris), _p(ext), n)
    return tris, ext

