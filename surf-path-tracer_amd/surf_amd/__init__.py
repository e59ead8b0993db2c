"""ctypes binding of libsurf_hip.so (include/surf_hip.h).

Python is test/bench plumbing here: the product is the C-ABI library (HIP
kernels for gfx950 + C++ host API).  Importing this module never falls back
to anything: if the library is missing, `load()` raises.

Mirrors the reference interface for the hot path:
  Scene.indoor(...)            main.cpp:161-346 scene (Mesh/BvhBLAS/Instance/GPUScene)
  Renderer(...)                WaveFrontRenderer (renderer.h:207-436)
    .render(frames, first, spp=) render loop: frames of spp samples per pixel (Renderer::render)
    .clear_accumulator()       IRenderer::clearAccumulator
    .accumulator()             float RGBA accumulator (rows of this shard)
    .finalize_rgba8()          wavefront_finalize.comp + RgbaToU32
    .trace_closest/.trace_any  ray_extend / ray_connect traversal (tests)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "lib", "libsurf_hip.so")
MGPU_LIB_PATH = os.path.join(_PKG, "lib", "libsurf_mgpu.so")
REPO_ROOT = os.path.dirname(_PKG)
ASSETS_DIR = os.path.join(REPO_ROOT, "assets")

SURF_OK = 0
_STATUS = {
    -1: "SURF_ERR_INVALID", -2: "SURF_ERR_HIP", -3: "SURF_ERR_NO_DEVICE", -4: "SURF_ERR_NO_SCENE",
    -5: "SURF_ERR_OOM", -6: "SURF_ERR_IO", -7: "SURF_ERR_LIMIT",
}


class SurfError(RuntimeError):
    def __init__(self, code: int, what: str, detail: str):
        super().__init__(f"{what} failed: {_STATUS.get(code, code)}: {detail}")
        self.code = code


class SceneDesc(C.Structure):
    _fields_ = [
        ("triangles", C.c_void_p), ("triangle_count", C.c_uint32),
        ("tri_ext", C.c_void_p),
        ("blas_indices", C.c_void_p), ("blas_index_count", C.c_uint32),
        ("blas_nodes", C.c_void_p), ("blas_node_count", C.c_uint32),
        ("materials", C.c_void_p), ("material_count", C.c_uint32),
        ("instances", C.c_void_p), ("instance_count", C.c_uint32),
        ("tlas_indices", C.c_void_p),
        ("tlas_nodes", C.c_void_p), ("tlas_node_count", C.c_uint32),
        ("lights", C.c_void_p), ("light_count", C.c_uint32),
        ("background", C.c_void_p),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("samples", C.c_uint64), ("n_ext", C.c_uint64), ("n_hit", C.c_uint64), ("n_cont", C.c_uint64),
        ("n_shadow", C.c_uint64), ("n_acc", C.c_uint64), ("n_unocc", C.c_uint64), ("iterations", C.c_uint64),
        ("tail_paths", C.c_uint64),
        ("ms_total", C.c_double), ("ms_extend", C.c_double), ("ms_shade", C.c_double), ("ms_connect", C.c_double),
        ("ms_regen", C.c_double), ("ms_tail", C.c_double), ("ms_accum", C.c_double), ("ms_sort", C.c_double),
        ("launches_extend", C.c_uint64), ("n_ext_wavefront", C.c_uint64),
        ("stack_depth", C.c_uint32), ("pool_capacity", C.c_uint32),
        ("energy", C.c_float), ("max_segments", C.c_uint32), ("tail_survivors", C.c_uint64),
        ("frame_window", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


CameraUBO = C.c_uint8 * 128

_lib = None

# Byte sizes of the reference records (include/surf_hip.h static_asserts).
RECORD_BYTES = {"triangles": 64, "tri_ext": 80, "blas_indices": 4, "blas_nodes": 48, "materials": 64,
                "instances": 160, "tlas_indices": 4, "tlas_nodes": 48, "lights": 8, "background": 64}


def load() -> C.CDLL:
    """Loads libsurf_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("SURF_HIP_LIB", LIB_PATH)   # tuning builds (make variants); still the HIP library
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run `make -C surf-path-tracer_amd` or __graft_entry__.build()")
    lib = C.CDLL(path)
    P, U32, I32, F = C.c_void_p, C.c_uint32, C.c_int, C.c_float
    sig = {
        "surf_abi_version": ([], I32), "surf_device_count": ([C.POINTER(I32)], I32),
        "surf_create": ([I32, U32, U32, U32, U32, C.POINTER(P)], I32),
        "surf_create_sharded": ([I32, U32, U32, U32, U32, U32, C.POINTER(P)], I32),
        "surf_destroy": ([P], None), "surf_last_error": ([P], C.c_char_p),
        "surf_shard_rows": ([P, P, C.POINTER(U32)], I32), "surf_get_device": ([P, C.POINTER(I32)], I32),
        "surf_shard_row_list": ([U32, U32, U32, U32, P, C.POINTER(U32)], I32),
        "surf_pack_rgba8": ([P, U32, F, I32, P], I32),
        "surf_set_pool_capacity": ([P, U32], I32), "surf_set_frame_batch": ([P, U32], I32),
        "surf_set_profiling": ([P, I32], I32), "surf_set_zero_cutoff": ([P, I32], I32), "surf_set_trace_mode": ([P, I32], I32), "surf_set_tail_policy": ([P, U32, U32, U32], I32), "surf_set_tail_coop": ([P, U32], I32),
        "surf_debug_capped": ([P, P, U32, C.POINTER(C.c_uint64)], I32),
        "surf_debug_issue_order": ([P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)], I32),
        "surf_debug_connect_staging": ([P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)], I32),
        "surf_debug_lane_resumed": ([P, C.POINTER(C.c_uint64)], I32),
        "surf_debug_segment_cycles": ([P, P, U32, P], I32),
        "surf_upload_scene": ([P, C.POINTER(SceneDesc)], I32),
        "surf_set_camera": ([P, P], I32),
        "surf_render": ([P, U32, U32, U32, U32], I32),
        "surf_clear_accumulator": ([P], I32), "surf_read_accumulator": ([P, P], I32),
        "surf_copy_accumulator_device": ([P, P], I32), "surf_finalize_rgba8": ([P, P], I32),
        "surf_get_stats": ([P, C.POINTER(Stats)], I32), "surf_synchronize": ([P], I32),
        "surf_trace_closest": ([P, U32, P, P, P, P, P, P, P], I32),
        "surf_trace_any": ([P, U32, P, P, P, P], I32),
        "surf_scene_build_indoor": ([C.c_char_p, I32, C.POINTER(P)], I32),
        "surf_scene_desc_get": ([P, C.POINTER(SceneDesc)], I32),
        "surf_scene_update": ([P, F], I32),
        "surf_update_instances": ([P, P, U32, P, P, U32, P, U32], I32),
        "surf_scene_camera": ([P, U32, U32, P], I32),
        "surf_scene_bvh_depths": ([P, C.POINTER(U32), C.POINTER(U32)], I32),
        "surf_scene_destroy": ([P], None),
        "surf_bvh_build": ([P, U32, U32, P, P, C.POINTER(U32)], I32),
        "surf_obj_load": ([C.c_char_p, U32, C.POINTER(P)], I32),
        "surf_write_ppm": ([C.c_char_p, U32, U32, P], I32), "surf_write_png": ([C.c_char_p, U32, U32, P], I32),
        "surf_display_rgba8": ([P, P], I32),
        "surf_mesh_data": ([P, C.POINTER(P), C.POINTER(P), C.POINTER(U32)], I32),
        "surf_mesh_destroy": ([P], None),
        "surf_ref_sinf": ([F], F), "surf_ref_cosf": ([F], F), "surf_ref_expf": ([F], F),
    }
    for name, (args, res) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # a library variant built before a diagnostics entry point existed
            # (tools/ab.sh SURF_HIP_LIB=...); tests/test_abi.py checks the product exports all
            if name.startswith("surf_debug_") and os.environ.get("SURF_HIP_LIB"):
                continue
            raise
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


_mgpu = None


def load_mgpu() -> C.CDLL:
    """Loads libsurf_mgpu.so (include/surf_mgpu.h: the RCCL gather and the row
    un-permute of a multi-GPU render); raises if it has not been built."""
    global _mgpu
    if _mgpu is not None:
        return _mgpu
    load()
    if not os.path.exists(MGPU_LIB_PATH):
        raise FileNotFoundError(f"{MGPU_LIB_PATH} not built: run `make -C surf-path-tracer_amd`")
    lib = C.CDLL(MGPU_LIB_PATH)
    P, U32, I32 = C.c_void_p, C.c_uint32, C.c_int
    sig = {
        "surf_mgpu_unique_id": ([P], I32),
        "surf_mgpu_create": ([P, U32, U32, U32, U32, U32, P, C.POINTER(P)], I32),
        "surf_mgpu_create_all": ([P, U32, U32, U32, U32, P], I32),
        "surf_mgpu_gather": ([P, P], I32), "surf_mgpu_gather_all": ([P, U32, P], I32),
        "surf_mgpu_destroy": ([P], None), "surf_mgpu_last_error": ([], C.c_char_p),
        "surf_mgpu_assemble": ([U32, U32, U32, U32, P, U32, P], I32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _mgpu = lib
    return lib


def assemble_slabs(width: int, height: int, shards: int, row_block: int, gathered: np.ndarray) -> np.ndarray:
    """The root's row un-permute of a multi-GPU gather, by libsurf_mgpu's native
    code (surf_mgpu_assemble): gathered is (shards, rows_per_slab, W, 4) float32,
    slab k holding shard k's rows in shard order (padding rows ignored)."""
    g = np.ascontiguousarray(gathered, dtype=np.float32)
    if g.ndim != 4 or g.shape[0] != shards or g.shape[2] != width or g.shape[3] != 4:
        raise ValueError(f"gathered shape {g.shape} is not ({shards}, rows, {width}, 4)")
    out = np.zeros((height, width, 4), np.float32)
    try:
        mg = load_mgpu()
    except OSError:
        # libsurf_mgpu.so (it links RCCL) not built or not loadable: the same
        # un-permute on the host in numpy -- a torch.distributed gather does not need RCCL's library
        for k in range(shards):
            rows = shard_rows(height, ShardSpec(k, shards, row_block))
            if len(rows) > g.shape[1]:
                raise ValueError(f"slab smaller than shard {k}")
            out[rows] = g[k, :len(rows)]
        return out
    rc = mg.surf_mgpu_assemble(width, height, shards, row_block, g.ctypes.data, g.shape[1], out.ctypes.data)
    if rc != SURF_OK:
        raise SurfError(rc, "surf_mgpu_assemble", mg.surf_mgpu_last_error().decode())
    return out


def pack_rgba8(acc: np.ndarray, samples: int, display: bool = False) -> np.ndarray:
    """surf_finalize_rgba8 / surf_display_rgba8 of a host accumulator (surf_pack_rgba8)."""
    a = np.ascontiguousarray(acc, dtype=np.float32).reshape(-1, 4)
    out = np.zeros(len(a), np.uint32)
    _check(load().surf_pack_rgba8(a.ctypes.data, len(a), np.float32(1.0) / np.float32(samples), 1 if display else 0,
                                  out.ctypes.data), "surf_pack_rgba8")
    return out


def _check(rc: int, what: str, ctx=None):
    if rc != SURF_OK:
        detail = load().surf_last_error(ctx)
        raise SurfError(rc, what, detail.decode() if detail else "")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = C.c_int(0)
    rc = load().surf_device_count(C.byref(n))
    return n.value if rc == SURF_OK else 0


class Scene:
    """Host scene built by the product's C++ host API (OBJ -> BVH -> GPUBatcher layout)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def indoor(cls, assets_dir: str = ASSETS_DIR, variant: int = 0) -> "Scene":
        h = C.c_void_p()
        _check(load().surf_scene_build_indoor(assets_dir.encode(), variant, C.byref(h)), "surf_scene_build_indoor")
        return cls(h)

    @property
    def handle(self):
        return self._h

    def update(self, delta_time: float):
        """GPUScene::update (scene.cpp:267-282): rotate instance 3, refit the TLAS, re-batch."""
        _check(load().surf_scene_update(self._h, delta_time), "surf_scene_update")

    def desc(self) -> SceneDesc:
        d = SceneDesc()
        _check(load().surf_scene_desc_get(self._h, C.byref(d)), "surf_scene_desc_get")
        return d

    def camera(self, width: int, height: int) -> bytes:
        ubo = CameraUBO()
        _check(load().surf_scene_camera(self._h, width, height, ubo), "surf_scene_camera")
        return bytes(ubo)

    def bvh_depths(self) -> tuple[int, int]:
        t, b = C.c_uint32(), C.c_uint32()
        _check(load().surf_scene_bvh_depths(self._h, C.byref(t), C.byref(b)), "surf_scene_bvh_depths")
        return t.value, b.value

    def buffers(self) -> dict[str, bytes]:
        """The ten reference-layout buffers of the GPUScene, as bytes."""
        d = self.desc()
        counts = {"triangles": d.triangle_count, "tri_ext": d.triangle_count, "blas_indices": d.blas_index_count,
                  "blas_nodes": d.blas_node_count, "materials": d.material_count, "instances": d.instance_count,
                  "tlas_indices": d.instance_count, "tlas_nodes": d.tlas_node_count, "lights": d.light_count,
                  "background": 1}
        out = {}
        for k, n in counts.items():
            ptr = getattr(d, k)
            out[k] = C.string_at(ptr, n * RECORD_BYTES[k]) if n else b""
        return out

    def close(self):
        if self._h:
            load().surf_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_image(path: str, rgba8: np.ndarray) -> None:
    """Writes an (H, W) uint32 RGBA8 image (R in the low byte) as PNG or, for a
    .ppm path, binary PPM (alpha dropped)."""
    img = np.ascontiguousarray(rgba8, dtype=np.uint32)
    h, w = img.shape
    fn = load().surf_write_ppm if path.lower().endswith(".ppm") else load().surf_write_png
    _check(fn(path.encode(), w, h, _ptr(img)), "surf_write_image")


def obj_load(path: str, threads: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Mesh(path) (mesh.cpp:69-154): parallel tinyobj-compatible OBJ/OBJ.GZ parse.
    Returns ((n, 16) float32 Triangle records, (n, 20) float32 TriExtension
    records); identical for every thread count."""
    h = C.c_void_p()
    _check(load().surf_obj_load(path.encode(), threads, C.byref(h)), "surf_obj_load")
    try:
        tp, xp, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
        _check(load().surf_mesh_data(h, C.byref(tp), C.byref(xp), C.byref(n)), "surf_mesh_data")
        k = n.value
        tris = np.ctypeslib.as_array(C.cast(tp, C.POINTER(C.c_float)), (k * 16,)).reshape(k, 16).copy() if k else np.zeros((0, 16), np.float32)
        ext = np.ctypeslib.as_array(C.cast(xp, C.POINTER(C.c_float)), (k * 20,)).reshape(k, 20).copy() if k else np.zeros((0, 20), np.float32)
    finally:
        load().surf_mesh_destroy(h)
    return tris, ext


def bvh_build(triangles: np.ndarray, threads: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """BvhBLAS::build (bvh.cpp:255-465) over (n, 16) float32 Triangle records
    (v0, v1, v2, centroid), multi-threaded (0 = default thread count).
    Returns (indices (n,) uint32, nodes (nodes_used, 12) float32 view of the
    48-B BvhNode records); identical for every thread count."""
    tris = np.ascontiguousarray(triangles, dtype=np.float32)
    n = tris.shape[0]
    idx = np.empty(n, np.uint32)
    nodes = np.zeros((2 * n, 12), np.float32)
    used = C.c_uint32()
    _check(load().surf_bvh_build(_ptr(tris), n, threads, _ptr(idx), _ptr(nodes), C.byref(used)), "surf_bvh_build")
    return idx, nodes[: used.value]


@dataclass
class ShardSpec:
    shard: int = 0
    shards: int = 1
    row_block: int = 0      # 0: contiguous rows; N: interleaved blocks of N rows


def shard_rows(height: int, spec: ShardSpec) -> np.ndarray:
    """Rows a shard owns -- same rule as surf_create_sharded."""
    r = np.arange(height, dtype=np.int64)
    if spec.row_block == 0:
        lo = height * spec.shard // spec.shards
        hi = height * (spec.shard + 1) // spec.shards
        return r[lo:hi]
    return r[(r // spec.row_block) % spec.shards == spec.shard]


def assemble_shards(width: int, height: int, parts: list[np.ndarray], specs: list[ShardSpec]) -> np.ndarray:
    """Places per-shard accumulator rows (shard order) into a full (H, W, 4) frame."""
    full = np.zeros((height, width, 4), dtype=np.float32)
    for part, spec in zip(parts, specs):
        rows = shard_rows(height, spec)
        full[rows] = np.asarray(part, dtype=np.float32).reshape(len(rows), width, 4)
    return full


class Renderer:
    """One surf_ctx: a shard of a width x height frame on one HIP device."""

    def __init__(self, scene: Scene, width: int, height: int, device: int = 0, shard: ShardSpec | None = None,
                 pool_capacity: int | None = None, frame_batch: int | None = None, camera: bytes | None = None):
        lib = load()
        self.width, self.height = width, height
        self.shard = shard or ShardSpec()
        h = C.c_void_p()
        _check(lib.surf_create_sharded(device, width, height, self.shard.shard, self.shard.shards,
                                       self.shard.row_block, C.byref(h)), "surf_create_sharded")
        self._h = h
        n = C.c_uint32()
        _check(lib.surf_shard_rows(h, None, C.byref(n)), "surf_shard_rows", h)
        self.rows = np.zeros(n.value, dtype=np.uint32)
        _check(lib.surf_shard_rows(h, _ptr(self.rows), C.byref(n)), "surf_shard_rows", h)
        if pool_capacity:
            _check(lib.surf_set_pool_capacity(h, pool_capacity), "surf_set_pool_capacity", h)
        if frame_batch:
            _check(lib.surf_set_frame_batch(h, frame_batch), "surf_set_frame_batch", h)
        d = scene.desc()
        _check(lib.surf_upload_scene(h, C.byref(d)), "surf_upload_scene", h)
        ubo = camera if camera is not None else scene.camera(width, height)
        buf = CameraUBO.from_buffer_copy(ubo)
        _check(lib.surf_set_camera(h, buf), "surf_set_camera", h)

    @property
    def handle(self):
        return self._h

    def debug_capped(self):
        """(count, sample ids) of paths ended by the segment cap in the current stream."""
        ids = np.zeros(64, np.uint32)
        n = C.c_uint64()
        _check(load().surf_debug_capped(self._h, _ptr(ids), 64, C.byref(n)), "surf_debug_capped", self._h)
        return int(n.value), ids[ids != 0xFFFFFFFF]

    def debug_issue_order(self):
        """(heavy pixels, permuted frames) of the current stream's issue order
        (surf_debug_issue_order); (0, 0) when it is frame-major throughout."""
        a, f = C.c_uint32(), C.c_uint32()
        _check(load().surf_debug_issue_order(self._h, C.byref(a), C.byref(f)), "surf_debug_issue_order", self._h)
        return int(a.value), int(f.value)

    def debug_lane_resumed(self):
        """Extension rays the capped lane walk left to k_extend_cont (SURF_LANE_CAP)
        since the accumulator was last cleared (surf_debug_lane_resumed)."""
        n = C.c_uint64()
        _check(load().surf_debug_lane_resumed(self._h, C.byref(n)), "surf_debug_lane_resumed", self._h)
        return int(n.value)

    def debug_connect_staging(self):
        """(records, triangles) of the emitters' BLAS the last k_connect launch
        walked from LDS (surf_debug_connect_staging); (0, 0) when none was staged."""
        a, t = C.c_uint32(), C.c_uint32()
        _check(load().surf_debug_connect_staging(self._h, C.byref(a), C.byref(t)), "surf_debug_connect_staging", self._h)
        return int(a.value), int(t.value)

    def debug_segment_cycles(self, origin, direction, throughput, seed: int, segment: int = 1, reps: int = 64):
        """Diagnostics: mean shader-clock cycles of one drain segment's pieces on
        a lone wave (surf_debug_segment_cycles): walk, shade, shadow walk,
        cosine sample, light sample, hit normal."""
        rec = np.zeros(12, np.float32)
        rec[0:3] = origin
        rec[4:7] = direction
        rec[8:11] = throughput
        u = rec.view(np.uint32)
        u[3] = 0
        u[7] = (segment << 2)
        u[11] = seed & 0xFFFFFFFF
        out = np.zeros(15, np.uint64)
        _check(load().surf_debug_segment_cycles(self._h, _ptr(rec), reps, _ptr(out)), "surf_debug_segment_cycles", self._h)
        names = ("walk", "shade", "shadow_walk", "cosine", "light_sample", "normal", "checksum", "interior_cycles",
                 "leaf_cycles", "walks", "leaves", "triangles", "visits2", "prologue_cycles", "instance_loop_cycles")
        return {k: float(out[i]) / reps for i, k in enumerate(names) if k != "checksum"}

    def set_zero_cutoff(self, on):
        """True / False, or None for the automatic default (on for 1-sample frames, off for multi-sample frames)."""
        _check(load().surf_set_zero_cutoff(self._h, -1 if on is None else (1 if on else 0)), "surf_set_zero_cutoff", self._h)

    def update_instances(self, scene: Scene):
        """Re-uploads the scene's instance records, TLAS and lights (after Scene.update)."""
        d = scene.desc()
        _check(load().surf_update_instances(self._h, d.instances, d.instance_count, d.tlas_indices, d.tlas_nodes,
                                            d.tlas_node_count, d.lights, d.light_count), "surf_update_instances", self._h)

    def set_tail_policy(self, threshold_paths: int = 0, lanes_per_wave: int = 0, stage_segments: int = 0):
        """Drain policy of the tail kernel (0 = automatic); stage_segments is the
        per-stage segment budget before the survivors move on (0 = one stage)."""
        _check(load().surf_set_tail_policy(self._h, threshold_paths, lanes_per_wave, stage_segments), "surf_set_tail_policy",
               self._h)

    def set_tail_coop(self, max_paths: int):
        """Single-stage drain as the cooperative tail when <= max_paths paths remain (0 = never)."""
        _check(load().surf_set_tail_coop(self._h, max_paths), "surf_set_tail_coop", self._h)

    def set_trace_mode(self, mode: int):
        """0: one ray per lane; 1: one ray per wave (lanes as planes, the cooperative tail's traversal),
        for trace_closest/trace_any."""
        _check(load().surf_set_trace_mode(self._h, mode), "surf_set_trace_mode", self._h)

    def set_profiling(self, on: bool):
        _check(load().surf_set_profiling(self._h, 1 if on else 0), "surf_set_profiling", self._h)

    def render(self, frames: int, first_frame: int = 0, max_segments: int = 0, spp: int = 1):
        """`frames` frames of `spp` samples per pixel (Renderer::render with
        samplesPerFrame = spp, renderer.cpp:160-188): first_frame is the sample
        count before the call (the reference's totalSamples; the frame index for
        spp 1); frame k is seeded from first_frame + k * spp and its samples
        chain their RNG state."""
        _check(load().surf_render(self._h, frames, first_frame, max_segments, spp), "surf_render", self._h)

    def synchronize(self):
        _check(load().surf_synchronize(self._h), "surf_synchronize", self._h)

    def clear_accumulator(self):
        _check(load().surf_clear_accumulator(self._h), "surf_clear_accumulator", self._h)

    def accumulator(self) -> np.ndarray:
        out = np.zeros((len(self.rows), self.width, 4), dtype=np.float32)
        _check(load().surf_read_accumulator(self._h, _ptr(out)), "surf_read_accumulator", self._h)
        return out

    def copy_accumulator_to(self, device_ptr: int):
        _check(load().surf_copy_accumulator_device(self._h, C.c_void_p(device_ptr)), "surf_copy_accumulator_device", self._h)

    def finalize_rgba8(self) -> np.ndarray:
        out = np.zeros((len(self.rows), self.width), dtype=np.uint32)
        _check(load().surf_finalize_rgba8(self._h, _ptr(out)), "surf_finalize_rgba8", self._h)
        return out

    def display_rgba8(self) -> np.ndarray:
        """The displayed image: fs_quad.frag's sqrt gamma on the RGBA8 finalize image."""
        out = np.zeros((len(self.rows), self.width), dtype=np.uint32)
        _check(load().surf_display_rgba8(self._h, _ptr(out)), "surf_display_rgba8", self._h)
        return out

    def stats(self) -> dict:
        s = Stats()
        _check(load().surf_get_stats(self._h, C.byref(s)), "surf_get_stats", self._h)
        return s.as_dict()

    def trace_closest(self, o: np.ndarray, d: np.ndarray):
        o = np.ascontiguousarray(o, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, dtype=np.float32).reshape(-1, 3)
        n = len(o)
        t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        inst, prim = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        _check(load().surf_trace_closest(self._h, n, _ptr(o), _ptr(d), _ptr(t), _ptr(u), _ptr(v), _ptr(inst), _ptr(prim)),
               "surf_trace_closest", self._h)
        return t, u, v, inst, prim

    def trace_any(self, o: np.ndarray, d: np.ndarray, tmax: np.ndarray) -> np.ndarray:
        o = np.ascontiguousarray(o, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, dtype=np.float32).reshape(-1, 3)
        tmax = np.ascontiguousarray(tmax, dtype=np.float32)
        occ = np.zeros(len(o), np.uint8)
        _check(load().surf_trace_any(self._h, len(o), _ptr(o), _ptr(d), _ptr(tmax), _ptr(occ)), "surf_trace_any", self._h)
        return occ

    def close(self):
        if self._h:
            load().surf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
