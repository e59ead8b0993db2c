"""The CPU oracle (oracle/cpu_ref.cpp) against what can pin it here.

The reference is unbuildable in this image (glm, tinyobjloader and Vulkan
headers are absent; stand-ins are not allowed), so no reference output exists
to compare with: "parity unpinned".  These tests pin the oracle to the data
the reference ships (asset triangle counts, scene composition of main.cpp),
to an independent restatement of its RNG (pure Python), and to properties the
algorithm must satisfy (BVH closest hit == brute-force closest hit)."""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def py_wang(s):
    """wangHash, surf_math.cpp:31-42, restated in Python."""
    m = 0xFFFFFFFF
    s = ((s ^ 61) ^ (s >> 16)) & m
    s = (s * 9) & m
    s = s ^ (s >> 4)
    s = (s * 0x27D4EB2D) & m
    s = s ^ (s >> 15)
    return s


def py_init_seed(s):
    return py_wang(((s + 1) * 0x11) & 0xFFFFFFFF)


def py_xorshift(s, n):
    out = []
    for _ in range(n):
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        out.append(s)
    return out


def test_asset_facts(oracle_scene):
    # OBJ files of the reference (assets/*.obj): triangle counts after triangulation
    assert oracle_scene.mesh_tris() == [15744, 188, 960, 2]
    assert oracle_scene.instance_count() == 11           # main.cpp:360
    assert oracle_scene.light_count() == 2               # cubeL, cubeR
    # 16,894 unique and 32,836 instanced triangles
    tris = dict(zip(["susanne", "cube", "lens", "plane"], oracle_scene.mesh_tris()))
    assert sum(tris.values()) == 16894
    inst = 2 * tris["susanne"] + 2 * tris["cube"] + tris["lens"] + 6 * tris["plane"]
    assert inst == 32836                                   # floor + 5 walls = 6 planes


def test_rng_known_answers():
    for seed in [0, 1, 7, 1799, 123456789, 0xFFFFFFF0]:
        assert oracle.init_seed(seed) == py_init_seed(seed)
        s = py_init_seed(seed)
        assert oracle.random_u32_stream(s, 64) == py_xorshift(s, 64)


def test_rng_golden_fixture():
    with open(os.path.join(GOLDEN, "rng.json")) as f:
        g = json.load(f)
    for case in g["cases"]:
        assert oracle.init_seed(case["seed"]) == case["init"]
        assert oracle.random_u32_stream(case["init"], len(case["stream"])) == case["stream"]


def _random_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform([-9, -0.9, -9], [9, 8.9, 9], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


def test_bvh_closest_equals_brute_force(oracle_scene):
    o, d = _random_rays(4000, 1)
    t, u, v, inst, prim = oracle_scene.trace_closest(o, d)
    tb, ib, pb = oracle_scene.trace_brute(o, d)
    hit = inst != 0xFFFFFFFF
    assert hit.mean() > 0.95                   # closed room
    assert np.array_equal(hit, ib != 0xFFFFFFFF)
    assert np.array_equal(t[hit], tb[hit])     # same f32 arithmetic -> identical depth
    same = (inst == ib) & (prim == pb)
    assert same[hit].mean() > 0.999            # ties at shared edges may resolve differently


def test_any_hit_consistent_with_closest(oracle_scene):
    o, d = _random_rays(4000, 2)
    t, *_ = oracle_scene.trace_closest(o, d)
    tmax = np.float32(0.5) * np.minimum(t, np.float32(30.0)) + np.float32(0.25)
    occ = oracle_scene.trace_any(o, d, tmax)
    assert np.array_equal(occ.astype(bool), t < tmax)


def test_primary_rays_hit_the_room(oracle_scene):
    (eo, ed), (so, sd, st) = oracle_scene.record_rays(64, 64, 0, 0, 64 * 64, max_ext=1 << 16, max_shadow=1 << 16)
    assert len(eo) >= 64 * 64 and len(so) > 0
    t, *_ = oracle_scene.trace_closest(eo, ed)
    assert np.isfinite(t).all()


def test_render_deterministic_and_row_local(oracle_scene):
    acc, cnt, _ = oracle_scene.render(48, 32, 3)
    acc2, cnt2, _ = oracle_scene.render(48, 32, 3)
    assert np.array_equal(acc, acc2) and cnt == cnt2
    part, _, _ = oracle_scene.render(48, 32, 3, rows=(10, 20))
    assert np.array_equal(part, acc[10:20])               # paths depend on pixel+frame only
    assert np.all(acc[..., 3] == 3.0)
    assert cnt["samples"] == 48 * 32 * 3
    assert cnt["n_ext"] == cnt["samples"] + cnt["n_cont"]   # each path: 1 primary + continuations
    # radiance is non-negative and finite
    assert np.isfinite(acc).all() and (acc[..., :3] >= 0).all()


def test_render_golden_fixture(oracle_scene):
    """Regression fixture of the oracle itself (tests/golden/make_golden.py).
    Not a reference pin: it detects unintended oracle changes."""
    g = np.load(os.path.join(GOLDEN, "oracle_32x24x2.npz"))
    acc, cnt, _ = oracle_scene.render(32, 24, 2)
    assert np.array_equal(acc, g["acc"])
    assert [cnt[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")] == list(g["counts"])


def test_zero_throughput_cutoff_is_radiance_neutral(oracle_scene):
    """Ending paths whose throughput is exactly (0,0,0) must not change a bit of
    the accumulated radiance (the product enables it by default)."""
    oracle.set_zero_cutoff(False)
    a, ca, _ = oracle_scene.render(96, 64, 6)
    b0, _, _ = oracle_scene.render(1280, 720, 1, rows=(300, 306))
    oracle.set_zero_cutoff(True)
    try:
        b, cb, _ = oracle_scene.render(96, 64, 6)
        b1, _, _ = oracle_scene.render(1280, 720, 1, rows=(300, 306))
    finally:
        oracle.set_zero_cutoff(False)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(b0.view(np.uint32), b1.view(np.uint32))
    assert cb["n_ext"] < ca["n_ext"]          # it does remove segments


def test_segment_cap(oracle_scene):
    acc, cnt, _ = oracle_scene.render(32, 16, 2, max_segments=8)
    assert cnt["max_segments"] <= 8
    assert cnt["n_ext"] <= 8 * cnt["samples"]


def test_finalize_rgba8_rounding():
    acc = np.array([[0.5, 1.5, 255.0, 512.0], [np.nan, -1.0, 254.5, 255.0], [3e9, 2.5, 0.0, 255.0]], np.float32)
    out = oracle.finalize_rgba8(acc, np.float32(1.0 / 255.0))
    b = lambda w, k: (int(w) >> (8 * k)) & 0xFF
    scaled = (acc * np.float32(1.0 / 255.0)) * np.float32(255.0)
    for i in range(3):
        for k in range(4):
            x = scaled[i, k]
            want = 0 if not np.isfinite(x) or abs(x) >= 2**31 else int(min(max(np.rint(x), 0), 255))
            assert b(out[i], k) == want, (i, k, x)
