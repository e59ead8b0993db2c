"""GPU parity: the HIP wavefront path against the CPU oracle on the same inputs.

Bar: bit-exact.  Every value the kernels produce (hit records, occlusion,
per-pixel float radiance, event counts) must equal the oracle's bit for bit:
the kernels replay the reference's f32 operation order, its traversal order
and glibc's sinf/cosf/expf (csrc/device/surf_math.h).  The north-star
tolerance (per-pixel L2 < 1e-3 vs the CPU reference) is also asserted so a
failure reports by how much it missed.
"""
import numpy as np
import pytest

import oracle
import surf_amd

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
UNSET = 0xFFFFFFFF


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    surf_amd.load()
    assert surf_amd.device_count() > 0, "no HIP device: -m gpu tests need an MI355X"


def l2_report(a, b):
    a = a[..., :3].astype(np.float64)
    b = b[..., :3].astype(np.float64)
    per = np.sqrt(((a - b) ** 2).sum(-1))
    return float(np.sqrt((per ** 2).mean())), float(per.max()), float((per > 1e-3).mean())


@pytest.mark.parametrize("mode", [0, 1], ids=["lane-per-ray", "wave-lanes-as-planes"])
def test_closest_hit_records_bitexact(oracle_scene, product_scene, mode):
    W = H = 96
    (eo, ed), (so, sd, st) = oracle_scene.record_rays(W, H, 0, 0, W * H)
    rng = np.random.default_rng(5)
    ro = rng.uniform([-9, -0.9, -9], [9, 8.9, 9], size=(20000, 3)).astype(np.float32)
    rd = rng.normal(size=(20000, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    o = np.concatenate([eo, so, ro])
    d = np.concatenate([ed, sd, rd])
    r = surf_amd.Renderer(product_scene, W, H)
    r.set_trace_mode(mode)
    gpu = r.trace_closest(o, d)
    cpu = oracle_scene.trace_closest(o, d)
    names = ["t", "u", "v", "inst", "prim"]
    for n, g, c in zip(names, gpu, cpu):
        bad = np.nonzero(g.view(np.uint32) != c.view(np.uint32))[0]
        assert len(bad) == 0, f"{n}: {len(bad)} of {len(g)} differ, first {bad[:5]}"
    assert (gpu[3] != UNSET).mean() > 0.9


def test_boundary_rays_bitexact(oracle_scene, product_scene):
    """Rays the instance cull and the slab fast paths must not get wrong: aimed
    at surface points (hits at the end of a shadow segment, tmax exactly the
    distance), grazing along axis planes (zero direction components: 1/d = inf),
    and from outside the room toward it."""
    W = H = 64
    (eo, ed), _ = oracle_scene.record_rays(W, H, 2, 0, W * H)
    t, _, _, inst, _ = oracle_scene.trace_closest(eo, ed)
    hit = inst != UNSET
    P = (eo[hit] + t[hit, None] * ed[hit])[:6000]
    rng = np.random.default_rng(11)
    src = rng.uniform([-12, -2, -12], [12, 11, 12], size=(len(P), 3)).astype(np.float32)
    dv = (P - src).astype(np.float32)
    dist = np.linalg.norm(dv, axis=1).astype(np.float32)
    dn = (dv / dist[:, None]).astype(np.float32)
    axis = np.zeros((3000, 3), np.float32)
    axis[np.arange(3000), rng.integers(0, 3, 3000)] = rng.choice([-1.0, 1.0], 3000).astype(np.float32)
    ao = rng.uniform([-9, -0.9, -9], [9, 8.9, 9], size=(3000, 3)).astype(np.float32)
    o = np.concatenate([src, ao]).astype(np.float32)
    d = np.concatenate([dn, axis]).astype(np.float32)
    r = surf_amd.Renderer(product_scene, W, H)
    for mode in (0, 1):
        r.set_trace_mode(mode)
        gpu = r.trace_closest(o, d)
        cpu = oracle_scene.trace_closest(o, d)
        for n, g, c in zip(["t", "u", "v", "inst", "prim"], gpu, cpu):
            bad = np.nonzero(g.view(np.uint32) != c.view(np.uint32))[0]
            assert len(bad) == 0, f"mode {mode} {n}: {len(bad)} of {len(g)} differ, first {bad[:5]}"
        for tm in (dist, np.nextafter(dist, np.float32(0)), np.nextafter(dist, np.float32(np.inf))):
            tmax = np.concatenate([tm, np.full(3000, 1e30, np.float32)]).astype(np.float32)
            assert np.array_equal(r.trace_any(o, d, tmax), oracle_scene.trace_any(o, d, tmax)), f"mode {mode}"


@pytest.mark.parametrize("mode", [0, 1], ids=["lane-per-ray", "wave-lanes-as-planes"])
def test_any_hit_bitexact(oracle_scene, product_scene, mode):
    W = H = 96
    _, (so, sd, st) = oracle_scene.record_rays(W, H, 1, 0, W * H)
    r = surf_amd.Renderer(product_scene, W, H)
    r.set_trace_mode(mode)
    g = r.trace_any(so, sd, st)
    c = oracle_scene.trace_any(so, sd, st)
    assert len(so) > 1000
    assert np.array_equal(g, c)


def test_lane_two_level_walk_bitexact(oracle_scene, monkeypatch):
    """The one-ray-per-lane traversal over the two-level records (blasTraceW:
    one fetch per two BVH levels, the default for HBM-resident BVHs such as
    C5's), forced on the bundled scene (SURF_LANEW=1): closest-hit records,
    any-hit and a render with its event counts equal the oracle's."""
    monkeypatch.setenv("SURF_LANEW", "1")
    p = surf_amd.Scene.indoor()
    try:
        W = H = 96
        (eo, ed), (so, sd, st) = oracle_scene.record_rays(W, H, 0, 0, W * H)
        rng = np.random.default_rng(13)
        ro = rng.uniform([-9, -0.9, -9], [9, 8.9, 9], size=(20000, 3)).astype(np.float32)
        rd = rng.normal(size=(20000, 3)).astype(np.float32)
        rd /= np.linalg.norm(rd, axis=1, keepdims=True)
        o, d = np.concatenate([eo, so, ro]), np.concatenate([ed, sd, rd])
        r = surf_amd.Renderer(p, W, H)
        gpu, cpu = r.trace_closest(o, d), oracle_scene.trace_closest(o, d)
        for n, g, c in zip(["t", "u", "v", "inst", "prim"], gpu, cpu):
            bad = np.nonzero(g.view(np.uint32) != c.view(np.uint32))[0]
            assert len(bad) == 0, f"{n}: {len(bad)} of {len(g)} differ, first {bad[:5]}"
        assert np.array_equal(r.trace_any(so, sd, st), oracle_scene.trace_any(so, sd, st))
        r.render(4, 0, 0)
        g = r.accumulator()
        stats = r.stats()
        r.close()
        oracle.set_zero_cutoff(True)
        try:
            c, cnt, _ = oracle_scene.render(W, H, 4)
        finally:
            oracle.set_zero_cutoff(False)
        _assert_bitexact(g, c, "lane two-level walk 96x96x4")
        _assert_counts(stats, cnt)
    finally:
        p.close()


@pytest.mark.parametrize("walk,cap", [("one-level", "4"), ("one-level", "24"), ("two-level", "2"), ("two-level", "12")])
def test_lane_walk_cap_resume_bitexact(oracle_scene, monkeypatch, walk, cap):
    """The capped lane walk (SURF_LANE_CAP): a ray whose BLAS walk takes more
    than `cap` node visits (W-record visits in the two-level walk, forced on
    the bundled scene by SURF_LANEW=1) is finished from the lane's state (its
    next node, its stack, depth and hit so far, then the instances after it)
    by k_extend_cont, the lane walk again with 64 such rays to a wave.  With
    caps small enough that many rays hand over: a render and its event counts
    equal the oracle's, and rays were resumed."""
    monkeypatch.setenv("SURF_LANEW", "1" if walk == "two-level" else "0")
    monkeypatch.setenv("SURF_LANE_CAP", cap)
    p = surf_amd.Scene.indoor()
    try:
        W = H = 96
        r = surf_amd.Renderer(p, W, H)
        r.render(4, 0, 0)
        g = r.accumulator()
        stats = r.stats()
        resumed = r.debug_lane_resumed()
        r.close()
        oracle.set_zero_cutoff(True)
        try:
            c, cnt, _ = oracle_scene.render(W, H, 4)
        finally:
            oracle.set_zero_cutoff(False)
        _assert_bitexact(g, c, f"capped lane walk (cap {cap}) 96x96x4")
        _assert_counts(stats, cnt)
        assert resumed > 1000, resumed
    finally:
        p.close()


def _render_both(oracle_scene, product_scene, W, H, frames, first=0, max_seg=0, **kw):
    """GPU render (zero-throughput cutoff on, the product default) against the
    oracle in reference semantics (no cutoff) for radiance, and against the
    oracle with the cutoff for event counts (the cutoff only removes segments)."""
    r = surf_amd.Renderer(product_scene, W, H, **kw)
    r.render(frames, first, max_seg)
    g = r.accumulator()
    stats = r.stats()
    oracle.set_zero_cutoff(False)
    c, _, _ = oracle_scene.render(W, H, frames, first_frame=first, max_segments=max_seg)
    oracle.set_zero_cutoff(True)
    try:
        c2, cnt, _ = oracle_scene.render(W, H, frames, first_frame=first, max_segments=max_seg)
    finally:
        oracle.set_zero_cutoff(False)
    assert np.array_equal(c.view(np.uint32), c2.view(np.uint32)), "cutoff changed the oracle's radiance"
    return g, c, stats, cnt, r


def _assert_bitexact(g, c, what):
    rms, mx, frac = l2_report(g, c)
    assert rms < 1e-3, f"{what}: per-pixel L2 RMS {rms} (max {mx}, >1e-3 on {frac:.4%} of pixels)"
    bad = np.argwhere(g.view(np.uint32) != c.view(np.uint32))
    assert len(bad) == 0, f"{what}: {len(bad)} accumulator words differ (RMS {rms:.3e}), first {bad[:4].tolist()}"


def _assert_counts(stats, cnt):
    for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc"):
        assert stats[k] == cnt[k], (k, stats[k], cnt[k])


def test_render_64x64x4_bitexact(oracle_scene, product_scene):
    g, c, stats, cnt, _ = _render_both(oracle_scene, product_scene, 64, 64, 4)
    _assert_bitexact(g, c, "64x64x4")
    _assert_counts(stats, cnt)


@pytest.mark.parametrize("policy,coop,engine", [((0, 0, 16), 60000, "pair"), ((0, 0, 16), 60000, "coop"),
                                                ((0, 8, 4), 0, "lanes"), ((1 << 30, 0, 8), 1 << 30, "pair"),
                                                ((1 << 30, 0, 8), 1 << 30, "coop"), ((1, 0, 0), 0, "lanes")],
                         ids=["staged+pair", "staged+coop", "8-lanes-staged", "pair-from-start", "coop-from-start",
                              "wavefront-to-end"])
def test_drain_policies_bitexact(oracle_scene, product_scene, policy, coop, engine, monkeypatch):
    """Every drain schedule (lane stages with survivor hand-off, the partner-wave tail (k_tail_pair: idle waves
    trace their sibling's shadow rays), the one-path-per-wave tail, tail from
    the first phase, wavefront to the end) gives the same radiance and event
    counts."""
    monkeypatch.setenv("SURF_TAIL_PAIR", "0" if engine == "coop" else "1")
    r0 = surf_amd.Renderer(product_scene, 96, 64)
    r0.set_tail_policy(*policy)
    r0.set_tail_coop(coop)
    r0.render(4, 0, 0)
    g = r0.accumulator()
    st = r0.stats()
    oracle.set_zero_cutoff(True)
    try:
        c2, cnt, _ = oracle_scene.render(96, 64, 4)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c2, f"drain policy {policy}")
    _assert_counts(st, cnt)
    r0.close()


@pytest.mark.parametrize("sort,block,connect", [("0", "128", "0"), ("1", "128", "0"), ("1", "256", "0"), ("1", "128", "1")],
                         ids=["unsorted", "order-index", "extend-block-256", "connect-global-tables"])
def test_ray_order_and_launch_shapes_bitexact(oracle_scene, product_scene, sort, block, connect, monkeypatch):
    """The ray order and the launch shapes are lane interleaving only: no sort
    (SURF_SORT=0) and the order[] gather (default), k_extend in 128- or
    256-thread workgroups (SURF_EXTEND_BLOCK), k_connect with LDS or global
    trace tables (SURF_CONNECT_GLOBAL) all give the oracle's radiance and event
    counts bit for bit."""
    W, H, F = 128, 96, 4
    monkeypatch.setenv("SURF_SORT", sort)
    monkeypatch.setenv("SURF_EXTEND_BLOCK", block)
    monkeypatch.setenv("SURF_CONNECT_GLOBAL", connect)
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=8192)
    r.render(F, 0, 0)
    g = r.accumulator()
    st = r.stats()
    oracle.set_zero_cutoff(True)
    try:
        c2, cnt, _ = oracle_scene.render(W, H, F)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c2, f"ray order sort={sort} extend block={block} connect global={connect}")
    _assert_counts(st, cnt)
    r.close()


@pytest.mark.parametrize("reorder,key,overlap", [("1", "2", "1"), ("0", "2", "1"), ("1", "1", "1"), ("1", "0", "1"),
                                                 ("1", "2", "0")],
                         ids=["default", "frame-major-issue", "ascending-mask-key", "start-instance-key", "connect-serialized"])
def test_issue_order_keys_overlap_bitexact(oracle_scene, product_scene, reorder, key, overlap, monkeypatch):
    """Scheduling only: the class-ordered issue of a multi-frame stream (pixels
    whose centre ray first hits a heavy instance, all frames first;
    SURF_REORDER), the pool's ray-order key (heavy-BLAS mask, most heavy
    first or ascending, or start instance; SURF_KEY) and k_connect on its own
    graph stream (SURF_OVERLAP)
    change no sample: radiance and event counts equal the oracle's."""
    W, H, F = 96, 64, 6
    monkeypatch.setenv("SURF_REORDER", reorder)
    monkeypatch.setenv("SURF_KEY", key)
    monkeypatch.setenv("SURF_OVERLAP", overlap)
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=4096)
    r.render(F, 0, 0)
    heavy, permuted = r.debug_issue_order()
    if reorder == "1":      # the class-ordered issue must be engaged, not trivially skipped
        assert 0 < heavy < W * H and permuted == F, (heavy, permuted)
    else:
        assert (heavy, permuted) == (0, 0)
    g = r.accumulator()
    st = r.stats()
    oracle.set_zero_cutoff(True)
    try:
        c2, cnt, _ = oracle_scene.render(W, H, F)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c2, f"reorder={reorder} key={key} overlap={overlap}")
    _assert_counts(st, cnt)
    r.close()


def test_permuted_stream_continued_bitexact(oracle_scene, product_scene, monkeypatch):
    """A class-ordered (permuted) stream continued by a second call: render(6)
    issues its six frames heavy pixels first; render(6, first=6) continues the
    same sample stream (no restart), so frames 6..11 follow the permuted head
    frame-major.  The 12 frames equal the oracle's bit for bit."""
    W, H, F = 96, 64, 6
    monkeypatch.setenv("SURF_REORDER", "1")
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=4096)
    r.render(F, 0, 0)
    heavy, permuted = r.debug_issue_order()
    assert 0 < heavy < W * H and permuted == F, (heavy, permuted)
    r.render(F, F, 0)
    assert r.debug_issue_order() == (heavy, permuted), "the second call must continue, not restart, the stream"
    g = r.accumulator()
    st = r.stats()
    r.close()
    oracle.set_zero_cutoff(True)
    try:
        c2, cnt, _ = oracle_scene.render(W, H, 2 * F)
    finally:
        oracle.set_zero_cutoff(False)
    assert np.all(g[..., 3] == 2 * F)
    _assert_bitexact(g, c2, "permuted stream continued across calls")
    _assert_counts(st, cnt)


@pytest.mark.parametrize("staged", ["1", "0"], ids=["light-blas-in-lds", "light-blas-global"])
def test_connect_light_blas_staging_bitexact(oracle_scene, product_scene, staged, monkeypatch):
    """k_connect with the emitters' BLAS node records staged in LDS (the lights'
    instances walk them there, beside a 16-bit traversal stack; the default
    for the bundled scene) and without (SURF_LDS_LIGHTBLAS=0): the same node
    records and decisions, so radiance and event counts equal the oracle's."""
    monkeypatch.setenv("SURF_LDS_LIGHTBLAS", staged)
    W, H, F = 96, 64, 4
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(F, 0, 0)
    g = r.accumulator()
    st = r.stats()
    recs, tris = r.debug_connect_staging()
    r.close()
    if staged == "1":       # the staged walk must have run, on a BLAS deeper than a root leaf
        assert recs > 8 and tris > 0, (recs, tris)
    else:
        assert (recs, tris) == (0, 0)
    oracle.set_zero_cutoff(True)
    try:
        c, cnt, _ = oracle_scene.render(W, H, F)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c, f"light BLAS staged={staged}")
    _assert_counts(st, cnt)


@pytest.mark.parametrize("cutoff", [None, True], ids=["reference-no-cutoff", "cutoff-on-both"])
def test_render_spp4_per_frame_bitexact(oracle_scene, product_scene, cutoff):
    """Multi-sample frames (config().samplesPerFrame = 4; renderer.cpp:160-188):
    frame f is seeded once per pixel from the running sample count 4f, and its
    four samples run in sequence, each drawing jitter, lens sample and path from
    the RNG state the previous sample's path left.  96x64, 3 frames: the GPU
    (sample chains continued by k_shade and the drain) equals the oracle bit for
    bit with equal event counts -- in reference semantics (the automatic
    default: no throughput cutoff for multi-sample frames) and with the cutoff
    on both sides."""
    W, H, F, K = 96, 64, 3, 4
    r = surf_amd.Renderer(product_scene, W, H)
    if cutoff is not None:
        r.set_zero_cutoff(cutoff)
    r.render(F, 0, 0, spp=K)
    g = r.accumulator()
    st = r.stats()
    r.close()
    assert np.all(g[..., 3] == F * K) and st["samples"] == W * H * F * K
    oracle.set_zero_cutoff(bool(cutoff))
    try:
        c, cnt, _ = oracle_scene.render(W, H, F, spp=K)
        one, _, _ = oracle_scene.render(W, H, F * K)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c, f"{F} frames x {K} samples, cutoff {cutoff}")
    _assert_counts(st, cnt)
    assert not np.array_equal(c.view(np.uint32), one.view(np.uint32)), "chained samples must differ from 1-spp frames"


@pytest.mark.parametrize("policy,coop,engine", [((1 << 30, 0, 8), 1 << 30, "pair"), ((1 << 30, 0, 8), 1 << 30, "coop"),
                                                ((0, 8, 4), 0, "lanes"), ((1, 0, 0), 0, "lanes")],
                         ids=["pair-from-start", "coop-from-start", "8-lanes-staged", "wavefront-to-end"])
def test_spp_chains_through_drain_bitexact(oracle_scene, product_scene, policy, coop, engine, monkeypatch):
    """A frame's sample chain continued inside every drain engine (the next
    camera sample drawn on the lane or wave that ended the previous one), and
    the drop-in loop (one frame of 3 samples per render() call, each call's
    first sample index the running count): equal to the oracle bit for bit."""
    monkeypatch.setenv("SURF_TAIL_PAIR", "0" if engine == "coop" else "1")
    W, H, F, K = 64, 48, 4, 3
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=4096)
    r.set_tail_policy(*policy)
    r.set_tail_coop(coop)
    r.render(F, 0, 0, spp=K)
    g = r.accumulator()
    st = r.stats()
    r.clear_accumulator()
    for f in range(F):                    # main.cpp's loop: render() per frame
        r.render(1, f * K, 0, spp=K)
    g2 = r.accumulator()
    r.close()
    c, cnt, _ = oracle_scene.render(W, H, F, spp=K)
    _assert_bitexact(g, c, f"spp {K} drain {engine} {policy}")
    _assert_counts(st, cnt)
    _assert_bitexact(g2, c, f"spp {K} one frame per call, drain {engine}")


def test_spp_window_and_offset_bitexact(oracle_scene, product_scene):
    """Multi-sample frames through a radiance window of two frames (6 passes,
    frame_batch a multiple of spp) and from a sample offset (first sample index
    7, as after 7 earlier samples): the window's slot reuse and the seeds."""
    W, H, K = 48, 40, 3
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=2048, frame_batch=2 * K)
    r.render(5, 7, 0, spp=K)
    g = r.accumulator()
    r.close()
    c, _, _ = oracle_scene.render(W, H, 5, first_frame=7, spp=K)
    _assert_bitexact(g, c, "5 frames x 3 samples from sample 7 through a 6-pass window")
    bad = surf_amd.Renderer(product_scene, W, H, frame_batch=4)
    with pytest.raises(surf_amd.SurfError):
        bad.render(2, 0, 0, spp=3)        # a window of 4 passes cannot hold whole 3-sample frames
    bad.close()


def test_render_c1_256x256x16_bitexact(oracle_scene, product_scene):
    g, c, stats, cnt, _ = _render_both(oracle_scene, product_scene, 256, 256, 16)
    _assert_bitexact(g, c, "C1 256x256x16")
    _assert_counts(stats, cnt)


def test_render_first_frame_offset(oracle_scene, product_scene):
    g, c, stats, cnt, _ = _render_both(oracle_scene, product_scene, 48, 40, 3, first=37)
    _assert_bitexact(g, c, "frames 37..39")


def test_segment_cap_c2_semantics(oracle_scene, product_scene):
    g, c, stats, cnt, _ = _render_both(oracle_scene, product_scene, 64, 48, 3, max_seg=8)
    _assert_bitexact(g, c, "max 8 segments")
    _assert_counts(stats, cnt)


def test_c2_1280x720_cap8_rows(oracle_scene, product_scene):
    """C2 at its full resolution (BASELINE.json configs[1]: 1280x720, at most 8
    segments): the GPU renders the whole frame as one stream (the cap ends
    paths in k_shade, the drain included), the oracle three bands of rows in
    reference semantics; bit for bit, and the event counts of the bands'
    paths are consistent (every capped path still adds its radiance)."""
    W, H, F = 1280, 720, 4
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(F, 0, 8)
    g = r.accumulator()
    st = r.stats()
    r.close()
    assert np.all(g[..., 3] == F)
    assert st["max_segments"] <= 8
    for a, b in ((0, 8), (356, 364), (712, 720)):
        c, _, _ = oracle_scene.render(W, H, F, rows=(a, b), max_segments=8)
        _assert_bitexact(g[a:b], c, f"C2 1280x720x{F} cap 8 rows {a}..{b - 1}")


def test_window_grows_with_stream_bitexact(oracle_scene, product_scene):
    """The radiance ring follows the requested stream: a first 2-frame stream
    sizes it at the floor (256 passes), a later 300-frame stream grows it (the
    graph is re-captured on the new ring), and a stream opened by a one-frame
    call (the drop-in loop) gets the loop floor, 4096; every render equals the
    oracle's."""
    W, H = 16, 12
    r = surf_amd.Renderer(product_scene, W, H)
    assert r.stats()["frame_window"] == 0
    r.render(2, 0, 0)
    g1 = r.accumulator()
    assert r.stats()["frame_window"] == 256
    r.clear_accumulator()
    r.render(300, 0, 0)
    g2 = r.accumulator()
    assert r.stats()["frame_window"] == 300
    r.close()
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(1, 0, 0)
    assert r.stats()["frame_window"] == 4096
    g3 = r.accumulator()
    r.close()
    oracle.set_zero_cutoff(True)
    try:
        c1, _, _ = oracle_scene.render(W, H, 2)
        c2, _, _ = oracle_scene.render(W, H, 300)
        c3, _, _ = oracle_scene.render(W, H, 1)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g1, c1, "2-frame stream")
    _assert_bitexact(g2, c2, "300-frame stream after the ring grew")
    _assert_bitexact(g3, c3, "one-frame stream on the 4096-slot ring")


def test_full_resolution_rows(oracle_scene, product_scene):
    """1280x720 (C2/C3 resolution): GPU renders the whole frame, the oracle a band of rows."""
    W, H, F = 1280, 720, 2
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(F, 0, 0)
    g = r.accumulator()
    c, _, _ = oracle_scene.render(W, H, F, rows=(356, 364))
    _assert_bitexact(g[356:364], c, "1280x720 rows 356..363")
    assert np.isfinite(g).all() and np.all(g[..., 3] == F)


def test_c3_subset_1280x720x16_bitexact(oracle_scene, product_scene):
    """SURVEY.md 8d's C3 parity subset: 1280x720 at 16 spp, unbounded + RR,
    the GPU rendering the whole frame as one stream (its drain included), the
    oracle three bands of rows (top, middle, bottom), compared bit for bit."""
    W, H, F = 1280, 720, 16
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(F, 0, 0)
    g = r.accumulator()
    assert np.all(g[..., 3] == F)
    for a, b in ((0, 8), (356, 364), (712, 720)):
        c, _, _ = oracle_scene.render(W, H, F, rows=(a, b))
        _assert_bitexact(g[a:b], c, f"1280x720x16 rows {a}..{b - 1}")
    r.close()


def test_pool_and_batch_invariance(product_scene):
    """Compaction/regeneration/batching must not change any sample."""
    W, H, F = 80, 60, 5
    ref = surf_amd.Renderer(product_scene, W, H)
    ref.render(F)
    a = ref.accumulator()
    small = surf_amd.Renderer(product_scene, W, H, pool_capacity=1000, frame_batch=2)
    small.render(F)
    b = small.accumulator()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    again = surf_amd.Renderer(product_scene, W, H)
    again.render(2)
    again.render(3, first_frame=2)
    assert np.array_equal(a.view(np.uint32), again.accumulator().view(np.uint32))
    # the drop-in loop: one frame per render() call (main.cpp:381-446, short replays)
    loop = surf_amd.Renderer(product_scene, W, H)
    for f in range(F):
        loop.render(1, first_frame=f)
    assert np.array_equal(a.view(np.uint32), loop.accumulator().view(np.uint32))


@pytest.mark.parametrize("shards,block", [(2, 0), (3, 16), (4, 8)])
def test_row_shards_assemble_bitexact(product_scene, shards, block):
    W, H, F = 96, 72, 3
    full = surf_amd.Renderer(product_scene, W, H)
    full.render(F)
    a = full.accumulator()
    specs = [surf_amd.ShardSpec(s, shards, block) for s in range(shards)]
    parts = []
    for sp in specs:
        r = surf_amd.Renderer(product_scene, W, H, shard=sp)
        r.render(F)
        parts.append(r.accumulator())
    b = surf_amd.assemble_shards(W, H, parts, specs)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_finalize_rgba8_matches_oracle(product_scene):
    W, H, F = 64, 32, 3
    r = surf_amd.Renderer(product_scene, W, H)
    r.render(F)
    acc = r.accumulator()
    got = r.finalize_rgba8().reshape(-1)
    want = oracle.finalize_rgba8(acc, np.float32(1.0) / np.float32(F))
    assert np.array_equal(got, want)
    st = r.stats()
    e = np.float32(0.0)
    for p in acc.reshape(-1, 4) * (np.float32(1.0) / np.float32(F)):
        e = np.float32(e + np.float32(np.float32(p[0] + p[1]) + p[2]))
    assert np.float32(st["energy"]) == e, "Lumen energy: serial pixel-order sum (renderer.cpp:191-201)"
    # display step (fs_quad.frag:22-24): sqrt of the UNORM8 finalize image, back to UNORM8
    disp = r.display_rgba8().reshape(-1)
    ch = np.stack([(want >> (8 * k)) & 0xFF for k in range(4)], 1).astype(np.float32)
    g = np.rint(np.sqrt(ch / np.float32(255.0)) * np.float32(255.0)).clip(0, 255).astype(np.uint32)
    assert np.array_equal(disp, g[:, 0] | (g[:, 1] << 8) | (g[:, 2] << 16) | (g[:, 3] << 24))


def test_cutoff_off_matches_reference_counts(oracle_scene, product_scene):
    """With the cutoff disabled the GPU traces exactly the reference's segments."""
    W, H, F = 64, 48, 2
    r = surf_amd.Renderer(product_scene, W, H)
    r.set_zero_cutoff(False)
    r.render(F)
    g = r.accumulator()
    st = r.stats()
    c, cnt, _ = oracle_scene.render(W, H, F)
    _assert_bitexact(g, c, "cutoff off")
    _assert_counts(st, cnt)


def test_deterministic_rerun(product_scene):
    r = surf_amd.Renderer(product_scene, 64, 64)
    r.render(2)
    a = r.accumulator()
    r.clear_accumulator()
    r.render(2)
    assert np.array_equal(a.view(np.uint32), r.accumulator().view(np.uint32))


def test_animation_update_render_bitexact():
    """Row f3: GPUScene::update (rotate instance 3, TLAS refit) then the
    instance/TLAS re-upload (surf_update_instances): renders before and after
    match the oracle's, bit for bit, and the re-upload equals a fresh upload."""
    W, H, F = 48, 32, 2
    o = oracle.OracleScene()
    p = surf_amd.Scene.indoor()
    try:
        r = surf_amd.Renderer(p, W, H)
        r.set_zero_cutoff(False)
        r.render(F, 0, 0)
        c, _, _ = o.render(W, H, F)
        assert np.array_equal(r.accumulator().view(np.uint32), c.view(np.uint32))
        for dt in (0.7, 2.1):
            o.update(dt)
            p.update(dt)
            r.update_instances(p)
            r.clear_accumulator()
            r.render(F, 4, 0)
            g = r.accumulator()
            c, _, _ = o.render(W, H, F, first_frame=4)
            _assert_bitexact(g, c, f"after update dt={dt}")
            fresh = surf_amd.Renderer(p, W, H)
            fresh.set_zero_cutoff(False)
            fresh.render(F, 4, 0)
            assert np.array_equal(fresh.accumulator().view(np.uint32), g.view(np.uint32))
            fresh.close()
        r.close()
    finally:
        o.close()
        p.close()


def test_dropin_loop_lag_across_reads_and_updates():
    """The interactive loop (main.cpp:381-446) on the lagged stream: one-frame
    render() calls return with up to a pool of their samples unissued; a read
    in the middle (stats) drains exactly the frames requested so far; an
    animation update drains the pending samples under the old transforms
    before re-uploading; after the clear the loop goes on.  Every observed
    accumulator equals the oracle's, bit for bit."""
    W, H = 48, 32
    o = oracle.OracleScene()
    p = surf_amd.Scene.indoor()
    try:
        r = surf_amd.Renderer(p, W, H)
        r.set_zero_cutoff(False)
        for f in range(3):
            r.render(1, first_frame=f)
        assert r.stats()["samples"] == W * H * 3
        c, _, _ = o.render(W, H, 3)
        _assert_bitexact(r.accumulator(), c, "3 lagged one-frame calls")
        for f in range(3, 6):
            r.render(1, first_frame=f)
        p.update(0.7)
        r.update_instances(p)                 # the pending frames 3..5 run under the old transforms
        c, _, _ = o.render(W, H, 6)
        _assert_bitexact(r.accumulator(), c, "6 one-frame calls, drained by the update")
        o.update(0.7)
        r.clear_accumulator()
        for f in range(4):
            r.render(1, first_frame=6 + f)
        c, _, _ = o.render(W, H, 4, first_frame=6)
        _assert_bitexact(r.accumulator(), c, "4 one-frame calls after the update")
        r.close()
    finally:
        o.close()
        p.close()


@pytest.mark.parametrize("pipeline", ["1", "0"], ids=["replays-in-flight", "synchronous"])
def test_dropin_loop_pipelined_bitexact(pipeline, monkeypatch):
    """A long drop-in loop (one frame per call, far past the lag's pool): each
    call queues its replays before reading the previous one's counters and may
    return with replays in flight (SURF_PIPELINE, default on); a read in the
    middle and at the end drains them.  The accumulators equal the oracle's
    bit for bit, and every call's device time is counted once."""
    monkeypatch.setenv("SURF_PIPELINE", pipeline)
    W, H, N1, N2 = 32, 24, 17, 23
    o = oracle.OracleScene()
    p = surf_amd.Scene.indoor()
    try:
        r = surf_amd.Renderer(p, W, H)
        r.set_zero_cutoff(False)
        for f in range(N1):
            r.render(1, first_frame=f)
        c1, _, _ = o.render(W, H, N1)
        _assert_bitexact(r.accumulator(), c1, f"{N1} one-frame calls (pipeline={pipeline})")
        for f in range(N1, N1 + N2):
            r.render(1, first_frame=f)
        st = r.stats()
        assert st["samples"] == W * H * (N1 + N2) and st["ms_total"] > 0.0
        c2, _, _ = o.render(W, H, N1 + N2)
        _assert_bitexact(r.accumulator(), c2, f"{N1 + N2} one-frame calls (pipeline={pipeline})")
        r.close()
    finally:
        o.close()
        p.close()


def test_c5_deep_bvh_bitexact():
    """C5: 10.2M-triangle lattice BLAS (HBM-resident, depth 36,
    built by the parallel builder) -- hit records, a small render and three row
    bands of a full 1280x720 render equal the oracle's, whose BLAS comes from
    the reference's sequential build."""
    W, H, F = 64, 48, 2
    o = oracle.OracleScene(variant=1)
    p = surf_amd.Scene.indoor(variant=1)
    try:
        r = surf_amd.Renderer(p, W, H)
        (eo, ed), _ = o.record_rays(W, H, 0, 0, W * H)
        g = r.trace_closest(eo, ed)
        c = o.trace_closest(eo, ed)
        for k in range(5):
            assert np.array_equal(np.asarray(g[k]).view(np.uint32), np.asarray(c[k]).view(np.uint32)), f"hit field {k}"
        r.set_zero_cutoff(False)
        r.render(F, 0, 0)
        c, _, _ = o.render(W, H, F)
        _assert_bitexact(r.accumulator(), c, "C5 64x48x2")
        r.close()
        # C5 at its full resolution (1280x720): the whole frame on the GPU (drain
        # included), one band of rows per third of the image on the oracle
        W, H = 1280, 720
        r = surf_amd.Renderer(p, W, H)
        r.render(F, 0, 0)
        g = r.accumulator()
        r.close()
        assert np.all(g[..., 3] == F)
        for a in (120, 360, 600):
            c, _, _ = o.render(W, H, F, rows=(a, a + 4))
            _assert_bitexact(g[a:a + 4], c, f"C5 1280x720x{F} rows {a}..{a + 3}")
    finally:
        o.close()
        p.close()


@pytest.mark.parametrize("variant", [2, 3], ids=["tlas-51-instances-lds-tables", "tlas-91-instances-global-tables"])
def test_general_tlas_bitexact(variant):
    """The interior-node TLAS walk (BvhTLAS::intersect / intersectAny,
    bvh.cpp:654-778; ray_extend.comp:105-165): near-first child order, the far
    child pushed, leaf instance loops, on scenes whose TLAS splits (depth > 0)
    -- with <= 64 instances (LDS trace/shading tables) and > 64 (global
    tables), in the lane traversal and in the drain's wave traversal.  Hit
    records, any-hit and a render (its drain on the cooperative engine) with
    its event counts equal the oracle's bit for bit."""
    o = oracle.OracleScene(variant=variant)
    p = surf_amd.Scene.indoor(variant=variant)
    try:
        assert p.bvh_depths()[0] > 0, "TLAS did not split"
        W, H = 64, 48
        r = surf_amd.Renderer(p, W, H, frame_batch=16)
        with pytest.raises(surf_amd.SurfError):
            r.set_trace_mode(2)           # modes are 0 (lane) and 1 (wave)
        (eo, ed), (so, sd, st) = o.record_rays(W, H, 0, 0, W * H)
        rng = np.random.default_rng(7)
        ro = rng.uniform([-9, -0.9, -9], [9, 8.9, 9], size=(20000, 3)).astype(np.float32)
        rd = rng.normal(size=(20000, 3)).astype(np.float32)
        rd /= np.linalg.norm(rd, axis=1, keepdims=True)
        oo, dd = np.concatenate([eo, so, ro]), np.concatenate([ed, sd, rd])
        cpu = o.trace_closest(oo, dd)
        cpu_any = o.trace_any(so, sd, st)
        # mode 0: one ray per lane; mode 1: one ray per wave (the drain's walk,
        # here the general-TLAS wave walk: traceWaveTlas)
        for mode in (0, 1):
            r.set_trace_mode(mode)
            gpu = r.trace_closest(oo, dd)
            for n, g, c in zip(["t", "u", "v", "inst", "prim"], gpu, cpu):
                bad = np.nonzero(g.view(np.uint32) != c.view(np.uint32))[0]
                assert len(bad) == 0, f"mode {mode} {n}: {len(bad)} of {len(g)} differ, first {bad[:5]}"
            assert len(np.unique(gpu[3][gpu[3] != UNSET])) > 30, "rays should hit many instances"
            assert len(so) > 500 and np.array_equal(r.trace_any(so, sd, st), cpu_any), f"mode {mode} any-hit"
        r.set_trace_mode(0)
        r.render(3, 0, 0)
        g = r.accumulator()
        stats = r.stats()
        r.close()
        assert stats["tail_survivors"] > 0, "the drain should run the cooperative (one path per wave) engine"
        oracle.set_zero_cutoff(True)
        try:
            c, cnt, _ = o.render(W, H, 3)
        finally:
            oracle.set_zero_cutoff(False)
        _assert_bitexact(g, c, f"general TLAS variant {variant}")
        _assert_counts(stats, cnt)
    finally:
        o.close()
        p.close()


def test_c4_row_shards_1080p_bitexact(oracle_scene, product_scene):
    """C4 geometry (1920x1080): the 8 row shards of an 8-GPU run
    (rows interleaved one by one, ShardSpec(k, 8, 1)) rendered in turn on one
    GPU.  Two rows of every shard equal the oracle's bit for bit, and the
    assembled frame equals the 1-GPU frame bit for bit."""
    W, H, F, G = 1920, 1080, 4, 8
    full = surf_amd.Renderer(product_scene, W, H, frame_batch=16)
    full.render(F, 0, 0)
    a = full.accumulator()
    full.close()
    specs = [surf_amd.ShardSpec(k, G, 1) for k in range(G)]
    parts = []
    oracle.set_zero_cutoff(True)
    try:
        for k, spec in enumerate(specs):
            r = surf_amd.Renderer(product_scene, W, H, shard=spec, frame_batch=16)
            r.render(F, 0, 0)
            part = r.accumulator()
            r.close()
            rows = surf_amd.shard_rows(H, spec)
            assert part.shape == (len(rows), W, 4) and np.all(part[..., 3] == F)
            for j in (len(rows) // 2, len(rows) // 2 + 7):    # rows near the glass Suzanne band
                c, _, _ = oracle_scene.render(W, H, F, rows=(int(rows[j]), int(rows[j]) + 1))
                _assert_bitexact(part[j:j + 1], c, f"C4 shard {k} row {rows[j]}")
            parts.append(part)
    finally:
        oracle.set_zero_cutoff(False)
    b = surf_amd.assemble_shards(W, H, parts, specs)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "8-shard assembly differs from the 1-GPU frame"


def test_stream_past_window_bitexact(oracle_scene, product_scene):
    """A sample stream longer than the frame window (here 3 frames) issues frame
    f only once frame f - window is accumulated; the radiance slots are reused
    and the result is unchanged (bit-exact vs the oracle)."""
    W, H, F = 96, 64, 10
    r = surf_amd.Renderer(product_scene, W, H, pool_capacity=4096, frame_batch=3)
    r.render(4, 0, 0)
    r.render(F - 4, 4, 0)
    g = r.accumulator()
    r.close()
    oracle.set_zero_cutoff(True)
    try:
        c, _, _ = oracle_scene.render(W, H, F)
    finally:
        oracle.set_zero_cutoff(False)
    _assert_bitexact(g, c, "stream of 10 frames through a 3-frame window")
