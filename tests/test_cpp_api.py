"""The drop-in C++ API end to end: examples/render_indoor.cpp builds the scene,
BVHs, camera and WaveFrontRenderer exactly as the reference's main.cpp does
(sources/main.cpp:141-442) and writes the presented image (the RGBA8 finalize
image through fs_quad.frag's sqrt gamma).  Its pixels must equal the same
presentation of the CPU oracle's accumulator, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "surf-path-tracer_amd", "build", "render_indoor")


def present(acc, frames):
    """wavefront_finalize.comp + RgbaToU32 (oracle), then fs_quad.frag: sqrt of
    the UNORM8 value, back to UNORM8 (round to nearest even)."""
    h, w = acc.shape[:2]
    rgba = oracle.finalize_rgba8(acc, np.float32(1.0) / np.float32(frames))
    ch = np.stack([(rgba >> (8 * k)) & 0xFF for k in range(3)], 1).astype(np.float32)
    g = np.rint(np.sqrt(ch / np.float32(255.0)) * np.float32(255.0)).clip(0, 255)
    return g.astype(np.uint8).reshape(h, w, 3)


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    head, rest = data.split(b"\n", 3)[:3], data.split(b"\n", 3)[3]
    w, h = map(int, head[1].split())
    return np.frombuffer(rest, np.uint8).reshape(h, w, 3)


def test_example_binary_built():
    assert os.path.exists(EXE), "render_indoor not built (make -C surf-path-tracer_amd)"


@pytest.mark.gpu
def test_cpp_api_render_matches_oracle(oracle_scene, tmp_path):
    W, H, F = 64, 48, 3
    out = tmp_path / "indoor.ppm"
    r = subprocess.run([EXE, os.path.join(REPO, "assets"), str(W), str(H), str(F), str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if "Mrays/s" in l]
    assert len(lines) == F and f"{F:05d} samples" in lines[-1]
    acc, _, _ = oracle_scene.render(W, H, F)
    assert np.array_equal(read_ppm(out), present(acc, F))
    loop = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(loop) == 1 and '"frames": %d' % F in loop[0] and '"lumen_output": false' in loop[0]


@pytest.mark.gpu
def test_cpp_api_lumen_output(oracle_scene, tmp_path):
    """WF_LUMEN_OUTPUT (renderer.cpp:31,955-969): with lumenOutput, frameInfo()
    reports the serial pixel-order energy of the frames rendered so far."""
    W, H, F = 48, 32, 3
    out = tmp_path / "indoor.ppm"
    r = subprocess.run([EXE, os.path.join(REPO, "assets"), str(W), str(H), str(F), str(out), "--lumen"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if "Mrays/s" in l]
    assert len(lines) == F
    for f, line in enumerate(lines, start=1):
        acc, _, _ = oracle_scene.render(W, H, f)
        e = np.float32(0.0)
        for p in acc.reshape(-1, 4) * (np.float32(1.0) / np.float32(f)):
            e = np.float32(e + np.float32(np.float32(p[0] + p[1]) + p[2]))
        assert line.endswith("%010.2f Lumen" % e), (line, e)


@pytest.mark.gpu
def test_cpp_api_samples_per_frame(oracle_scene, tmp_path):
    """RendererConfig::samplesPerFrame = 3 (the UI's spp slider, main.cpp:415):
    each render() adds one frame of 3 samples per pixel seeded once from the
    running sample count and continuing one RNG stream (renderer.cpp:160-188).
    The presented image equals the oracle's multi-sample frames bit for bit."""
    W, H, F, K = 48, 32, 3, 3
    out = tmp_path / "indoor_spp3.ppm"
    r = subprocess.run([EXE, os.path.join(REPO, "assets"), str(W), str(H), str(F), str(out), "--spp", str(K)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if "Mrays/s" in l]
    assert len(lines) == F and f"{F * K:05d} samples ({K} spp)" in lines[-1]
    acc, _, _ = oracle_scene.render(W, H, F, spp=K)
    assert np.array_equal(read_ppm(out), present(acc, F * K))
    loop = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(loop) == 1 and '"samples_per_frame": %d' % K in loop[0]


EXE_MGPU = os.path.join(REPO, "surf-path-tracer_amd", "build", "render_indoor_mgpu")


def test_mgpu_example_built():
    assert os.path.exists(EXE_MGPU), "render_indoor_mgpu not built (make -C surf-path-tracer_amd)"


@pytest.mark.gpu
@pytest.mark.parametrize("spp", [1, 2])
def test_cpp_mgpu_example_matches_oracle(oracle_scene, tmp_path, spp):
    """examples/render_indoor_mgpu (SURVEY.md 8e from C++): row shards on the
    visible GPUs (all of this box's: one; a node's eight run the same binary),
    each rendered on its own thread, one RCCL gather through libsurf_mgpu
    (ncclCommInitAll + ncclGather), the root's un-permute and the host RGBA8
    packing.  The presented image equals the oracle's bit for bit."""
    import surf_amd
    W, H, F = 64, 48, 3
    out = tmp_path / "indoor_mgpu.ppm"
    r = subprocess.run([EXE_MGPU, os.path.join(REPO, "assets"), str(W), str(H), str(F), str(out), "--gpus",
                        str(surf_amd.device_count()), "--row-block", "1", "--spp", str(spp)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1 and '"gather_ms"' in line[0]
    acc, _, _ = oracle_scene.render(W, H, F, spp=spp)
    assert np.array_equal(read_ppm(out), present(acc, F * spp))
