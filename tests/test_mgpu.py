"""Multi-GPU image assembly of libsurf_mgpu.so on CPU: the root's
row un-permute (surf_mgpu_assemble), the shard row rule it shares with
surf_create_sharded (surf_shard_row_list), and the host RGBA8 packing of an
assembled frame (surf_pack_rgba8) against the oracle's RgbaToU32.  The RCCL
gather itself runs in the -m gpu test of examples/render_indoor_mgpu."""
import numpy as np
import pytest

import oracle
import surf_amd


@pytest.mark.parametrize("height,shards,block", [(48, 2, 16), (37, 3, 0), (1080, 8, 1), (720, 5, 7), (5, 8, 1)])
def test_shard_row_list_matches_rule(height, shards, block):
    import ctypes as C
    lib = surf_amd.load()
    seen = []
    for k in range(shards):
        n = C.c_uint32()
        assert lib.surf_shard_row_list(height, k, shards, block, None, C.byref(n)) == 0
        rows = np.zeros(max(1, n.value), np.uint32)
        assert lib.surf_shard_row_list(height, k, shards, block, rows.ctypes.data, C.byref(n)) == 0
        want = surf_amd.shard_rows(height, surf_amd.ShardSpec(k, shards, block))
        assert np.array_equal(rows[: n.value], want)
        seen.extend(rows[: n.value].tolist())
    assert sorted(seen) == list(range(height))
    assert lib.surf_shard_row_list(height, shards, shards, block, None, C.byref(C.c_uint32())) == -1


@pytest.mark.parametrize("height,shards,block", [(48, 2, 16), (37, 3, 0), (72, 4, 8), (11, 8, 1)])
def test_native_assemble_matches_python(height, shards, block):
    W = 13
    rng = np.random.default_rng(height * 31 + shards)
    specs = [surf_amd.ShardSpec(k, shards, block) for k in range(shards)]
    parts = [rng.standard_normal((len(surf_amd.shard_rows(height, s)), W, 4)).astype(np.float32) for s in specs]
    want = surf_amd.assemble_shards(W, height, parts, specs)
    maxr = max(len(p) for p in parts)
    slabs = np.full((shards, maxr, W, 4), np.nan, np.float32)      # padding rows must be ignored
    for k, p in enumerate(parts):
        slabs[k, : len(p)] = p
    got = surf_amd.assemble_slabs(W, height, shards, block, slabs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    with pytest.raises(surf_amd.SurfError):
        surf_amd.assemble_slabs(W, height, shards, block, slabs[:, :0] if maxr else slabs)


def test_assemble_without_mgpu_library(monkeypatch):
    """A torch.distributed gather needs no RCCL library of ours: without
    libsurf_mgpu.so the un-permute runs in numpy, with the same result."""
    W, height, shards, block = 9, 37, 3, 4
    rng = np.random.default_rng(5)
    slabs = rng.standard_normal((shards, 13, W, 4)).astype(np.float32)
    # the expected frame from the shard row rule itself, not from assemble_slabs
    # (which would take the fallback too if the library were missing)
    want = np.zeros((height, W, 4), np.float32)
    for k in range(shards):
        rows = surf_amd.shard_rows(height, surf_amd.ShardSpec(k, shards, block))
        want[rows] = slabs[k, : len(rows)]
    assert np.array_equal(surf_amd.assemble_slabs(W, height, shards, block, slabs).view(np.uint32), want.view(np.uint32))

    def missing():
        raise OSError("libsurf_mgpu.so not built")
    monkeypatch.setattr(surf_amd, "load_mgpu", missing)
    got = surf_amd.assemble_slabs(W, height, shards, block, slabs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    with pytest.raises(ValueError):
        surf_amd.assemble_slabs(W, height, shards, block, slabs[:, :5])


def test_ctx_device_getter_is_exported():
    import ctypes as C
    lib = surf_amd.load()
    dev = C.c_int(-7)
    assert lib.surf_get_device(None, C.byref(dev)) == -1   # SURF_ERR_INVALID
    assert dev.value == -7


def test_host_pack_rgba8_matches_oracle():
    rng = np.random.default_rng(3)
    acc = (rng.standard_normal((4096, 4)) * 3.0).astype(np.float32)
    acc[:8] = [[np.inf, -np.inf, np.nan, 0], [1e30, -1e30, 0.5, 255], [0.5 / 255, 1.5 / 255, 2.5 / 255, 1],
               [1, 1, 1, 1], [0, 0, 0, 0], [-0.0, 2, 3, 4], [254.5 / 255, 255.5 / 255, 1e-40, 7], [3, 3, 3, 3]]
    for spp in (1, 3, 16):
        got = surf_amd.pack_rgba8(acc, spp)
        want = oracle.finalize_rgba8(acc, np.float32(1.0) / np.float32(spp))
        assert np.array_equal(got, want), spp
        disp = surf_amd.pack_rgba8(acc, spp, display=True)
        ch = np.stack([(want >> (8 * k)) & 0xFF for k in range(4)], 1).astype(np.float32)
        g = np.rint(np.sqrt(ch / np.float32(255.0)) * np.float32(255.0)).clip(0, 255).astype(np.uint32)
        assert np.array_equal(disp, g[:, 0] | (g[:, 1] << 8) | (g[:, 2] << 16) | (g[:, 3] << 24))
