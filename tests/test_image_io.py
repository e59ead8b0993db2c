"""Image output: the PPM / PNG writers of the C-ABI
(surf_write_ppm, surf_write_png) produce files a standard decoder reads back
pixel for pixel.  CPU only (host code)."""
import numpy as np
import pytest

import surf_amd

PIL = pytest.importorskip("PIL.Image")


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 2 ** 32, (h, w), dtype=np.uint64).astype(np.uint32)


@pytest.mark.parametrize("h,w", [(1, 1), (7, 13), (72, 128)])
def test_png_roundtrip(tmp_path, h, w):
    img = _img(h, w, h * w)
    path = str(tmp_path / "x.png")
    surf_amd.write_image(path, img)
    got = np.asarray(PIL.open(path).convert("RGBA"), dtype=np.uint32)
    want = np.stack([(img >> (8 * k)) & 0xFF for k in range(4)], -1)
    assert got.shape == (h, w, 4) and np.array_equal(got, want)


def test_ppm_roundtrip(tmp_path):
    img = _img(33, 17, 5)
    path = str(tmp_path / "x.ppm")
    surf_amd.write_image(path, img)
    got = np.asarray(PIL.open(path).convert("RGB"), dtype=np.uint32)
    want = np.stack([(img >> (8 * k)) & 0xFF for k in range(3)], -1)
    assert np.array_equal(got, want)


def test_bad_arguments(tmp_path):
    with pytest.raises(surf_amd.SurfError):
        surf_amd.write_image(str(tmp_path / "no_such_dir" / "x.png"), _img(2, 2, 1))
