"""Convert a little-endian PFM (as written by oracle/cpu_ref_bench) to a PNG
with the reference's present-pass gamma (sqrt, fs_quad.frag:22-24)."""
import sys
import numpy as np
from PIL import Image

def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4")
    return np.flipud(data.reshape(h, w, 3))

if __name__ == "__main__":
    img = read_pfm(sys.argv[1])
    img = np.sqrt(np.clip(img, 0.0, 1.0))
    Image.fromarray((img * 255.0 + 0.5).astype(np.uint8)).save(sys.argv[2])
