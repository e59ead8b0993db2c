"""C2 bench lines of gpurun_out/cap3 and the capped-path diagnostics on a small render."""
import json, sys
sys.path.insert(0, "surf-path-tracer_amd")
for f in ("c2_1", "c2_2"):
    d = json.load(open(f"gpurun_out/cap3/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["kernel_ms_profile_pass"]["ms_shade"])
import torch  # noqa: F401
import surf_amd
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 48)
r.render(2, 0, 8)
print(r.debug_capped())
