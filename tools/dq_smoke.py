"""Smallest run of the lane-decoupled build (BDPT_DQ=1): one 32x32x4 Caustic frame
against the C oracle, then the stats (python tools/dq_smoke.py [scene W H spp rr])."""
import json
import os
import sys

os.environ.setdefault("BDPT_DQ", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bidirectional-path-tracing_amd"), os.path.join(REPO, "scenes"),
                os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

import bdpt_amd  # noqa: E402
import oracle as O  # noqa: E402
import variants  # noqa: E402

a = sys.argv[1:]
name = a[0] if a else "caustic"
W, H, spp, rr = (int(x) for x in (a[1:5] if len(a) >= 5 else (32, 32, 4, 8)))
cam = variants.SCENES[name]["camera"]
cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(name)), cfg)
it.init()
fb = it.render_frame().reshape(-1, 3).astype(np.float64)
st = it.stats()
ref, _ = O.Scene(variants.obj_path(name)).render(O.make_params(cam, W, H, spp, rr))
ref = ref.reshape(-1, 3).astype(np.float64)
err = np.linalg.norm(fb - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-8)
print(json.dumps({"scene": name, "W": W, "H": H, "spp": spp, "rr": rr, "kernel": st["kernel"],
                  "kernel_ms": round(st["kernel_ms"], 3), "max_rel_l2": float(err.max()),
                  "ref_sum": float(ref.sum()), "gpu_sum": float(fb.sum())}), flush=True)
assert np.isfinite(fb).all() and err.max() <= 1e-4, "decoupled build differs from the oracle"
