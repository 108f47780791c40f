"""Finds a camera sample whose GPU result differs from the C oracle's (a debugging
aid; the oracle is the checker here, as in tests/).

    python tools/rr_find.py [scene W H spp rr_depth row_step russian_roulette]

1. every row_step-th row rendered alone on the GPU and by the oracle: the rows
   whose framebuffers differ (per-pixel relative L2 > 1e-4);
2. in the first such row, bisection over the row's samples (BDPT_SAMPLE_RANGE on
   the GPU, Scene.render_row_samples on the oracle) down to one sample;
3. that sample's Li and splats from the oracle, the GPU single-sample API and
   the frame kernel.
"""
import concurrent.futures as cf
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, p) for p in ("bidirectional-path-tracing_amd", "scenes", "oracle", "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bdpt_amd  # noqa: E402
import oracle as O  # noqa: E402
import variants  # noqa: E402

a = sys.argv[1:]
scene = a[0] if a else "hardlight"
W, H, spp, rr, step, rrm = (int(x) for x in (a[1:7] if len(a) >= 7 else (512, 512, 1024, 2, 20, 1)))
cam = variants.SCENES[scene]["camera"]
cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr,
                      russian_roulette=bdpt_amd.RR_LUMINANCE if rrm else bdpt_amd.RR_NONE)
it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(scene)), cfg)
it.init()
sc = O.Scene(variants.obj_path(scene))
p = O.make_params(cam, W, H, spp, rr, russian_roulette=rrm)
fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream


def gpu_row(row, rng=None):
    if rng:
        os.environ["BDPT_DEBUG_KNOBS"] = "1"
        os.environ["BDPT_SAMPLE_RANGE"] = f"{rng[0]},{rng[1]}"
    fb.zero_()
    it.render_device(fb.data_ptr(), stream, row_offset=row, row_stride=H)
    st = it.stats()
    os.environ.pop("BDPT_SAMPLE_RANGE", None)
    assert st["schedule_errors"] == 0 and st["capped_samples"] == 0, st
    return fb.cpu().numpy().astype(np.float64).reshape(-1, 3)


def err(g, r):
    r = r.astype(np.float64).reshape(-1, 3)
    e = np.linalg.norm(g - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)
    return e


def log(**kw):
    print(json.dumps(kw), flush=True)


t0 = time.time()
rows = list(range(0, H, step))
with cf.ThreadPoolExecutor(16) as ex:  # the oracle releases the GIL in its C calls
    ref = dict(zip(rows, ex.map(lambda r: sc.render_row_samples(p, r, 0, W * spp), rows)))
bad = []
for r in rows:
    e = err(gpu_row(r), ref[r])
    if e.max() > 1e-4:
        bad.append(r)
    log(row=r, max_rel_l2=float(e.max()), over=int((e > 1e-4).sum()))
log(bad_rows=bad, seconds=round(time.time() - t0, 1))
if not bad:
    sys.exit(0)
row = bad[0]
lo, hi = 0, W * spp
while hi - lo > 1:
    mid = (lo + hi) // 2
    e = err(gpu_row(row, (lo, mid)), sc.render_row_samples(p, row, lo, mid))
    if e.max() > 1e-4:
        hi = mid
    else:
        lo = mid
    log(range=[lo, hi], left_bad=bool(e.max() > 1e-4))
j, k = lo // spp, lo % spp
pixel = row * W + j
Li_o, fb_o = sc.sample(p, pixel, k)
g = gpu_row(row, (lo, lo + 1))
ref1 = fb_o.reshape(-1, 3).astype(np.float64).copy()
ref1[pixel] += Li_o / spp
e = err(g, ref1)
diff = np.nonzero(e > 1e-4)[0]
log(sample={"row": row, "j": j, "k": k, "pixel": pixel}, oracle_Li=Li_o.tolist(),
    differing_pixels=diff[:20].tolist(), n_differing=int(len(diff)),
    gpu=[g[i].tolist() for i in diff[:5]], oracle=[ref1[i].tolist() for i in diff[:5]])
from test_gpu_parity import driver_ray  # noqa: E402

ray, sampler = driver_ray(p, scene, pixel, k)
Li_s = it.render(ray, sampler)
log(single_sample_api_Li=[float(x) for x in Li_s], matches_oracle=bool(np.allclose(Li_s, Li_o, rtol=1e-6, atol=0)))
O.walk_stats(True)
sc.sample(p, pixel, k)
log(oracle_walk=O.walk_stats(True))
