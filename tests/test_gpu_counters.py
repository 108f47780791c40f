"""The frame kernels walk the reference's paths: exact work counters.

Since round 5 the frame kernels without Russian roulette compute the weight-only
arithmetic (MIS recursion, pdf ratios, throughput, contributions) on the
hardware reciprocal / square root (`BDPT_FAST_WEIGHTS`). The claim
is that nothing that steers a path depends on it. The image tolerance alone
cannot show that (a path that diverged would move a pixel by less than 1e-4 at
high spp), so these tests compare the frame kernel's counting pass
(`FLAG_COUNT`, the same seeds and schedule) with the C oracle's per-frame
counters on the same (pixel, sample) set:

* RNG draws (every draw of bdpt.h in order), light vertices stored
  (bdpt.h:211-215) and light-vertex reads (one per connectVertices call,
  bdpt.h:145-150) must be equal: one differing direction, hit or roulette
  outcome changes them;
* closest-hit rays must equal the oracle's minus its re-traced primary rays
  (bdpt.h:70 repeats :225 with the same ray; the GPU reuses that hit);
* shadow rays and camera splats (visibility queries issued, unoccluded splats)
  must be equal too. A connection's cosine taken from a direction normalised
  on the fast path could in principle flip sign where its contribution is zero
  (DESIGN.md §1): the tests count such differences and allow none.
"""
import numpy as np
import pytest

import bdpt_amd
import oracle as O
import variants

pytestmark = pytest.mark.gpu

_scenes = {}


def gpu_counts(name, W, H, spp, rr, row_offset=0, row_stride=1, russian_roulette=0):
    if name not in _scenes:
        _scenes[name] = bdpt_amd.Scene(variants.obj_path(name))
    cam = bdpt_amd.Camera(**variants.SCENES[name]["camera"])
    cfg = bdpt_amd.Config(camera=cam, width=W, height=H, spp=spp, rr_depth=rr, russian_roulette=russian_roulette)
    it = bdpt_amd.BDPTIntegrator(_scenes[name], cfg)
    it.init()
    it.render_frame(row_offset=row_offset, row_stride=row_stride, flags=bdpt_amd.FLAG_COUNT)
    st = it.stats()
    return st["counters"], st["samples"], st["kernel"]


def oracle_counts(name, W, H, spp, rr, rows, russian_roulette=0):
    p = O.make_params(variants.SCENES[name]["camera"], W, H, spp, rr)
    p.russian_roulette = russian_roulette
    O.counters(True)
    _, n = O.Scene(variants.obj_path(name)).render(p, rows=rows)
    return O.counters(True), n


CASES = [
    # (scene, W, H, spp, rrDepth, row_offset, row_stride, russian_roulette)
    ("caustic", 64, 64, 16, 8, 0, 1, 0),        # G2: the default frame kernel (configs[1]'s scene and rrDepth)
    ("caustic", 512, 512, 16, 8, 200, 512, 0),  # one full-width row of the configs[1] frame (an L0-style shard)
    ("hardlight", 64, 64, 16, 2, 0, 1, 0),      # G3 at configs[2]'s rrDepth: the short-subpath build
    ("hardlight", 64, 64, 16, 8, 0, 1, 0),      # G3: the Phong lobe's fast powers (BDPT_FAST_POW)
    ("cbox_low", 64, 64, 4, 8, 0, 1, 0),        # G1
    ("caustic", 64, 64, 4, 8, 0, 1, 1),         # Russian roulette (IEEE weights; its throughput steers)
]


@pytest.mark.parametrize("name,W,H,spp,rr,off,stride,rrmode", CASES)
def test_gpu_counting_pass_equals_oracle_counters(name, W, H, spp, rr, off, stride, rrmode):
    g, n, kernel = gpu_counts(name, W, H, spp, rr, off, stride, rrmode)
    rows = list(range(off, H, stride))
    o, n_ref = oracle_counts(name, W, H, spp, rr, rows, rrmode)
    assert n == n_ref == len(rows) * W * spp
    assert o["eye_retraces"] > 0
    steer = {k: (g[k], o[k]) for k in ("rng_draws", "light_verts", "light_vert_reads")}
    steer["closest_rays"] = (g["closest_rays"], o["closest_rays"] - o["eye_retraces"])
    queries = {k: (g[k], o[k]) for k in ("shadow_rays", "splats")}
    bad = {k: v for k, v in {**steer, **queries}.items() if v[0] != v[1]}
    assert not bad, f"{kernel}: counters differ from the oracle's (gpu, oracle): {bad}"
