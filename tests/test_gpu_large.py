"""BASELINE.json configs[1], [3] and [4] at their full size on one GPU.

* configs[1]: CausticSample 512x512, 256 spp (the bench workload; 67.1 M camera samples),
  as shipped (NO_RR = 1) and with Russian roulette (NO_RR = 0, bench.py --russian-roulette)
* configs[2]: HardLightSample 512x512, 1024 spp (rrDepth 2: the short-subpath build)
* configs[3]: CausticSample 1024x1024, 1024 spp (1.07 G camera samples)
* configs[4]: synthetic 1M-triangle scene, 2048x2048, 512 spp (2.15 G samples)

Parity at full size, two ways:
1. a two-row shard of the full-size frame against the reference's own render of
   that shard (tests/golden/L1_*, L2_*: oracle/_ref/ref_bdpt, make_goldens.py):
   the shard's rows per pixel (eye estimates + the splats landing on them),
   and block sums of the whole frame (every camera splat of the shard);
2. the full frame rendered in one launch equals the sum of its two interleaved
   row shards (each rendered separately) — the additivity the multi-GPU split
   relies on — and is finite and non-negative.
Tolerance: per-pixel relative L2 <= 1e-4 (north star); block sums <= 1e-5.
"""
import os

import numpy as np
import pytest

import bdpt_amd
import variants

pytestmark = pytest.mark.gpu

TOL = 1e-4
LARGE = ["L0_caustic_512x512_spp256_rows8", "L1_caustic_1024x1024_spp1024_rows2", "L2_synth1m_2048x2048_spp512_rows2",
         "L3_hardlight_512x512_spp1024_rows8", "L4_caustic_rr_512x512_spp256_rows8"]
_scenes = {}


def integrator(name, W, H, spp, rr, russian_roulette=0):
    if name not in _scenes:
        _scenes[name] = bdpt_amd.Scene(variants.obj_path(name))
    cam = bdpt_amd.Camera(**variants.SCENES[name]["camera"])
    it = bdpt_amd.BDPTIntegrator(_scenes[name], bdpt_amd.Config(camera=cam, width=W, height=H, spp=spp, rr_depth=rr,
                                                                russian_roulette=russian_roulette))
    it.init()
    return it


def rel_l2(a, r, floor=1e-8):
    a = a.reshape(-1, 3).astype(np.float64)
    r = r.reshape(-1, 3).astype(np.float64)
    return np.linalg.norm(a - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), floor)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", LARGE)
def test_gpu_full_size_shard_matches_reference(name, golden_manifest):
    m = golden_manifest["large_framebuffers"][name]
    W, H, blk = m["width"], m["height"], m["block"]
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))
    it = integrator(m["scene"], W, H, m["spp"], m["rr_depth"], m.get("russian_roulette", 0))
    fb = it.render_frame(row_offset=m["row_offset"], row_stride=m["row_stride"]).reshape(H, W, 3)
    assert it.stats()["samples"] == m["samples"]
    assert np.all(np.isfinite(fb)) and fb.min() >= 0.0
    rows = g["rows"]
    e = rel_l2(fb[rows], g["fb_rows"])
    assert e.max() <= TOL, f"shard rows: max per-pixel rel L2 {e.max():.3g}"
    blocks = fb.astype(np.float64).reshape(H // blk, blk, W // blk, blk, 3).sum(axis=(1, 3))
    eb = rel_l2(blocks, g["blocks"], floor=1e-6)
    assert eb.max() <= 1e-5, f"block sums: max rel L2 {eb.max():.3g}"


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", [n for n in LARGE if "_rr_" not in n])  # (a Russian-roulette frame is one
# trapped subpath's serial chain of millions of bounces, DESIGN.md §8: three of them do not fit the suite)
def test_gpu_full_size_frame_is_sum_of_row_shards(name, golden_manifest):
    m = golden_manifest["large_framebuffers"][name]
    W, H, spp, rr = m["width"], m["height"], m["spp"], m["rr_depth"]
    it = integrator(m["scene"], W, H, spp, rr, m.get("russian_roulette", 0))
    full = it.render_frame().copy()
    assert it.stats()["samples"] == W * H * spp
    assert np.all(np.isfinite(full)) and full.min() >= 0.0
    ms_full = it.stats()["kernel_ms"]
    acc = np.zeros_like(full)
    for r in range(2):
        sh = integrator(m["scene"], W, H, spp, rr, m.get("russian_roulette", 0))
        acc += sh.render_frame(row_offset=r, row_stride=2)
    e = rel_l2(acc, full)
    assert e.max() <= TOL, f"max per-pixel rel L2 {e.max():.3g}"
    print(f"{name}: full frame {W}x{H}x{spp} kernel {ms_full:.1f} ms = "
          f"{W * H * spp / ms_full * 1e-3:.1f} Msamples/s")
