"""Frames rendered again and again on one context: every lane slot's MT19937 ring
(DevScene::mt_ring) then holds the outputs and the generate-ahead cursor of
whatever sample used the slot last (mt_ring_ahead). Round 4 found a cursor left
from a slot's previous seed next to the new seed's tag after outputs 0..226
were materialized alone; the frame drifted from the reference by one sample's
estimate in a few pixels from the second frame on (HardLight 512^2 x 1024 with
Russian roulette, 1.3e-3). Each frame here must be the reference's.
"""
import numpy as np
import pytest

import bdpt_amd
import oracle as O
import variants
from test_gpu_parity import TOL, report, rr_integrator

pytestmark = pytest.mark.gpu


def _repeat(it, ref, frames=4, **kw):
    for f in range(frames):
        if it.rgb is not None:
            it.rgb[:] = 0  # render_frame adds into the integrator's rgb, as the reference's frames do
        fb = it.render_frame(**kw).reshape(-1)
        st = it.stats()
        assert st["schedule_errors"] == 0 and st["capped_samples"] == 0
        worst, exact, _ = report(fb, ref)
        assert worst <= TOL, f"frame {f}: max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


@pytest.mark.parametrize("rr", [6, 40])
def test_gpu_rr_closed_box_frames_on_one_context(rr, tmp_path):
    """Closed box, Russian roulette: every subpath ends by roulette only, so most
    samples (all at rrDepth 40) draw past the lazy window. A full frame fills every lane slot; the
    row shards after it put other samples into those slots (the same frame again
    would mostly give each slot its old sample, whose outputs the ring holds)."""
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    W, H, spp = 96, 96, 8
    it = rr_integrator(None, W, H, spp, rr, obj=obj, cam=cam)
    sc = O.Scene(obj)
    p = O.make_params(cam, W, H, spp, rr, 0, russian_roulette=1)
    for off, stride in [(0, 1), (1, 3), (0, 2), (2, 5), (0, 1)]:
        ref, _ = sc.render(p, threads=8, rows=list(range(off, H, stride)))
        _repeat(it, ref.reshape(-1), frames=1, row_offset=off, row_stride=stride)


def test_gpu_deep_rr_depth_frames_on_one_context(tmp_path):
    """rrDepth 40 without roulette (the deep build: every sample draws ~400
    numbers in the closed box): the same ring, shard after shard."""
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    W, H, spp, rr = 128, 96, 8, 40
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(obj), cfg)
    it.init()
    sc = O.Scene(obj)
    p = O.make_params(cam, W, H, spp, rr, 0)
    for off, stride in [(0, 1), (1, 3), (0, 2), (2, 5)]:
        ref, _ = sc.render(p, threads=8, rows=list(range(off, H, stride)))
        _repeat(it, ref.reshape(-1), frames=1, row_offset=off, row_stride=stride)


def test_gpu_rr_hardlight_shards_on_one_context():
    """HardLight with Russian roulette (where the drift was seen): a full frame,
    then row shards of it on the same context, each against the oracle."""
    W, H, spp, rr = 128, 128, 64, 2
    it = rr_integrator("hardlight", W, H, spp, rr)
    sc = O.Scene(variants.obj_path("hardlight"))
    p = O.make_params(variants.SCENES["hardlight"]["camera"], W, H, spp, rr, 0, russian_roulette=1)
    full, _ = sc.render(p, threads=8)
    _repeat(it, full.reshape(-1), frames=2)
    shard, _ = sc.render(p, threads=8, rows=list(range(0, H, 5)))
    _repeat(it, shard.reshape(-1), frames=3, row_offset=0, row_stride=5)
