"""The Russian-roulette continuation pass (bdpt_kernels.hip: park_lane, the chain
kernel, resume launches; bdpt_capi.cpp: BDPT_PARK_DEPTH / BDPT_PARK_ROUNDS) against
the reference compiled with NO_RR = 0 (bdpt.h:18, :68, :129-132, :188, :201-204).

A light or eye walk deeper than the park depth leaves the megakernel; the chain
kernel walks its delta bounces with the whole wave (coop_closest) and a resume
launch of the megakernel continues the sample in its own lane slot. Forcing a
park depth of 1-3 hands nearly every roulette walk over, several times per
sample, so the goldens exercise saving and restoring the sample, the wave walk,
the MT19937 ring of another slot, and the resume rounds — the frames must stay
the reference's (per-pixel relative L2 <= 1e-4, float reassociation only).
"""
import numpy as np
import pytest

import bdpt_amd
import oracle as O
import variants
from conftest import load_golden
from test_gpu_parity import RR_CASES, TOL, report, rr_integrator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth,rounds", [("1", "3"), ("3", "1")])
@pytest.mark.parametrize("name", RR_CASES[:5])
def test_gpu_park_every_walk_matches_reference_golden(name, depth, rounds, golden_manifest, monkeypatch):
    monkeypatch.setenv("BDPT_PARK_DEPTH", depth)
    monkeypatch.setenv("BDPT_PARK_ROUNDS", rounds)
    m = golden_manifest["rr_framebuffers"][name]
    it = rr_integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    st = it.stats()
    assert st["capped_samples"] == 0 and st["schedule_errors"] == 0
    assert st["launches"] == 1 + 2 * int(rounds)
    assert st["parked_samples"] > 0, "no walk reached the park depth"
    worst, exact, _ = report(fb, load_golden(name))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"


@pytest.mark.parametrize("rr,W,H,spp", [(6, 16, 12, 4), (40, 12, 8, 2)])
def test_gpu_park_closed_box_matches_oracle(rr, W, H, spp, tmp_path, monkeypatch):
    """Closed box: every subpath ends by roulette only, far past the lazy MT19937
    window, so the chain kernel draws from (and generates ahead into) the ring of
    the slot it continues."""
    monkeypatch.setenv("BDPT_PARK_DEPTH", "2")
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    it = rr_integrator(None, W, H, spp, rr, obj=obj, cam=cam)
    fb = it.render_frame().reshape(-1)
    st = it.stats()
    assert st["capped_samples"] == 0 and st["parked_samples"] > 0
    ref, _ = O.Scene(obj).render(O.make_params(cam, W, H, spp, rr, 0, russian_roulette=1))
    worst, exact, _ = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"rr={rr}: max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


def test_gpu_park_off_and_on_give_the_same_frame(monkeypatch):
    """The pass moves work between kernels, not arithmetic: the default depth and
    no parking at all give the same frame (up to the framebuffer adds' order)."""
    frames = []
    for depth in ("0", "2"):
        monkeypatch.setenv("BDPT_PARK_DEPTH", depth)
        it = rr_integrator("caustic", 48, 40, 8, 3)
        frames.append(it.render_frame().copy())
        st = it.stats()
        assert (st["parked_samples"] > 0) == (depth != "0")
        assert st["launches"] == (1 if depth == "0" else 9)
    a, b = (f.reshape(-1, 3).astype(np.float64) for f in frames)
    err = np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-8)
    assert err.max() <= TOL


def test_gpu_park_not_in_counting_pass(monkeypatch):
    """The counting pass keeps every walk in the megakernel (its counters are the
    megakernel's): no chain or resume launches."""
    monkeypatch.setenv("BDPT_PARK_DEPTH", "1")
    it = rr_integrator("caustic", 32, 32, 4, 3)
    it.render_frame(flags=bdpt_amd.FLAG_COUNT)
    st = it.stats()
    assert st["launches"] == 1 and st["parked_samples"] == 0
