"""Debugging knobs that change what a frame computes are read only with
BDPT_DEBUG_KNOBS=1 (bdpt_capi.cpp debug_knob): BDPT_SAMPLE_RANGE set
alone leaves the frame whole, and with the switch the frame holds exactly the
range's samples and bdpt_stats.samples counts them (hi - lo)."""
import numpy as np
import pytest

from test_gpu_parity import integrator

pytestmark = pytest.mark.gpu


def test_gpu_sample_range_needs_debug_switch(monkeypatch):
    W, H, spp = 32, 16, 4
    it = integrator("caustic", W, H, spp, 8)
    full = it.render_frame().reshape(-1).copy()
    n_full = it.stats()["samples"]
    assert n_full == W * H * spp

    monkeypatch.setenv("BDPT_SAMPLE_RANGE", "128,640")
    monkeypatch.delenv("BDPT_DEBUG_KNOBS", raising=False)
    it2 = integrator("caustic", W, H, spp, 8)
    ignored = it2.render_frame().reshape(-1).copy()
    assert it2.stats()["samples"] == n_full
    rel = np.linalg.norm(ignored - full) / np.linalg.norm(full)
    assert rel < 1e-5, rel  # the whole frame (float reassociation only)

    monkeypatch.setenv("BDPT_DEBUG_KNOBS", "1")
    it3 = integrator("caustic", W, H, spp, 8)
    part = it3.render_frame().reshape(-1)
    assert it3.stats()["samples"] == 640 - 128
    assert np.linalg.norm(part) < np.linalg.norm(full)
