"""INTEGRATION.md's reference-side binding, run on the GPU through the reference's own types.

oracle/_ref/adapter/adapter_check is the reference's Renderer / Scene /
BDPTIntegrator code (integrator.cpp, renderer.cpp, main.cpp) with the adapter
header and the registration edits of INTEGRATION.md §2-§3 extracted verbatim
(oracle/ref/make_adapter.py, built in the development container by
`make -C oracle/ref adapter`), linked against the product library:
* `frame`: a `type = "bdpt_gpu"` scene file through loadTOML -> Renderer::init
  (factory edit) -> Renderer::render (offline-branch edit: renderFrame) against
  the reference goldens (per-pixel relative L2 <= 1e-4), and Renderer::cleanUp's
  EXR;
* `samples`: GpuBDPTIntegrator::render(ray, sampler) against the reference's
  BDPTIntegrator::render(ray, sampler) on the same Scene and Sampler state, for
  thousands of camera samples: Li bit for bit, the std::mt19937 state after the
  call equal, the camera splats bit for bit;
* the reference's own command line (main.cpp's main) rendering a bdpt_gpu scene.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import variants
from conftest import load_golden

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AD = os.path.join(REPO, "oracle", "_ref", "adapter")
CHECK = os.path.join(AD, "adapter_check")
CLI = os.path.join(AD, "tinyrender")
TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _built():
    if not os.path.exists(CHECK):
        pytest.skip("oracle/_ref/adapter not built (make -C oracle/ref adapter in the development container)")


def _toml(tmp_path, name, W, H, spp, rr=None, kind="bdpt_gpu"):
    p = tmp_path / f"{name}_{W}x{H}_{spp}.toml"
    p.write_text(variants.toml_text(name, W, H, spp, rr, kind=kind))
    return p


def _rel_l2(fb, ref):
    a, r = fb.reshape(-1, 3).astype(np.float64), ref.reshape(-1, 3).astype(np.float64)
    return np.linalg.norm(a - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)


@pytest.mark.parametrize("golden", ["G1_cbox_low_64x64_spp4", "G2_caustic_64x64_spp16", "G3_hardlight_64x64_spp16",
                                    "G4_hardlight_mirror_64x64_spp16", "G5_caustic_80x48_spp1"])
def test_adapter_frame_through_renderer_matches_golden(tmp_path, golden_manifest, golden):
    m = golden_manifest["framebuffers"][golden]
    W, H, spp, rr = m["width"], m["height"], m["spp"], m["rr_depth"]
    toml = _toml(tmp_path, m["scene"], W, H, spp, rr)
    out = tmp_path / "fb.f32"
    r = subprocess.run([CHECK, "frame", str(toml), str(W), str(H), str(spp), str(out)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '"integrator": "GpuBDPTIntegrator"' in r.stdout
    fb = np.fromfile(out, np.float32).reshape(H, W, 3)
    ref = load_golden(golden)
    err = _rel_l2(fb, ref)
    assert np.isfinite(fb).all() and err.max() <= TOL, f"max per-pixel rel L2 {err.max():.3g}"
    exr = toml.with_suffix(".exr")  # Renderer::cleanUp -> Integrator::save (integrator.cpp:26-30)
    assert exr.exists() and exr.stat().st_size > W * H * 6


@pytest.mark.parametrize("name, W, H, spp, rr, n, stride", [
    ("caustic", 64, 64, 16, 8, 1500, 37),
    ("hardlight", 64, 64, 16, 2, 1500, 41),
    ("cbox_low", 64, 64, 4, 5, 1000, 53),
    ("hardlight_mirror", 64, 64, 16, 5, 1000, 29),
    ("caustic", 80, 48, 1, 12, 500, 7),  # spp 1: pixel centre, no jitter draws; deeper paths
])
def test_adapter_render_ray_sampler_equals_reference_integrator(tmp_path, name, W, H, spp, rr, n, stride):
    toml = _toml(tmp_path, name, W, H, spp, rr)
    r = subprocess.run([CHECK, "samples", str(toml), str(W), str(H), str(spp), str(n), str(stride)],
                       capture_output=True, text=True, timeout=600)
    out = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
    assert r.returncode == 0, r.stdout + r.stderr
    assert out["samples"] == n
    assert out["li_mismatch"] == 0 and out["state_mismatch"] == 0 and out["splat_mismatch"] == 0, out
    assert out["nonzero_li"] > n // 4  # the check is not vacuous
    if name != "hardlight_mirror":
        assert out["splat_pixels"] > 0


def test_reference_cli_renders_bdpt_gpu_scene(tmp_path):
    """main.cpp's own main (run(): loadTOML, Renderer::init / render / cleanUp)
    with the registration edits: a bdpt_gpu scene renders on the GPU and the EXR
    lands next to the scene file."""
    toml = _toml(tmp_path, "caustic", 64, 64, 16, 8)
    r = subprocess.run([CLI, str(toml), "nogui"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Render took:" in r.stdout
    assert toml.with_suffix(".exr").exists()


# The same binding over the reference built with NO_RR = 0 (oracle/_ref/adapter/rr): the
# adapter reads the macro (bdpt.h:18) and asks the library for Russian roulette.
CHECK_RR = os.path.join(AD, "rr", "adapter_check")


@pytest.mark.parametrize("golden", ["R1_caustic_rr_64x64_spp16", "R2_hardlight_rr_64x64_spp16",
                                    "R3_cbox_low_rr_64x64_spp4"])
def test_adapter_rr_frame_matches_reference_golden(tmp_path, golden_manifest, golden):
    m = golden_manifest["rr_framebuffers"][golden]
    W, H, spp, rr = m["width"], m["height"], m["spp"], m["rr_depth"]
    toml = _toml(tmp_path, m["scene"], W, H, spp, rr)
    out = tmp_path / "fb.f32"
    r = subprocess.run([CHECK_RR, "frame", str(toml), str(W), str(H), str(spp), str(out)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fb = np.fromfile(out, np.float32).reshape(H, W, 3)
    err = _rel_l2(fb, load_golden(golden))
    assert err.max() <= TOL, f"max per-pixel rel L2 {err.max():.3g}"


@pytest.mark.parametrize("name, W, H, spp, rr, n, stride", [
    ("caustic", 64, 64, 16, 3, 1500, 37),
    ("hardlight", 64, 64, 16, 2, 1000, 41),
    ("cbox_low", 64, 64, 4, 1, 800, 53),
])
def test_adapter_rr_render_ray_sampler_equals_reference_integrator(tmp_path, name, W, H, spp, rr, n, stride):
    """Russian roulette through the reference's own Sampler: every draw past
    rrDepth, every stored rrProbability; Li, generator state and splats bit for bit."""
    toml = _toml(tmp_path, name, W, H, spp, rr)
    r = subprocess.run([CHECK_RR, "samples", str(toml), str(W), str(H), str(spp), str(n), str(stride)],
                       capture_output=True, text=True, timeout=600)
    out = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
    assert r.returncode == 0, r.stdout + r.stderr
    assert out["li_mismatch"] == 0 and out["state_mismatch"] == 0 and out["splat_mismatch"] == 0, out
    assert out["nonzero_li"] > n // 4
