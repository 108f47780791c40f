"""The lane-decoupled frame-kernel build (bdpt_kernels_dq.hip, BDPT_DQ=1) against
the reference: connection tasks (connectToCamera, connectToLight,
connectVertices) run by other lanes than the camera sample's owner, the owner's
walks continuing meanwhile. Same per-sample arithmetic and random-number order
as the default build, so the bar is the same: per-pixel relative L2 <= 1e-4
against the reference's frames (tests/golden, oracle/_ref/ref_bdpt), and the C
oracle at other sizes and seeds. The library reads BDPT_DQ per render.
"""
import os

import numpy as np
import pytest

import bdpt_amd
import oracle as O
import variants
from conftest import load_golden
from test_gpu_parity import FB_CASES, STRATEGY, TOL, integrator, rel_l2, report

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(autouse=True)
def dq_build(monkeypatch):
    monkeypatch.setenv("BDPT_DQ", "1")
    monkeypatch.setenv("BDPT_SPLIT_MAX_RR", "0")


@pytest.mark.parametrize("name", FB_CASES + ["G9_caustic_lt_64x64_spp16", "G10_caustic_pt_64x64_spp16",
                                             "G11_hardlight_lt_64x64_spp16", "G12_hardlight_pt_64x64_spp16"])
def test_gpu_dq_matches_reference_golden(name, golden_manifest):
    m = golden_manifest["framebuffers"][name]
    it = integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"], STRATEGY[m.get("strategy", "bdpt")])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    st = it.stats()
    assert st["kernel"] == "bdpt_frame_kernel_dq"
    assert st["samples"] == m["samples"]
    worst, exact, whole = report(fb, load_golden(name))
    assert np.all(np.isfinite(fb))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


def test_gpu_dq_bench_frame_rows_match_reference(golden_manifest):
    """The bench workload (Caustic 512x512, 256 spp) on the reference's 8-row shard
    (golden L0): the rows per pixel and the block sums of every splat."""
    name = "L0_caustic_512x512_spp256_rows8"
    m = golden_manifest["large_framebuffers"][name]
    W, H, blk = m["width"], m["height"], m["block"]
    g = np.load(os.path.join(GOLD, name + ".npz"))
    it = integrator(m["scene"], W, H, m["spp"], m["rr_depth"])
    fb = it.render_frame(row_offset=m["row_offset"], row_stride=m["row_stride"]).reshape(H, W, 3)
    assert it.stats()["kernel"] == "bdpt_frame_kernel_dq"
    e = rel_l2(fb[g["rows"]], g["fb_rows"])
    assert e.max() <= TOL, f"shard rows: max per-pixel rel L2 {e.max():.3g}"
    blocks = fb.astype(np.float64).reshape(H // blk, blk, W // blk, blk, 3).sum(axis=(1, 3))
    eb = rel_l2(blocks, g["blocks"])
    assert eb.max() <= 1e-5, f"block sums: max rel L2 {eb.max():.3g}"


@pytest.mark.parametrize("name,W,H,spp,rr", [("caustic", 40, 24, 3, 3), ("hardlight", 33, 17, 5, 6),
                                             ("cbox_low", 24, 24, 2, 12), ("hardlight_mirror", 32, 32, 4, 28),
                                             ("caustic", 16, 16, 64, 1), ("caustic", 48, 40, 2, 2)])
def test_gpu_dq_matches_oracle_other_configs(name, W, H, spp, rr):
    """Odd sizes, rrDepth 1..28 (the decoupled build's range), spp 2..64: the
    oracle renders the same seeds; rrDepth 28 pushes up to 28 tasks per eye vertex."""
    it = integrator(name, W, H, spp, rr)
    fb = it.render_frame().reshape(-1)
    assert it.stats()["kernel"] == "bdpt_frame_kernel_dq"
    cam = variants.SCENES[name]["camera"]
    ref, _ = O.Scene(variants.obj_path(name)).render(O.make_params(cam, W, H, spp, rr))
    e = rel_l2(fb, ref)
    assert e.max() <= TOL, f"max per-pixel rel L2 {e.max():.3g}"


def test_gpu_dq_row_shards_sum_to_full_frame():
    it = integrator("caustic", 64, 48, 8, 8)
    full = it.render_frame().copy()
    acc = np.zeros_like(full)
    for r in range(3):
        acc += integrator("caustic", 64, 48, 8, 8).render_frame(row_offset=r, row_stride=3)
    assert rel_l2(acc, full).max() <= TOL


def test_gpu_dq_counting_pass_matches_default_counts(monkeypatch):
    """The counting pass of both builds on the same seeds: the same closest hits,
    light vertices and connection reads per frame (the schedule differs, the
    work of every sample does not)."""
    it = integrator("caustic", 64, 64, 4, 8)
    it.render_frame(flags=bdpt_amd.FLAG_COUNT)
    dq = it.stats()["counters"]
    monkeypatch.setenv("BDPT_DQ", "0")
    it.render_frame(flags=bdpt_amd.FLAG_COUNT)
    assert it.stats()["kernel"] == "bdpt_frame_kernel"
    ref = it.stats()["counters"]
    for k in ("closest_rays", "shadow_rays", "light_verts", "light_vert_reads", "splats", "rng_draws"):
        assert dq[k] == ref[k], (k, dq[k], ref[k])
