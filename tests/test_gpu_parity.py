"""GPU parity: the HIP path (through the C-ABI) against the reference.

Tolerance (BASELINE.json north_star): per-pixel relative L2
||gpu - ref||_2 / max(||ref||_2, 1e-8) <= 1e-4 on every pixel. The GPU replays
the reference's exact per-sample arithmetic and RNG stream, so the only
differences left are the order in which float contributions are summed into
a pixel (device atomics vs. the reference's serial order); all contributions
are non-negative, so that reassociation error is a few ulps.
"""
import numpy as np
import pytest

import bdpt_amd
import oracle as O
import variants
from conftest import load_golden

pytestmark = pytest.mark.gpu

TOL = 1e-4

FB_CASES = ["G1_cbox_low_64x64_spp4", "G2_caustic_64x64_spp16", "G3_hardlight_64x64_spp16",
            "G4_hardlight_mirror_64x64_spp16", "G5_caustic_80x48_spp1", "G6_caustic_512x512_spp4_rows16",
            "G7_hardlight_512x512_spp4_rows32", "G8_synth1m_48x32_spp2",
            # the reference built with LIGHT_TRACING / PATH_TRACING = 1 (bdpt.h:16-17)
            "G9_caustic_lt_64x64_spp16", "G10_caustic_pt_64x64_spp16", "G11_hardlight_lt_64x64_spp16",
            "G12_hardlight_pt_64x64_spp16"]
STRATEGY = {"bdpt": bdpt_amd.STRATEGY_BDPT, "lt": bdpt_amd.STRATEGY_LIGHT_TRACING,
            "pt": bdpt_amd.STRATEGY_PATH_TRACING}

_scenes = {}


def scene(name):
    if name not in _scenes:
        _scenes[name] = bdpt_amd.Scene(variants.obj_path(name))
    return _scenes[name]


def integrator(name, W, H, spp, rr, strategy=0):
    cam = bdpt_amd.Camera(**variants.SCENES[name]["camera"])
    cfg = bdpt_amd.Config(camera=cam, width=W, height=H, spp=spp, rr_depth=rr, strategy=strategy)
    it = bdpt_amd.BDPTIntegrator(scene(name), cfg)
    it.init()
    return it


def rel_l2(fb, ref):
    a = fb.reshape(-1, 3).astype(np.float64)
    r = ref.reshape(-1, 3).astype(np.float64)
    return np.linalg.norm(a - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)


def report(fb, ref):
    e = rel_l2(fb, ref)
    exact = np.mean((fb.reshape(-1).view(np.uint32) == ref.reshape(-1).view(np.uint32)))
    whole = np.linalg.norm(fb.astype(np.float64) - ref) / max(np.linalg.norm(ref.astype(np.float64)), 1e-30)
    return e.max(), exact, whole


@pytest.mark.parametrize("name", FB_CASES)
def test_gpu_matches_reference_golden(name, golden_manifest):
    m = golden_manifest["framebuffers"][name]
    it = integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"], STRATEGY[m.get("strategy", "bdpt")])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    assert it.stats()["samples"] == m["samples"]
    ref = load_golden(name)
    worst, exact, whole = report(fb, ref)
    assert np.all(np.isfinite(fb))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


@pytest.mark.parametrize("name,W,H,spp,rr", [("caustic", 64, 64, 16, 8), ("hardlight", 64, 64, 16, 2),
                                             ("hardlight_mirror", 48, 48, 8, 5), ("synth1m", 32, 24, 2, 8)])
def test_gpu_full_traversal_equals_culled_traversal(name, W, H, spp, rr):
    """The reference's own binary tree walked without culling (FULL) and the
    4-wide hierarchy with distance culling give the same closest hits."""
    a = integrator(name, W, H, spp, rr)
    fa = a.render_frame().copy()
    b = integrator(name, W, H, spp, rr)
    fb = b.render_frame(flags=bdpt_amd.FLAG_FULL_TRAVERSAL).copy()
    assert rel_l2(fa, fb).max() <= TOL


# beyond 100 diagonals (the slack decision) and within the camera ray's max_t of 1000 (renderer.cpp:192)
@pytest.mark.parametrize("name,dist", [("caustic", 150.0), ("hardlight", 250.0), ("caustic", 280.0)])
def test_gpu_far_camera_takes_the_slack_test_and_matches_oracle(name, dist):
    """A camera more than 100 scene diagonals away: the host keeps the interior
    boxes' ambiguity slack (node_slack_needed) and the frame
    still equals the oracle's (a narrow field of view keeps the box in view)."""
    cam = dict(variants.SCENES[name]["camera"])
    eye, at = np.array(cam["eye"], np.float64), np.array(cam["at"], np.float64)
    fwd = (at - eye) / np.linalg.norm(at - eye)
    diag = 2.0 * np.sqrt(3.0)  # ~ the Cornell boxes' diagonal
    cam["eye"] = list(at - fwd * dist * diag)
    cam["fov"] = float(np.degrees(2 * np.arctan(1.2 / (dist * diag))))
    W, H, spp, rr = 32, 32, 4, variants.SCENES[name]["rr_depth"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    it = bdpt_amd.BDPTIntegrator(scene(name), cfg)
    it.init()
    fb = it.render_frame().reshape(-1)
    ref, _ = O.Scene(variants.obj_path(name)).render(O.make_params(cam, W, H, spp, rr))
    assert (ref.reshape(-1, 3).sum(1) > 0).mean() > 0.2  # the box is in view
    worst, exact, _ = report(fb, ref)
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


# coordinates ~250 diagonals from 0: the slack-free interior test (by one fma per
# plane in the BDPT_SLAB_FMA builds); ~350: past kFmaCoordDiags, the slack test (bdpt_capi.cpp)
# (HardLight's 0.08-unit light keeps its area only up to ~100 diagonals: float
# coordinates near 800 flatten its faces, and the loader then finds no emitter)
@pytest.mark.parametrize("name,diags", [("caustic", 250.0), ("caustic", 350.0), ("hardlight", 100.0)])
def test_gpu_translated_scene_matches_oracle(name, diags, tmp_path):
    """The scene and camera moved far from the origin along (1, 1, 1): both sides
    of the host's coordinate-magnitude condition on the slack-free interior test
    render the oracle's frame."""
    with open(variants.obj_path(name)) as f:
        v = np.array([line.split()[1:4] for line in f if line.startswith("v ")], np.float64)
    off = np.full(3, diags * np.linalg.norm(v.max(0) - v.min(0)))  # |coordinate| ~ diags diagonals per axis
    path = variants.translated_obj(name, str(tmp_path), off)
    cam = dict(variants.SCENES[name]["camera"])
    cam["eye"] = [float(np.float32(e + o)) for e, o in zip(cam["eye"], off)]
    cam["at"] = [float(np.float32(a + o)) for a, o in zip(cam["at"], off)]
    W, H, spp, rr = 32, 32, 4, variants.SCENES[name]["rr_depth"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(path), cfg)
    it.init()
    fb = it.render_frame().reshape(-1)
    ref, _ = O.Scene(path).render(O.make_params(cam, W, H, spp, rr))
    assert (ref.reshape(-1, 3).sum(1) > 0).mean() > 0.2  # the box is in view
    worst, exact, _ = report(fb, ref)
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


@pytest.mark.parametrize("kind,diags", [("path", 250.0), ("path", 350.0), ("direct", 250.0), ("direct", 350.0)])
def test_gpu_translated_scene_path_and_direct_match_oracle(kind, diags, tmp_path):
    """The path tracer and the direct integrator take the same per-render choice
    of interior-box test (bdpt_capi.cpp pt_scene): the Caustic scene moved ~250
    and ~350 diagonals from 0 along (1, 1, 1), both sides of the condition."""
    with open(variants.obj_path("caustic")) as f:
        v = np.array([line.split()[1:4] for line in f if line.startswith("v ")], np.float64)
    off = np.full(3, diags * np.linalg.norm(v.max(0) - v.min(0)))
    path = variants.translated_obj("caustic", str(tmp_path), off)
    cam = dict(variants.SCENES["caustic"]["camera"])
    cam["eye"] = [float(np.float32(e + o)) for e, o in zip(cam["eye"], off)]
    cam["at"] = [float(np.float32(a + o)) for a, o in zip(cam["at"], off)]
    W, H, spp = 32, 24, 4
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp)
    sc = bdpt_amd.Scene(path)
    if kind == "path":
        fb = bdpt_amd.PathTracerIntegrator(sc, cfg, bdpt_amd.PathSettings()).render_frame().reshape(-1)
        params = O.make_path_params(cam, W, H, spp)
    else:
        ds = bdpt_amd.DirectSettings(sampling_strategy="mis", emitter_samples=2, bsdf_samples=2)
        fb = bdpt_amd.DirectIntegrator(sc, cfg, ds).render_frame().reshape(-1)
        params = O.make_direct_params(cam, W, H, spp, strategy="mis", emitter_samples=2, bsdf_samples=2)
    ref, _ = O.Scene(path).render(params)
    assert (ref.reshape(-1, 3).sum(1) > 0).mean() > 0.2  # the box is in view
    worst, exact, _ = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


@pytest.mark.parametrize("name,W,H,spp,rr", [
    ("caustic", 24, 40, 3, 1),    # rrDepth 1: both walks stop at once (2 draws)
    ("caustic", 24, 40, 3, 2),
    ("caustic", 40, 24, 5, 12),   # deeper than any shipped scene
    ("hardlight", 33, 17, 7, 3),
    ("hardlight_mirror", 32, 32, 2, 9),
    ("cbox_low", 17, 29, 1, 6),
    ("cbox_low", 16, 12, 4, 28),  # the deepest rrDepth the lazy MT19937 window covers (226 draws)
    ("synth1m", 12, 8, 2, 8),     # 1M triangles, 4-wide stack spills past the LDS entries
])
def test_gpu_matches_oracle_other_configs(name, W, H, spp, rr):
    it = integrator(name, W, H, spp, rr)
    fb = it.render_frame().reshape(-1)
    sc = O.Scene(variants.obj_path(name))
    ref, n = sc.render(O.make_params(variants.SCENES[name]["camera"], W, H, spp, rr))
    assert n == W * H * spp
    worst, exact, _ = report(fb, ref)
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


@pytest.mark.parametrize("rr,W,H,spp", [(29, 16, 12, 2), (40, 16, 12, 2), (150, 12, 8, 2), (300, 8, 6, 2)])
def test_gpu_deep_rr_depth_continues_mt19937_from_ring(rr, W, H, spp, tmp_path):
    """rrDepth > 28 in a closed box (every path runs to rrDepth): samples draw
    past the lazy window (227) and, from rrDepth ~80, past a full MT19937 state
    (624): the megakernel continues from the lanes' HBM rings, same image as
    the oracle's real std::mt19937 restatement."""
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    fb = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(obj), cfg).render_frame().reshape(-1)
    O.counters(True)
    ref, n = O.Scene(obj).render(O.make_params(cam, W, H, spp, rr))
    draws = O.counters(True)["rng_draws"] / n
    assert draws > {29: 150, 40: 200, 150: 550, 300: 900}[rr]  # mean draws per sample: many past 227 / 624
    worst, exact, _ = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"rr={rr}: max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


def test_gpu_rr_depth_limits():
    """rrDepth past 1024 is refused, and so is an unknown flag (bit 2 was the
    round-1 wavefront schedule)."""
    it = integrator("cbox_low", 8, 8, 1, 8)
    with pytest.raises(bdpt_amd.BdptError, match="flag"):
        it.render_frame(flags=4)
    it = integrator("cbox_low", 8, 8, 1, 1025)
    with pytest.raises(bdpt_amd.BdptError, match="rr_depth"):
        it.render_frame()


def test_gpu_many_materials_take_the_hbm_table_build(tmp_path):
    """408 materials: the BSDF records (72 B each) outgrow the 24 KiB LDS table,
    so bdpt_render runs the HBM-table build of the megakernel and the single-
    sample kernel reads them from HBM per launch — same frame and sample as the
    oracle. The path / direct frame kernels (LDS table only) and rrDepth > 28
    (no deep HBM build) refuse such a scene instead of rendering it wrong."""
    obj = variants.many_materials_obj(str(tmp_path))
    cam = variants.SCENES["cbox_low"]["camera"]
    W, H, spp, rr = 32, 24, 4, 5
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    sc = bdpt_amd.Scene(obj)
    assert sc.info()["materials"] == 408
    fb = bdpt_amd.BDPTIntegrator(sc, cfg).render_frame().reshape(-1)
    osc = O.Scene(obj)
    p = O.make_params(cam, W, H, spp, rr)
    ref, _ = osc.render(p)
    worst, exact, _ = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"
    it = bdpt_amd.BDPTIntegrator(sc, cfg)
    it.init()
    for pixel, k in [(300, 1), (500, 3)]:
        it.rgb[:] = 0
        Li_ref, splats_ref = osc.sample(p, pixel, k)
        ray, sampler = driver_ray(p, "cbox_low", pixel, k)
        assert np.allclose(it.render(ray, sampler), Li_ref, rtol=1e-6, atol=0)
        assert rel_l2(it.rgb.reshape(-1), splats_ref).max() <= TOL
    with pytest.raises(bdpt_amd.BdptError, match="LDS table"):
        bdpt_amd.PathTracerIntegrator(sc, cfg).render_frame()
    deep = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=8, height=8, spp=1, rr_depth=29)
    with pytest.raises(bdpt_amd.BdptError, match="rr_depth"):
        bdpt_amd.BDPTIntegrator(sc, deep).render_frame()


@pytest.mark.parametrize("name", ["G1_cbox_low_64x64_spp4", "G2_caustic_64x64_spp16"])
def test_gpu_hbm_table_build_matches_golden(name, golden_manifest, monkeypatch):
    """The HBM-table build forced on a small scene (BDPT_BSDF_IN_HBM=1 at context
    creation): the reference's frame."""
    monkeypatch.setenv("BDPT_BSDF_IN_HBM", "1")
    m = golden_manifest["framebuffers"][name]
    it = integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"], STRATEGY[m.get("strategy", "bdpt")])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    worst, exact, _ = report(fb, load_golden(name))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"


def test_gpu_camera_facing_away_renders_black():
    cam = dict(variants.SCENES["caustic"]["camera"])
    cam["at"] = [0.0, 0.8, 10.0]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=16, height=16, spp=4, rr_depth=8)
    it = bdpt_amd.BDPTIntegrator(scene("caustic"), cfg)
    it.init()
    fb = it.render_frame()
    sc = O.Scene(variants.obj_path("caustic"))
    ref, _ = sc.render(O.make_params(cam, 16, 16, 4, 8))
    assert np.array_equal(fb.reshape(-1), ref)


def test_gpu_row_shards_sum_to_full_frame():
    full = integrator("hardlight", 48, 32, 8, 2).render_frame().copy()
    acc = np.zeros_like(full)
    for r in range(4):
        it = integrator("hardlight", 48, 32, 8, 2)
        acc += it.render_frame(row_offset=r, row_stride=4)
    assert rel_l2(acc, full).max() <= 1e-5


def test_gpu_empty_shard_leaves_framebuffer_untouched():
    it = integrator("cbox_low", 8, 8, 2, 5)
    it.rgb[:] = 7.0
    fb = it.render_frame(row_offset=8, row_stride=1)
    assert it.stats()["samples"] == 0
    assert np.all(fb == 7.0)


def driver_ray(p, name, pixel, k, eye=None):
    """The camera ray and sampler the offline driver hands to render() for
    sample k of `pixel` (renderer.cpp:162-192: jitter draws first when spp > 1)."""
    W, spp = p.width, p.spp
    cam = O.camera(p)
    c2w = cam[16:32].reshape(4, 4)  # column-major: c2w[col][row]
    invW, invH, angle, aspect = cam[64:68]
    rs = np.random.RandomState(260450963 + pixel * spp + k)
    u = rs.randint(0, 2**32, size=2, dtype=np.uint32).astype(np.float32) / np.float32(2**32)
    j, i = pixel % W, pixel // W
    f32 = np.float32
    y = (f32(1) - (f32(i) + f32(0.5)) * invH) * f32(2) - f32(1)
    x = ((f32(j) + f32(0.5)) * invW) * f32(2) - f32(1)
    px = ((x + (u[0] - f32(0.5)) * invW) * angle) * aspect
    py = (y + (u[1] - f32(0.5)) * invH) * angle
    d = [(c2w[0][r] * px + c2w[1][r] * py) + (c2w[2][r] * f32(-1) + c2w[3][r] * f32(0)) for r in range(3)]
    d = np.array(d, np.float32)
    d = d * (f32(1) / np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
    sampler = bdpt_amd.Sampler.for_sample(pixel, spp, k)
    assert np.float32(sampler.next()) == u[0] and np.float32(sampler.next()) == u[1]  # the jitter draws
    eye = eye if eye is not None else variants.SCENES[name]["camera"]["eye"]
    return bdpt_amd.Ray(tuple(eye), tuple(d), 1.0, 1000.0), sampler


@pytest.mark.parametrize("rr", [40, 150])
def test_gpu_single_sample_api_deep_rr_depth(rr, tmp_path):
    """render(ray, sampler) past the lazy MT19937 window: in the closed box
    every path runs to rrDepth (hundreds of draws per sample); the sample kernel
    continues the caller's generator state in HBM, same Li, splats and final
    generator state as the oracle."""
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    W, H, spp = 8, 6, 2
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr)
    it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(obj), cfg)
    it.init()
    p = O.make_params(cam, W, H, spp, rr)
    sc = O.Scene(obj)
    for pixel, k in [(0, 0), (27, 1), (47, 1)]:
        it.rgb[:] = 0
        Li_ref, splats_ref = sc.sample(p, pixel, k)
        ray, sampler = driver_ray(p, None, pixel, k, eye=cam["eye"])
        Li = it.render(ray, sampler)
        assert np.allclose(Li, Li_ref, rtol=1e-6, atol=0), (pixel, Li, Li_ref)
        assert rel_l2(it.rgb.reshape(-1), splats_ref).max() <= TOL


@pytest.mark.parametrize("pixel,k", [(0, 0), (2080, 3), (1000, 15), (4095, 7), (2500, 9)])
def test_gpu_single_sample_api_matches_oracle(pixel, k):
    """BDPTIntegrator.render(ray, sampler) == the reference's render() for one sample."""
    W = H = 64
    spp = 16
    it = integrator("caustic", W, H, spp, 8)
    p = O.make_params(variants.SCENES["caustic"]["camera"], W, H, spp, 8)
    sc = O.Scene(variants.obj_path("caustic"))
    Li_ref, splats_ref = sc.sample(p, pixel, k)
    ray, sampler = driver_ray(p, "caustic", pixel, k)
    before = sampler.state.copy()
    Li = it.render(ray, sampler)
    assert np.allclose(Li, Li_ref, rtol=1e-6, atol=0), (Li, Li_ref)
    assert rel_l2(it.rgb.reshape(-1), splats_ref).max() <= TOL
    assert before[624] != sampler.state[624]  # the sampler advanced


def test_gpu_counting_pass_is_consistent():
    it = integrator("caustic", 32, 32, 8, 8)
    it.render_frame(flags=bdpt_amd.FLAG_COUNT)
    st = it.stats()
    c = st["counters"]
    n = st["samples"]
    assert n == 32 * 32 * 8
    assert c["closest_rays"] >= n and c["shadow_rays"] > 0
    assert c["rng_draws"] >= 10 * n // 2
    assert c["light_vert_reads"] >= c["light_verts"]
    # the count pass renders the same image
    it2 = integrator("caustic", 32, 32, 8, 8)
    assert rel_l2(it2.render_frame(), it.rgb).max() <= TOL


def test_gpu_full_size_caustic_properties(golden_manifest):
    """BASELINE config[1] size (512^2): finite, non-negative, energy consistent
    with the reference's 64^2 x 16 spp image mean, deterministic."""
    it = integrator("caustic", 512, 512, 16, 8)
    fb = it.render_frame().copy()
    assert np.all(np.isfinite(fb)) and fb.min() >= 0.0
    ref_mean = np.array(golden_manifest["framebuffers"]["G2_caustic_64x64_spp16"]["mean_rgb"])
    mean = fb.reshape(-1, 3).mean(0)
    assert np.all(np.abs(mean - ref_mean) / ref_mean < 0.03), (mean, ref_mean)
    it2 = integrator("caustic", 512, 512, 16, 8)
    assert rel_l2(it2.render_frame(), fb).max() <= TOL


def test_gpu_cli_renders_toml_to_reference_exr(tmp_path):
    """tinyrender_amd <scene.toml> (src/main.cpp:121-181 on the GPU path): the
    reference's own scene file shape (cbox_bdpt_glass.toml with the film and spp
    overridden) renders G1's configuration; its EXR decodes to the golden
    framebuffer within one half-precision ulp (the EXR is half; the GPU frame
    differs from the reference only by atomic summation order)."""
    import os
    import subprocess

    from test_config_exr import decode_exr

    obj = variants.obj_path("cbox_low")
    toml = tmp_path / "cbox_low.toml"
    toml.write_text(f'[input]\nobjfile = "{obj}"\n[camera]\neye = [ 0.0, 0.8, 3.8 ]\nat = [ 0.0, 0.8, 0.0 ]\n'
                    'up = [ 0.0, 1.0, 0.0 ]\nfov = 30.0\n[film]\nwidth = 64\nheight = 64\n[renderer]\n'
                    'realtime = false\ntype = "bdpt"\nrrDepth = 5\nrrProb = 0.95\nspp = 4\n')
    cli = os.path.join(os.path.dirname(bdpt_amd.LIB_PATH), "tinyrender_amd")
    r = subprocess.run([cli, str(toml), "nogui"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Render took" in r.stdout and "Saved EXR image to" in r.stdout
    img = decode_exr((tmp_path / "cbox_low.exr").read_bytes()).astype(np.float32)
    ref = load_golden("G1_cbox_low_64x64_spp4").reshape(64, 64, 3).astype(np.float16).astype(np.float32)
    assert np.allclose(img, ref, rtol=2 ** -10, atol=0)


PATH_CASES = ["P1_hardlight_path_64x64_spp4", "P2_caustic_path_64x64_spp4", "P3_caustic_path_mis_48x48_spp4",
              "P4_cbox_low_path_implicit_64x64_spp4", "P5_hardlight_path_maxdepth3_48x48_spp4"]


@pytest.mark.parametrize("name", PATH_CASES)
def test_gpu_path_tracer_matches_reference_golden(name, golden_manifest):
    """PathTracerIntegrator (path.h) on the GPU substrate against frames the
    reference rendered (explicit with Russian roulette, MIS direct light,
    implicit, bounded depth)."""
    m = golden_manifest["path_framebuffers"][name]
    cam = bdpt_amd.Camera(**variants.SCENES[m["scene"]]["camera"])
    cfg = bdpt_amd.Config(camera=cam, width=m["width"], height=m["height"], spp=m["spp"])
    it = bdpt_amd.PathTracerIntegrator(scene(m["scene"]), cfg, bdpt_amd.PathSettings(**m["path"]))
    fb = it.render_frame().reshape(-1)
    assert it.stats()["samples"] == m["samples"]
    assert it.stats()["counters"]["shadow_rays"] == 0  # counters[1]: level-stack overflows
    ref = load_golden(name)
    worst, exact, whole = report(fb, ref)
    assert np.all(np.isfinite(fb))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


def test_gpu_path_tracer_render_device_and_level_check(golden_manifest):
    """The asynchronous path-tracer entry bench.py uses (device framebuffer, the
    caller's stream), then check_levels() after the sync: same frame as the golden."""
    import torch

    name = sorted(golden_manifest["path_framebuffers"])[0]
    m = golden_manifest["path_framebuffers"][name]
    cam = bdpt_amd.Camera(**variants.SCENES[m["scene"]]["camera"])
    cfg = bdpt_amd.Config(camera=cam, width=m["width"], height=m["height"], spp=m["spp"])
    it = bdpt_amd.PathTracerIntegrator(scene(m["scene"]), cfg, bdpt_amd.PathSettings(**m["path"]))
    fb = torch.zeros(m["width"] * m["height"] * 3, dtype=torch.float32, device="cuda:0")
    s = torch.cuda.Stream()
    it.render_device(fb.data_ptr(), s.cuda_stream)
    s.synchronize()
    it.check_levels()
    assert rel_l2(fb.cpu().numpy(), load_golden(name)).max() <= TOL


def test_gpu_path_tracer_long_paths_match_oracle():
    """Russian roulette with rrProb 0.99 past depth 1: most samples draw more
    than 227 numbers and run on the ring-buffer generator; many recursion levels."""
    import oracle as O

    cam = variants.SCENES["cbox_low"]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=32, height=24, spp=4)
    ps = dict(rr_depth=1, rr_prob=0.99, emitter_samples=6, bsdf_samples=2)  # ~31 draws per level
    it = bdpt_amd.PathTracerIntegrator(scene("cbox_low"), cfg, bdpt_amd.PathSettings(**ps))
    fb = it.render_frame().reshape(-1)
    c = it.stats()["counters"]
    assert c["interior_visits"] > 0 and c["tri_tests"] > 0  # [2] / [3]: samples past 227 / 624 draws
    ref, _ = O.Scene(variants.obj_path("cbox_low")).render(O.make_path_params(cam, 32, 24, 4, **ps))
    worst, exact, whole = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


def test_gpu_cli_renders_path_toml(tmp_path):
    """tinyrender_amd on a type = "path" scene file (the reference's
    cbox_bdpt_path.toml settings) matches the reference golden P1."""
    import os
    import subprocess

    from test_config_exr import decode_exr

    toml = tmp_path / "hard_path.toml"
    toml.write_text(variants.path_toml_text("hardlight", 64, 64, 4))
    cli = os.path.join(os.path.dirname(bdpt_amd.LIB_PATH), "tinyrender_amd")
    r = subprocess.run([cli, str(toml)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = decode_exr((tmp_path / "hard_path.exr").read_bytes()).astype(np.float32)
    ref = load_golden("P1_hardlight_path_64x64_spp4").reshape(64, 64, 3).astype(np.float16).astype(np.float32)
    assert np.allclose(img, ref, rtol=2 ** -10, atol=0)


DIRECT_CASES = ["D1_caustic_direct_area_48x48_spp4", "D2_hardlight_direct_solidangle_48x48_spp4",
                "D3_caustic_direct_cosine_48x48_spp4", "D4_hardlight_direct_bsdf_48x48_spp4",
                "D5_caustic_direct_mis_48x48_spp4", "D6_hardlight_direct_mis_48x48_spp4"]


@pytest.mark.parametrize("name", DIRECT_CASES)
def test_gpu_direct_integrator_matches_reference_golden(name, golden_manifest):
    """DirectIntegrator (direct.h), each samplingStrategy, against frames the
    reference rendered (sphere emitters, double-precision sphere test)."""
    m = golden_manifest["direct_framebuffers"][name]
    cam = bdpt_amd.Camera(**variants.SCENES[m["scene"]]["camera"])
    cfg = bdpt_amd.Config(camera=cam, width=m["width"], height=m["height"], spp=m["spp"])
    d = m["direct"]
    ds = bdpt_amd.DirectSettings(sampling_strategy=d["strategy"], emitter_samples=d.get("emitter_samples", 1),
                                 bsdf_samples=d.get("bsdf_samples", 1))
    it = bdpt_amd.DirectIntegrator(scene(m["scene"]), cfg, ds)
    fb = it.render_frame().reshape(-1)
    assert it.stats()["samples"] == m["samples"]
    ref = load_golden(name)
    worst, exact, whole = report(fb, ref)
    assert np.all(np.isfinite(fb))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


@pytest.mark.parametrize("strategy", ["area", "solidAngle", "cosineHemisphere", "bsdf", "mis"])
def test_gpu_direct_integrator_matches_oracle(strategy):
    """Every strategy on the glossy/glass cbox at more samples per pixel than the goldens."""
    import oracle as O

    cam = variants.SCENES["caustic"]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=40, height=32, spp=8)
    ds = bdpt_amd.DirectSettings(sampling_strategy=strategy, emitter_samples=3, bsdf_samples=2)
    fb = bdpt_amd.DirectIntegrator(scene("caustic"), cfg, ds).render_frame().reshape(-1)
    ref, _ = O.Scene(variants.obj_path("caustic")).render(
        O.make_direct_params(cam, 40, 32, 8, strategy=strategy, emitter_samples=3, bsdf_samples=2))
    worst, exact, whole = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


def test_gpu_direct_integrator_rejects_unknown_strategy():
    """samplingStrategy's default "emitter" is not a strategy (direct.h:460-461)."""
    cam = variants.SCENES["caustic"]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=8, height=8, spp=1)
    it = bdpt_amd.DirectIntegrator(scene("caustic"), cfg, bdpt_amd.DirectSettings())
    with pytest.raises(bdpt_amd.BdptError, match="wrong strategy"):
        it.render_frame()


def test_gpu_cli_renders_direct_toml(tmp_path):
    """tinyrender_amd on a type = "direct" scene file matches the reference golden D5."""
    import os
    import subprocess

    from test_config_exr import decode_exr

    toml = tmp_path / "caustic_direct.toml"
    toml.write_text(variants.direct_toml_text("caustic", 48, 48, 4, strategy="mis", emitter_samples=2,
                                              bsdf_samples=2))
    cli = os.path.join(os.path.dirname(bdpt_amd.LIB_PATH), "tinyrender_amd")
    r = subprocess.run([cli, str(toml)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = decode_exr((tmp_path / "caustic_direct.exr").read_bytes()).astype(np.float32)
    ref = load_golden("D5_caustic_direct_mis_48x48_spp4").reshape(48, 48, 3).astype(np.float16).astype(np.float32)
    assert np.allclose(img, ref, rtol=2 ** -10, atol=0)
    bad = tmp_path / "bad.toml"
    bad.write_text(variants.direct_toml_text("caustic", 8, 8, 1, strategy="emitter"))
    r = subprocess.run([cli, str(bad)], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "Error: wrong strategy" in r.stdout


@pytest.mark.parametrize("integrator", ["bdpt", "path", "direct"])
def test_gpu_many_shapes_scene_matches_oracle(integrator, tmp_path):
    """7008 shapes: the shape -> emitter map no longer fits the LDS tables and is
    read from HBM (lds_shape_off == kNoLds); every integrator that maps a hit
    shape to its emitter still matches the oracle."""
    import oracle as O

    obj = variants.many_shapes_obj(str(tmp_path))
    cam = variants.CBOX_CAMERA
    W, H, spp = 32, 24, 4
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=5)
    sc = bdpt_amd.Scene(obj)
    assert sc.info()["shapes"] == 7008
    if integrator == "bdpt":
        fb = bdpt_amd.BDPTIntegrator(sc, cfg).render_frame().reshape(-1)
        p = O.make_params(cam, W, H, spp, 5)
    elif integrator == "path":
        fb = bdpt_amd.PathTracerIntegrator(sc, cfg, bdpt_amd.PathSettings(bsdf_samples=1)).render_frame().reshape(-1)
        p = O.make_path_params(cam, W, H, spp, bsdf_samples=1)
    else:
        ds = bdpt_amd.DirectSettings(sampling_strategy="mis", emitter_samples=2, bsdf_samples=2)
        fb = bdpt_amd.DirectIntegrator(sc, cfg, ds).render_frame().reshape(-1)
        p = O.make_direct_params(cam, W, H, spp, strategy="mis", emitter_samples=2, bsdf_samples=2)
    ref, _ = O.Scene(obj).render(p)
    worst, exact, whole = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f}, image {whole:.3g})"


@pytest.mark.parametrize("fn", ["sinf", "cosf", "sincos_s", "sincos_c", "powf"])
def test_gpu_device_libm_is_bit_exact(fn):
    """The device restatements of glibc 2.35's sinf / cosf / powf against the C
    oracle's (itself bit-exact to the host libm, test_oracle_golden.py): random
    bit patterns (|x| >= 120 takes the large-argument reduction), the angles the
    warps produce, and powf over the cosine / exponent domain the BSDFs use
    (zero, subnormal and 1 included)."""
    import oracle as O

    rng = np.random.default_rng(2024)
    n = 400_000
    y = None
    if fn == "powf":
        x = rng.random(n, dtype=np.float32)
        x[:64] = np.array([0.0, 1.0, 1e-45, 1e-40, 1.1754944e-38, 0.5, 0.999999, 1e-7] * 8, np.float32)
        x[64:20000] = (x[64:20000] ** 8).astype(np.float32)  # near 0
        ex = np.array([9.803922, 100.0, 30.0, 1.0, 0.0, 2.0, 5.5, 250.0], np.float32)
        y = ex[rng.integers(0, len(ex), n)]
        y[1::3] = (np.float32(1.0) / (y[1::3] + np.float32(2.0))).astype(np.float32)  # squareToPhongLobe exponent
        ref = np.frompyfunc(lambda a, b: O.lib().tro_powf(float(a), float(b)), 2, 1)(x, y).astype(np.float32)
    else:
        bits = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        x = bits.view(np.float32).copy()
        x[~np.isfinite(x)] = 1.0
        x[: n // 2] = (rng.random(n // 2, dtype=np.float32) * np.float32(np.pi) * np.float32(2.0)).astype(np.float32)
        f = O.lib().tro_sinf if fn in ("sinf", "sincos_s") else O.lib().tro_cosf
        ref = np.frompyfunc(lambda a: f(float(a)), 1, 1)(x).astype(np.float32)
    got = bdpt_amd.debug_math(fn, x, y)
    bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"{bad.size} mismatches, first x={x[bad[0]]!r} y={None if y is None else y[bad[0]]!r}"


@pytest.mark.parametrize("seed", range(8))
def test_gpu_randomized_configs_match_oracle(seed):
    """Seeded random configurations of the BDPT path (scene, odd sizes, spp,
    rrDepth up to 40 so some run on the deep build, strategy, a row shard, a
    non-default seed base) against the oracle."""
    rng = np.random.default_rng(1000 + seed)
    name = ["cbox_low", "caustic", "hardlight", "hardlight_mirror"][int(rng.integers(0, 4))]
    W, H = int(rng.integers(5, 33)), int(rng.integers(5, 33))
    spp = int(rng.integers(1, 7))
    rr = int(rng.choice([1, 2, 3, 5, 8, 13, 28, 33, 40]))
    strategy = int(rng.integers(0, 3))
    stride = int(rng.integers(1, 4))
    off = int(rng.integers(0, stride))
    base = int(rng.integers(0, 2 ** 32))
    cam = variants.SCENES[name]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr, strategy=strategy,
                          seed_base=base)
    fb = bdpt_amd.BDPTIntegrator(scene(name), cfg).render_frame(row_offset=off, row_stride=stride).reshape(-1)
    p = O.make_params(cam, W, H, spp, rr, strategy)
    p.seed_base = base
    ref, _ = O.Scene(variants.obj_path(name)).render(p, rows=list(range(off, H, stride)))
    worst, exact, _ = report(fb, ref)
    assert worst <= TOL, (f"{name} {W}x{H}x{spp} rr={rr} strategy={strategy} rows {off}::{stride} base={base}: "
                          f"max per-pixel rel L2 {worst:.3g}")


@pytest.mark.parametrize("integ", ["path", "path_mis", "direct_mis", "direct_area"])
def test_gpu_single_sample_api_other_integrators(integ):
    """PathTracerIntegrator / DirectIntegrator.render(ray, sampler) == the
    reference's render() of one sample (oracle), over several pixels."""
    name, W, H, spp = "caustic", 48, 48, 8
    cam = variants.SCENES[name]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp)
    if integ.startswith("path"):
        ps = dict(emitter_samples=2, bsdf_samples=2) if integ == "path_mis" else {}
        it = bdpt_amd.PathTracerIntegrator(scene(name), cfg, bdpt_amd.PathSettings(**ps))
        p = O.make_path_params(cam, W, H, spp, **ps)
    else:
        st = integ.split("_")[1]
        it = bdpt_amd.DirectIntegrator(scene(name), cfg, bdpt_amd.DirectSettings(sampling_strategy=st,
                                                                                  emitter_samples=2))
        p = O.make_direct_params(cam, W, H, spp, strategy=st, emitter_samples=2)
    sc = O.Scene(variants.obj_path(name))
    for pixel, k in [(0, 0), (1111, 3), (1200, 7), (2000, 5), (1500, 1), (700, 6)]:
        Li_ref, _ = sc.sample(p, pixel, k)
        ray, sampler = driver_ray(p, name, pixel, k)
        Li = it.render(ray, sampler)
        assert np.allclose(Li, Li_ref, rtol=1e-6, atol=0), (pixel, k, Li, Li_ref)


# ---- Russian roulette (the reference's NO_RR = 0 branch, bdpt.h:18, :68, :129-132, :188, :201-204)
RR_CASES = ["R1_caustic_rr_64x64_spp16", "R2_hardlight_rr_64x64_spp16", "R3_cbox_low_rr_64x64_spp4",
            "R4_caustic_rr1_48x48_spp4", "R5_hardlight_mirror_rr_48x48_spp4", "R6_caustic_rr_512x512_spp2_rows32"]


def rr_integrator(name, W, H, spp, rr, obj=None, cam=None):
    cam = cam or variants.SCENES[name]["camera"]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**cam), width=W, height=H, spp=spp, rr_depth=rr,
                          russian_roulette=bdpt_amd.RR_LUMINANCE)
    it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(obj) if obj else scene(name), cfg)
    it.init()
    return it


@pytest.mark.parametrize("name", RR_CASES)
def test_gpu_russian_roulette_matches_reference_golden(name, golden_manifest):
    """The RR build of the megakernel (bdpt_kernels_rr.hip) against the reference
    compiled with NO_RR = 0 (oracle/_ref/ref_bdpt_rr)."""
    m = golden_manifest["rr_framebuffers"][name]
    it = rr_integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    assert it.stats()["capped_samples"] == 0
    worst, exact, _ = report(fb, load_golden(name))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"


@pytest.mark.parametrize("rr,W,H,spp", [(2, 24, 16, 4), (6, 16, 12, 4), (40, 12, 8, 2)])
def test_gpu_russian_roulette_closed_box_matches_oracle(rr, W, H, spp, tmp_path):
    """In the closed box no path escapes: subpaths end only by roulette (p = 0.5
    once the throughput's luminance is below 0.01), so they run long and draw
    far past the lazy MT19937 window; same frame as the oracle's NO_RR = 0."""
    obj = variants.closed_box_obj(str(tmp_path))
    cam = variants.CLOSED_CAMERA
    it = rr_integrator(None, W, H, spp, rr, obj=obj, cam=cam)
    fb = it.render_frame().reshape(-1)
    assert it.stats()["capped_samples"] == 0
    O.walk_stats(True)
    ref, n = O.Scene(obj).render(O.make_params(cam, W, H, spp, rr, 0, russian_roulette=1))
    ws = O.walk_stats(True)
    assert ws["max_light_depth"] > rr + 2 and ws["max_eye_depth"] > rr + 2  # paths go past rrDepth
    worst, exact, _ = report(fb, ref.reshape(-1))
    assert worst <= TOL, f"rr={rr}: max per-pixel rel L2 {worst:.3g} (bit-exact {exact:.4f})"


@pytest.mark.parametrize("pixel,k", [(0, 0), (2080, 3), (1000, 15), (4095, 7), (2500, 9), (1234, 1)])
def test_gpu_russian_roulette_single_sample_matches_oracle(pixel, k):
    """render(ray, sampler) with NO_RR = 0: Li and the splat list as the oracle's sample."""
    W = H = 64
    spp, rr = 16, 3
    it = rr_integrator("caustic", W, H, spp, rr)
    p = O.make_params(variants.SCENES["caustic"]["camera"], W, H, spp, rr, 0, russian_roulette=1)
    sc = O.Scene(variants.obj_path("caustic"))
    Li_ref, splats_ref = sc.sample(p, pixel, k)
    ray, sampler = driver_ray(p, "caustic", pixel, k)
    Li = it.render(ray, sampler)
    assert np.allclose(Li, Li_ref, rtol=1e-6, atol=0), (Li, Li_ref)
    assert rel_l2(it.rgb.reshape(-1), splats_ref).max() <= TOL


def test_gpu_russian_roulette_limits():
    """An unknown mode is an error; rrDepth past 1024 is refused with roulette too."""
    it = rr_integrator("cbox_low", 8, 8, 1, 1025)
    with pytest.raises(bdpt_amd.BdptError, match="rr_depth"):
        it.render_frame()
    it = integrator("cbox_low", 8, 8, 1, 5)
    it.config.russian_roulette = 7
    with pytest.raises(bdpt_amd.BdptError, match="russian_roulette"):
        it.render_frame()


# Both frame-kernel builds on every BDPT golden: the default sweep order and the
# short-subpath build (BDPT_SPLIT_CONTINUE, bdpt_kernels_split.hip; chosen per render
# for rrDepth <= 3), forced through BDPT_SPLIT_MAX_RR, which the library reads per render.
@pytest.mark.parametrize("build,max_rr", [("default", "0"), ("split", "1024")])
@pytest.mark.parametrize("name", FB_CASES[:8] + ["G9_caustic_lt_64x64_spp16", "G12_hardlight_pt_64x64_spp16"])
def test_gpu_both_sweep_builds_match_reference_golden(name, build, max_rr, golden_manifest, monkeypatch):
    monkeypatch.setenv("BDPT_SPLIT_MAX_RR", max_rr)
    m = golden_manifest["framebuffers"][name]
    it = integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"], STRATEGY[m.get("strategy", "bdpt")])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    assert it.stats()["kernel"] == ("bdpt_frame_kernel_split" if build == "split" else "bdpt_frame_kernel")
    worst, exact, whole = report(fb, load_golden(name))
    assert worst <= TOL, f"{build}: max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"
