"""Per-function parity on the GPU: each piece of the BDPT path, through the
C-ABI, against the reference's own function on the same inputs.

Fixtures: tests/golden/kat_*.npz, made by tests/golden/make_kat_goldens.py with
oracle/_ref/ref_bdpt (the unmodified reference sources, `kat` and
`sample_state` modes of oracle/ref/ref_driver.cpp). The device functions
restate the reference's fp32 operation order and glibc's sinf / cosf / powf
bit for bit, so the bar is bit-exact (np.array_equal on the float32 bits).
"""
import os

import numpy as np
import pytest

import bdpt_amd
import variants

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BSDF_SCENES = ["caustic", "hardlight", "hardlight_mirror", "hardlight_phong", "cbox_low"]
_integ = {}


def kat(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def integrator(scene, W=64, H=64, spp=16, rr=None, kind="bdpt", **kw):
    key = (scene, W, H, spp, rr, kind, tuple(sorted(kw.items())))
    if key not in _integ:
        sc = bdpt_amd.Scene(variants.obj_path(scene))
        cam = bdpt_amd.Camera(**variants.SCENES[scene]["camera"])
        cfg = bdpt_amd.Config(camera=cam, width=W, height=H, spp=spp,
                              rr_depth=rr if rr is not None else variants.SCENES[scene]["rr_depth"])
        if kind == "path":
            it = bdpt_amd.PathTracerIntegrator(sc, cfg, bdpt_amd.PathSettings(**kw))
        elif kind == "direct":
            it = bdpt_amd.DirectIntegrator(sc, cfg, bdpt_amd.DirectSettings(**kw))
        else:
            it = bdpt_amd.BDPTIntegrator(sc, cfg)
        it.init()
        _integ[key] = it
    return _integ[key]


def same_bits(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32)) or np.array_equal(a, b)


@pytest.mark.parametrize("scene", BSDF_SCENES)
def test_gpu_bsdf_eval_pdf_sample_match_reference(scene):
    """BSDF::eval / pdf / sample (core.h:308-310) of every material of the scene:
    diffuse.h, perfectmirror.h, glass.h (Fresnel, TIR), mixture.h, phong.h."""
    g = kat(f"kat_bsdf_{scene}")
    it = integrator(scene)
    live = g["null"] == 0
    mat, wo, wi, u = g["mat"][live], g["wo"][live], g["wi"][live], g["u"][live]
    f = it.bsdf_eval(mat, wo, wi)
    assert same_bits(f, g["eval"][live]), np.abs(f - g["eval"][live]).max()
    pdf = it.bsdf_pdf(mat, wo, wi)
    assert same_bits(pdf, g["pdf"][live]), np.abs(pdf - g["pdf"][live]).max()
    sf, swi, spdf = it.bsdf_sample(mat, wo, u)
    assert same_bits(sf, g["sample_f"][live])
    assert same_bits(swi, g["sample_wi"][live])
    assert same_bits(spdf, g["sample_pdf"][live])
    for m in np.unique(mat):  # BSDF::getType() flags
        t, kind = it.scene.bsdf_type(int(m))
        assert t == int(g["type"][live][mat == m][0]), (m, t, kind)


def test_gpu_fresnel_matches_reference():
    g = kat("kat_fresnel")
    assert same_bits(bdpt_amd.debug_fresnel(g["inp"]), g["out"])


def test_gpu_triangle_test_matches_reference():
    """rayTriangleIntersect (core.h:379-400): hit / miss everywhere, (t, u, v) on hits."""
    g = kat("kat_triangle")
    out = bdpt_amd.debug_triangle(g["rays"], g["verts"])
    ref = g["out"]
    assert np.array_equal(out[:, 0], ref[:, 0])
    hit = ref[:, 0] == 1
    assert same_bits(out[hit, 1:], ref[hit, 1:])


@pytest.mark.parametrize("scene", ["caustic", "hardlight", "cbox_low"])
def test_gpu_intersect_matches_reference(scene):
    """AcceleratorBVH::intersect (accel.h:125-172) and the occlusion query
    (bvh.h:259-352) on camera rays, rays from inside the box (axis-parallel
    ones included) and shadow segments: acceptance and every field of the
    SurfaceInteraction it fills (t of an accepted hit, u, v, ids, p, frameNs.n,
    frameNg.n, wo)."""
    g = kat(f"kat_intersect_{scene}")
    it = integrator(scene)
    h = it.intersect(g["rays"])
    ref = g["out"]
    assert np.array_equal(h["hit"], ref[:, 0].astype(np.int32))
    k = ref[:, 0] == 1
    r = ref[k]
    hh = h[k]
    assert same_bits(hh["t"], r[:, 1]) and same_bits(hh["u"], r[:, 2]) and same_bits(hh["v"], r[:, 3])
    assert np.array_equal(hh["shape_id"], r[:, 4].view(np.int32))
    assert np.array_equal(hh["prim_id"], r[:, 5].view(np.int32))
    assert np.array_equal(hh["mat_id"], r[:, 6].view(np.int32))
    assert same_bits(hh["p"], r[:, 7:10]) and same_bits(hh["ns"], r[:, 10:13])
    assert same_bits(hh["ng"], r[:, 13:16]) and same_bits(hh["wo"], r[:, 16:19])
    occ = it.intersect(g["rays"], occlusion=True)
    assert np.array_equal(occ["hit"], ref[:, 20].astype(np.int32))


@pytest.mark.parametrize("scene", ["caustic", "hardlight", "synth1m"])
def test_gpu_intersect_adversarial_rays_match_reference(scene):
    """Where the traversal's exactness argument is thinnest (DESIGN.md §2 items
    5-6; tests/golden/make_kat_goldens.py adversarial_rays): grazing continuation
    rays and shadow segments along the large triangles (|det| down to 1e-8),
    rays through the curved mesh's shared vertices and edges (ties), rays
    starting on surfaces, and origins 100 - 10000 scene diagonals away. Closest
    hit (acceptance, t, u, v, shape, prim) and occlusion bit for bit against the
    reference's AcceleratorBVH; the in-scene batches run the frames' slack-free
    interior test, the far batch and the mixed batch the slack test (far origins
    themselves walk the reference's tree), each without the near cull, with the
    near cull skipped at |cos| < 0.02 to the origin triangle's plane normal, and
    with the frames' own rule (cull_near_for): the interpolated shading normal
    the path holds at the origin plus that triangle's graze code. Kinds 6 and 7
    leave the curved mesh nearly parallel to a triangle whose shading normal is
    tilted from its plane normal (1.7 k such rays in Caustic graze
    the plane at |cos| < 0.02 while |cos| to the shading normal is >= 0.02)."""
    g = kat(f"kat_adversarial_{scene}")
    it = integrator(scene)
    rays, kind, onrm, otri, osn = g["rays"], g["kind"], g["onrm"], g["otri"], g["osn"]
    far = kind == 4
    every = np.ones_like(far)
    cases = ((~far, None, None), (far, None, None), (every, None, None), (~far, onrm[~far], None),
             (every, onrm, None), (~far, osn[~far], otri[~far]), (every, osn, otri))
    for sel, nrm, tris in cases:
        h = it.intersect(rays[sel], origin_normals=nrm, origin_tris=tris)
        hit = g["hit"][sel].astype(np.int32)
        bad = np.flatnonzero(h["hit"] != hit)
        assert bad.size == 0, f"{bad.size} acceptance mismatches, kinds {np.bincount(kind[sel][bad])}"
        k = hit == 1
        assert same_bits(h["t"][k], g["t"][sel][k]) and same_bits(h["u"][k], g["u"][sel][k])
        assert same_bits(h["v"][k], g["v"][sel][k])
        assert np.array_equal(h["shape_id"][k], g["shape"][sel][k]) and np.array_equal(h["prim_id"][k],
                                                                                          g["prim"][sel][k])
        occ = it.intersect(rays[sel], occlusion=True, origin_normals=nrm, origin_tris=tris)
        bad = np.flatnonzero(occ["hit"] != g["occluded"][sel].astype(np.int32))
        assert bad.size == 0, f"{bad.size} occlusion mismatches, kinds {np.bincount(kind[sel][bad])}"


def test_gpu_splat_to_image_plane_matches_reference():
    """splatToImagePlane (bdpt.h:485-496), incl. points behind the camera and off
    the image (the reference's int truncation)."""
    g = kat("kat_splat")
    for W, H in [(64, 64), (512, 512), (80, 48)]:
        it = integrator("caustic", W, H, 1)
        xy = it.splat_to_image_plane(g[f"p_{W}x{H}"])
        assert np.array_equal(xy, g[f"xy_{W}x{H}"]), (W, H)


SAMPLERS = {
    "bdpt_caustic": dict(scene="caustic", kind="bdpt"),
    "bdpt_hardlight_rr12": dict(scene="hardlight", kind="bdpt"),
    "path_caustic": dict(scene="caustic", kind="path"),
    "direct_hardlight": dict(scene="hardlight", kind="direct", sampling_strategy="mis", emitter_samples=2,
                             bsdf_samples=2),
}


@pytest.mark.parametrize("name", list(SAMPLERS))
def test_gpu_render_ray_sampler_matches_reference(name):
    """Integrator::render(const Ray&, Sampler&) (integrator.h:31) from arbitrary
    std::mt19937 states (seeded, advanced across twists, arbitrary words and
    positions): Li, the sampler state after the call and the camera splats."""
    g = kat(f"kat_sampler_{name}")
    cfg = dict(SAMPLERS[name])
    scene, kind = cfg.pop("scene"), cfg.pop("kind")
    W, H, spp, rr = int(g["width"]), int(g["height"]), int(g["spp"]), int(g["rr"])
    it = integrator(scene, W, H, spp, rr if kind == "bdpt" else None, kind, **cfg)
    for i in range(g["rays"].shape[0]):
        r = g["rays"][i]
        ray = bdpt_amd.Ray(tuple(r[:3]), tuple(r[3:6]), float(r[6]), float(r[7]))
        s = bdpt_amd.Sampler.from_state(g["state_in"][i])
        if kind == "bdpt":
            Li, splats = it.render_sample(ray, s)
            acc = {}
            for px, v in splats:
                acc[px] = acc.get(px, np.zeros(3, np.float32)) + v
            n = int(g["nsplat"][i])
            assert len(acc) == n, (i, len(acc), n)
            for px, rr_, gg, bb in g["splats"][i][: min(n, 16)]:
                got = acc[int(np.float32(px).view(np.int32))]
                assert same_bits(got, np.array([rr_, gg, bb], np.float32)), (i, got)
        else:
            Li = it.render(ray, s)
        assert same_bits(Li, g["Li"][i]), (i, Li, g["Li"][i])
        assert np.array_equal(s.state, g["state_out"][i]), i


def test_gpu_sample_call_is_ordered_after_async_frame_on_another_stream(golden_manifest):
    """A frame rendered asynchronously on a caller's stream, then at once a
    render(ray, sampler) on the same context (its own stream): the context's
    buffers are not reused under the running frame."""
    import torch

    from conftest import load_golden

    name = "G2_caustic_64x64_spp16"
    m = golden_manifest["framebuffers"][name]
    sc = bdpt_amd.Scene(variants.obj_path("caustic"))
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**variants.SCENES["caustic"]["camera"]), width=64, height=64,
                          spp=16, rr_depth=8)
    it = bdpt_amd.BDPTIntegrator(sc, cfg)
    s = torch.cuda.Stream()
    fb = torch.zeros(64 * 64 * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    it.render_device(fb.data_ptr(), s.cuda_stream)
    g = kat("kat_sampler_bdpt_caustic")
    r = g["rays"][0]
    Li, _ = it.render_sample(bdpt_amd.Ray(tuple(r[:3]), tuple(r[3:6]), float(r[6]), float(r[7])),
                             bdpt_amd.Sampler.from_state(g["state_in"][0]))
    s.synchronize()
    assert same_bits(Li, g["Li"][0])
    ref = load_golden(name).reshape(-1, 3).astype(np.float64)
    out = fb.cpu().numpy().reshape(-1, 3).astype(np.float64)
    err = np.linalg.norm(out - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-8)
    assert err.max() <= 1e-4 and m["samples"] == 64 * 64 * 16
