"""CPU-side checks of the product library (no GPU needed):
the C-ABI loads and exports every entry point of include/bdpt_amd.h, the host
scene ingest reproduces the reference's triangle order / BVH exactly, and the
camera constants are bit-identical to the reference's glm computations."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

import bdpt_amd
import variants

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(REPO, "include", "bdpt_amd.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(bdpt_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    L = bdpt_amd.lib()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    assert b"gfx950" in L.bdpt_version()


def test_library_is_gfx950_code_object():
    with open(bdpt_amd.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_no_device_is_an_error_not_a_fallback():
    if bdpt_amd.device_count() > 0:
        pytest.skip("a GPU is present")
    scene = bdpt_amd.Scene(variants.obj_path("cbox_low"))
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.BDPTIntegrator(scene, bdpt_amd.Config())


@pytest.mark.parametrize("scene_name", ["cbox_low", "caustic", "hardlight", "hardlight_mirror", "synth1m"])
def test_ingest_matches_reference(scene_name, golden_manifest):
    meta = golden_manifest["scenes"][scene_name]
    s = bdpt_amd.Scene(variants.obj_path(scene_name))
    info = s.info()
    assert info["triangles"] == meta["triangles"]
    assert info["bvh_nodes"] == meta["nodes"]
    assert info["shapes"] == meta["shapes"] and info["materials"] == meta["materials"]
    assert info["emitters"] == meta["emitters"]
    tf, ti, nf, nu = s.export()
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(tf) == meta["tri_f32_sha256"]
    assert sha(ti) == meta["tri_i32_sha256"]
    assert sha(nf) == meta["node_f32_sha256"]
    assert sha(nu) == meta["node_u32_sha256"]


@pytest.mark.parametrize("scene_name", ["cbox_low", "caustic"])
def test_camera_constants_match_reference(scene_name, golden_manifest):
    meta = golden_manifest["scenes"][scene_name]
    cam = bdpt_amd.Camera(**{k: v for k, v in variants.SCENES[scene_name]["camera"].items()})
    got = bdpt_amd.camera_constants(cam, meta["width"], meta["height"])
    ref = np.array([float.fromhex(x) for x in meta["camera_f32"]], np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_ingest_errors_are_reported(tmp_path):
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 0\n")
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.Scene(str(bad))
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.Scene(str(tmp_path / "missing.obj"))
    nonorm = tmp_path / "nonorm.obj"
    nonorm.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    with pytest.raises(bdpt_amd.BdptError, match="normal"):
        bdpt_amd.Scene(str(nonorm))


def test_ingest_triangulation_matches_oracle_on_polygons(tmp_path):
    """Ear clipping of convex / concave polygons, negative indices, 'g' groups
    and per-face materials: product ingest == oracle ingest (both restate
    tinyobj v1.2.0)."""
    import oracle as O
    (tmp_path / "m.mtl").write_text("newmtl a\nKd 0.5 0.5 0.5\nKe 1 1 1\nillum 7\nnewmtl b\nKd 0.2 0.3 0.4\nillum 8\n"
                                    "Ks 0.5 0.5 0.5\nNs 20\n")
    obj = ["mtllib m.mtl", "o star"]
    n = 9
    for i in range(n):
        r = 1.0 if i % 2 == 0 else 0.4
        a = 2 * np.pi * i / n
        obj.append(f"v {r*np.cos(a):.6f} {r*np.sin(a):.6f} 0.000000")
    obj += ["vn 0 0 1", "usemtl a", "f " + " ".join(f"{i+1}//1" for i in range(n))]
    obj += ["g second", "v 0 0 1", "v 1 0 1", "v 1 1 1", "v 0 1 1", "usemtl b", "f -4//1 -3//1 -2//1 -1//1",
            "usemtl a", "f -4//1 -2//1 -1//1"]
    p = tmp_path / "poly.obj"
    p.write_text("\n".join(obj) + "\n")
    a = bdpt_amd.Scene(str(p)).export()
    b = O.Scene(str(p)).dump()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("gen", ["many_shapes_obj", "closed_box_obj"])
def test_ingest_matches_oracle_on_generated_scenes(gen, tmp_path):
    """The generated test scenes of the GPU suite (7008 shapes; the closed box
    for deep rrDepth): product ingest == oracle ingest, and the shape count that
    moves the shape -> emitter map out of the LDS tables."""
    import oracle as O
    obj = getattr(variants, gen)(str(tmp_path))
    s = bdpt_amd.Scene(obj)
    for x, y in zip(s.export(), O.Scene(obj).dump()):
        assert np.array_equal(x, y)
    info = s.info()
    assert info["shapes"] == (7008 if gen == "many_shapes_obj" else 9)
    assert info["emitters"] == 1


def test_sampler_state_is_std_mt19937():
    """Sampler (math.h:63-76) state as libstdc++ streams it: the 10000th output of
    std::mt19937(5489) is 4123659995 (the C++ standard's check value), and the
    C-ABI's bdpt_sampler_state(seed, draws) equals the Python mirror advanced by draws."""
    import ctypes

    s = bdpt_amd.Sampler(5489)
    for _ in range(9999):
        s.next_u32()
    assert s.next_u32() == 4123659995
    for seed, draws in [(260450963, 0), (1, 2), (7, 227), (99, 624), (12345, 1000)]:
        py = bdpt_amd.Sampler(seed)
        for _ in range(draws):
            py.next_u32()
        st = np.zeros(bdpt_amd.MT19937_WORDS, np.uint32)
        assert bdpt_amd.lib().bdpt_sampler_state(seed, draws, ctypes.c_void_p(st.ctypes.data)) == 0
        assert np.array_equal(st, py.state), (seed, draws)


def test_ingest_matches_oracle_with_many_materials(tmp_path):
    """408 materials (every BSDF kind): product ingest == oracle ingest, and the
    BSDF types the scene's illum values map to (diffuse / mixture / mirror / glass)."""
    import oracle as O
    obj = variants.many_materials_obj(str(tmp_path))
    s = bdpt_amd.Scene(obj)
    for x, y in zip(s.export(), O.Scene(obj).dump()):
        assert np.array_equal(x, y)
    assert s.info()["materials"] == 408
    kinds = {s.bsdf_type(i)[1] for i in range(408)}
    assert kinds == {1, 2, 3, 4}


# ---- bdpt_scene_create: the scene handed over from the caller's in-memory Scene
def _layout(scene):
    return [scene.export_layout(i) for i in range(len(bdpt_amd.LAYOUT_ARRAYS))]


@pytest.mark.parametrize("scene_name", ["cbox_low", "caustic", "hardlight_mirror"])
def test_scene_desc_round_trip_is_bit_identical(scene_name):
    """A descriptor rebuilt from a loaded scene's exports (triangles back in
    (shape, face) order, the BVH's object order, materials / emitters from the
    device records) gives every device array bit for bit. The reference's own
    Scene is the source in tests/test_adapter_cpu.py."""
    s = bdpt_amd.Scene(variants.obj_path(scene_name))
    d = s.to_desc()
    t = bdpt_amd.Scene.from_desc(d)
    assert _layout(t) == _layout(s)
    assert t.info() == s.info()


def _bad(d, **change):
    import dataclasses
    return dataclasses.replace(d, **change)


def test_scene_desc_is_validated():
    s = bdpt_amd.Scene(variants.obj_path("cbox_low"))
    d = s.to_desc()
    n = d.tri_shape.size
    cases = {
        "not (shape, face) order": _bad(d, tri_shape=d.tri_shape[::-1].copy()),
        "primID not the face index": _bad(d, tri_prim=np.zeros(n, np.int32)),
        "material out of range": _bad(d, tri_mat=np.full(n, len(d.materials), np.int32)),
        "order not a permutation": _bad(d, bvh_order=np.zeros(n, np.int32)),
        "emitter CDF length": _bad(d, emitters=[dict(d.emitters[0], cdf=d.emitters[0]["cdf"][:-1])]),
        "repeated emitter shape": _bad(d, emitters=[d.emitters[0], d.emitters[0]]),
        "texture": _bad(d, materials=[dict(d.materials[0], has_texture=1)] + d.materials[1:]),
    }
    bvh = d.bvh.copy()
    root = bvh[0]["right_offset"]
    bvh[1]["bmax"] = bvh[0]["bmax"] + 1.0  # a child box outside its parent's box
    cases["child box outside parent"] = _bad(d, bvh=bvh)
    bvh = d.bvh.copy()
    bvh[0]["right_offset"] = len(bvh) + 5
    cases["rightOffset out of range"] = _bad(d, bvh=bvh)
    leaf = int(np.nonzero(d.bvh["right_offset"] == 0)[0][0])
    bvh = d.bvh.copy()
    bvh[leaf]["nprims"] = 0
    cases["empty leaf"] = _bad(d, bvh=bvh)
    assert root > 0
    for what, bad in cases.items():
        with pytest.raises(bdpt_amd.BdptError, match="descriptor|texture"):
            bdpt_amd.Scene.from_desc(bad)
            pytest.fail(what)


@pytest.mark.parametrize("scene_name", ["caustic", "hardlight", "synth1m"])
def test_graze_codes_cover_the_shading_normal_tilt(scene_name):
    """The near-cull exemption (cull_near_for) is about the
    origin triangle's geometric plane, tested at run time against the
    interpolated shading normal n_s with a per-triangle margin (the graze code,
    top byte of the uploaded shape word, bdpt_capi.cpp graze_code). Check on the
    uploaded records: flat triangles (corner normals along the plane normal) carry
    code 0, and for every triangle |n_s - sgn n_g| <= code / 64 at random
    barycentric points (float32 interpolation and normalization as shade_hit)."""
    s = bdpt_amd.Scene(variants.obj_path(scene_name))
    rec = np.frombuffer(s.export_layout("shade"), np.float32).reshape(-1, 8, 4)
    words = rec.view(np.uint32)
    code = (words[:, 1, 3] >> 24).astype(np.int64)
    shape = words[:, 1, 3] & 0xFFFFFF
    tf, ti, _, _ = s.export()
    assert np.array_equal(shape, ti[:, 0].astype(np.uint32))  # the shape id survives the packing
    n = rec[:, 0:3, 0:3].astype(np.float64)
    v0, v1, v2 = rec[:, 5, :3].astype(np.float64), rec[:, 3, :3].astype(np.float64), rec[:, 4, :3].astype(np.float64)
    g = np.cross(v1 - v0, v2 - v0)
    gl = np.linalg.norm(g, axis=1)
    ok = gl > 0
    g[ok] /= gl[ok, None]
    nn = n / np.maximum(np.linalg.norm(n, axis=2, keepdims=True), 1e-300)
    cos = np.einsum("tkc,tc->tk", nn, g)
    flat = ok & (np.abs(np.abs(cos) - 1.0) < 1e-12).all(1) & ((cos > 0).all(1) | (cos < 0).all(1))
    assert (code[flat] == 0).all()
    assert (code[~ok] == 255).all()
    rng = np.random.default_rng(3)
    u = rng.random((code.size, 8)).astype(np.float32)
    v = (rng.random((code.size, 8)) * (1 - u)).astype(np.float32)
    w = (np.float32(1) - u - v).astype(np.float32)
    nf = rec[:, 0:3, 0:3]
    sn = ((nf[:, None, 0] * w[..., None] + nf[:, None, 1] * u[..., None]) + nf[:, None, 2] * v[..., None])
    sn = (sn / np.linalg.norm(sn, axis=2, keepdims=True)).astype(np.float64)
    sgn = np.sign(cos[:, :1])
    tilt = np.linalg.norm(sn - sgn[:, :, None] * g[:, None, :], axis=2).max(1)
    sel = ok & (code < 255)
    assert (tilt[sel] <= code[sel] / 64.0 + 1e-6).all(), float((tilt[sel] - code[sel] / 64.0).max())
    if scene_name != "synth1m":
        assert (code > 0).any() and (code == 0).any()  # the sphere is smooth, the walls are flat
