"""The C oracle (oracle/src) against the reference's own outputs.

The fixtures in tests/golden/ were rendered by the unmodified reference
(oracle/_ref/ref_bdpt, see tests/golden/make_goldens.py). A single-threaded
oracle render splats in the same order as the single-threaded reference, so the
framebuffers must be BIT-IDENTICAL. This is what pins the oracle.
"""
import hashlib

import numpy as np
import pytest

import oracle as O
import variants
from conftest import load_golden

FB_CASES = ["G1_cbox_low_64x64_spp4", "G2_caustic_64x64_spp16", "G3_hardlight_64x64_spp16",
            "G4_hardlight_mirror_64x64_spp16", "G5_caustic_80x48_spp1", "G6_caustic_512x512_spp4_rows16",
            "G7_hardlight_512x512_spp4_rows32", "G8_synth1m_48x32_spp2",
            # the reference's LIGHT_TRACING / PATH_TRACING builds (bdpt.h:16-17)
            "G9_caustic_lt_64x64_spp16", "G10_caustic_pt_64x64_spp16", "G11_hardlight_lt_64x64_spp16",
            "G12_hardlight_pt_64x64_spp16"]
STRATEGY = {"bdpt": 0, "lt": 1, "pt": 2}


@pytest.mark.parametrize("name", FB_CASES)
def test_oracle_framebuffer_bit_exact(name, golden_manifest):
    meta = golden_manifest["framebuffers"][name]
    sc = variants.SCENES[meta["scene"]]
    scene = O.Scene(variants.obj_path(meta["scene"]))
    p = O.make_params(sc["camera"], meta["width"], meta["height"], meta["spp"], meta["rr_depth"],
                      STRATEGY[meta.get("strategy", "bdpt")])
    rows = list(range(0, meta["height"], meta["row_stride"]))
    fb, n = scene.render(p, rows=rows)
    assert n == meta["samples"]
    ref = load_golden(name)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == meta["sha256"]
    mism = np.flatnonzero(fb.view(np.uint32) != ref.view(np.uint32))
    assert mism.size == 0, f"{mism.size} floats differ, first at {mism[:5]}"


RR_CASES = ["R1_caustic_rr_64x64_spp16", "R2_hardlight_rr_64x64_spp16", "R3_cbox_low_rr_64x64_spp4",
            "R4_caustic_rr1_48x48_spp4", "R5_hardlight_mirror_rr_48x48_spp4", "R6_caustic_rr_512x512_spp2_rows32"]


@pytest.mark.parametrize("name", RR_CASES)
def test_oracle_russian_roulette_bit_exact(name, golden_manifest):
    """NO_RR = 0 (bdpt.h:18): the reference built with its Russian-roulette
    branch (oracle/_ref/ref_bdpt_rr) against the oracle's russian_roulette = 1."""
    meta = golden_manifest["rr_framebuffers"][name]
    sc = variants.SCENES[meta["scene"]]
    scene = O.Scene(variants.obj_path(meta["scene"]))
    p = O.make_params(sc["camera"], meta["width"], meta["height"], meta["spp"], meta["rr_depth"], 0,
                      russian_roulette=1)
    rows = list(range(0, meta["height"], meta["row_stride"]))
    O.lib().tro_rr_overflow(1)
    fb, n = scene.render(p, rows=rows)
    assert n == meta["samples"] and O.lib().tro_rr_overflow(1) == 0
    ref = load_golden(name)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == meta["sha256"]
    mism = np.flatnonzero(fb.view(np.uint32) != ref.view(np.uint32))
    assert mism.size == 0, f"{mism.size} floats differ, first at {mism[:5]}"
    # the mode matters: NO_RR = 1 gives a different image on every scene
    p.russian_roulette = 0
    fb0, _ = scene.render(p, rows=rows)
    assert not np.array_equal(fb0, ref)


@pytest.mark.parametrize("scene_name", ["cbox_low", "caustic", "hardlight", "hardlight_mirror", "synth1m"])
def test_oracle_scene_ingest_matches_reference(scene_name, golden_manifest):
    meta = golden_manifest["scenes"][scene_name]
    scene = O.Scene(variants.obj_path(scene_name))
    st = scene.stats()
    assert st["triangles"] == meta["triangles"] and st["nodes"] == meta["nodes"]
    assert st["shapes"] == meta["shapes"] and st["materials"] == meta["materials"]
    assert st["emitters"] == meta["emitters"]
    tf, ti, nf, nu = scene.dump()
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(tf) == meta["tri_f32_sha256"]
    assert sha(ti) == meta["tri_i32_sha256"]
    assert sha(nf) == meta["node_f32_sha256"]
    assert sha(nu) == meta["node_u32_sha256"]


@pytest.mark.parametrize("scene_name", ["cbox_low", "caustic"])
def test_oracle_camera_matches_reference(scene_name, golden_manifest):
    meta = golden_manifest["scenes"][scene_name]
    sc = variants.SCENES[scene_name]
    p = O.make_params(sc["camera"], meta["width"], meta["height"], 1, sc["rr_depth"])
    cam = O.camera(p)
    ref = np.array([float.fromhex(x) for x in meta["camera_f32"]], np.float32)
    assert np.array_equal(cam.view(np.uint32), ref.view(np.uint32))


def test_mt19937_matches_numpy_legacy_seeding():
    # numpy's RandomState(int) uses the same init_genrand as std::mt19937(seed).
    for seed in (0, 1, 260450963, 260450963 + 4095, 2**32 - 1):
        rs = np.random.RandomState(seed)
        raw = rs.randint(0, 2**32, size=700, dtype=np.uint32)
        got = [O.lib().tro_mt19937_nth(seed, i) for i in (0, 1, 226, 227, 623, 624, 699)]
        assert got == [int(raw[i]) for i in (0, 1, 226, 227, 623, 624, 699)]


def test_sampler_float_conversion():
    # generate_canonical<float,24>: float(u)/2^32 clamped below 1.
    for seed in (7, 260450963):
        rs = np.random.RandomState(seed)
        raw = rs.randint(0, 2**32, size=50, dtype=np.uint32)
        exp = np.minimum(raw.astype(np.float32) / np.float32(2**32), np.float32(np.nextafter(np.float32(1), np.float32(0))))
        got = np.array([O.lib().tro_sampler_nth(seed, i) for i in range(50)], np.float32)
        assert np.array_equal(got, exp)


def test_glibc_mathf_restatement_matches_host_libm():
    # tr_sinf/tr_cosf/tr_powf restate glibc 2.35's FMA multiarch variants; on an
    # FMA+AVX2 host libm selects exactly those, so results must be bit-equal.
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for fn in ("sinf", "cosf"):
        getattr(libm, fn).restype = ctypes.c_float
        getattr(libm, fn).argtypes = [ctypes.c_float]
    libm.powf.restype = ctypes.c_float
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    with open("/proc/cpuinfo") as f:
        flags = f.read()
    if " fma " not in flags or " avx2 " not in flags:
        pytest.skip("host libm selects the non-FMA variant")
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 2 * np.pi, 20000), rng.uniform(-np.pi, np.pi, 20000)]).astype(np.float32)
    L = O.lib()
    for x in xs[:20000:7]:
        x = float(x)
        assert np.float32(L.tro_sinf(x)).view(np.uint32) == np.float32(libm.sinf(x)).view(np.uint32)
        assert np.float32(L.tro_cosf(x)).view(np.uint32) == np.float32(libm.cosf(x)).view(np.uint32)
    us = rng.uniform(0, 1, 5000).astype(np.float32)
    for y in (1 / np.float32(11.803922), np.float32(9.803922), np.float32(29.411765), np.float32(100.0)):
        for u in us[::5]:
            assert np.float32(L.tro_powf(float(u), float(y))).view(np.uint32) == \
                np.float32(libm.powf(float(u), float(y))).view(np.uint32)


PATH_CASES = ["P1_hardlight_path_64x64_spp4", "P2_caustic_path_64x64_spp4", "P3_caustic_path_mis_48x48_spp4",
              "P4_cbox_low_path_implicit_64x64_spp4", "P5_hardlight_path_maxdepth3_48x48_spp4"]


@pytest.mark.parametrize("name", PATH_CASES)
def test_oracle_path_tracer_bit_exact(name, golden_manifest):
    """PathTracerIntegrator (path.h) frames rendered by the reference."""
    meta = golden_manifest["path_framebuffers"][name]
    sc = variants.SCENES[meta["scene"]]
    p = O.make_path_params(sc["camera"], meta["width"], meta["height"], meta["spp"], **meta["path"])
    fb, n = O.Scene(variants.obj_path(meta["scene"])).render(p)
    assert n == meta["samples"]
    ref = load_golden(name)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == meta["sha256"]
    mism = np.flatnonzero(fb.view(np.uint32) != ref.view(np.uint32))
    assert mism.size == 0, f"{mism.size} floats differ, first at {mism[:5]}"


DIRECT_CASES = ["D1_caustic_direct_area_48x48_spp4", "D2_hardlight_direct_solidangle_48x48_spp4",
                "D3_caustic_direct_cosine_48x48_spp4", "D4_hardlight_direct_bsdf_48x48_spp4",
                "D5_caustic_direct_mis_48x48_spp4", "D6_hardlight_direct_mis_48x48_spp4"]


@pytest.mark.parametrize("name", DIRECT_CASES)
def test_oracle_direct_integrator_bit_exact(name, golden_manifest):
    """DirectIntegrator (direct.h), every sampling strategy, frames rendered by the reference."""
    meta = golden_manifest["direct_framebuffers"][name]
    sc = variants.SCENES[meta["scene"]]
    p = O.make_direct_params(sc["camera"], meta["width"], meta["height"], meta["spp"], **meta["direct"])
    fb, n = O.Scene(variants.obj_path(meta["scene"])).render(p)
    assert n == meta["samples"]
    ref = load_golden(name)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == meta["sha256"]
    mism = np.flatnonzero(fb.view(np.uint32) != ref.view(np.uint32))
    assert mism.size == 0, f"{mism.size} floats differ, first at {mism[:5]}"
