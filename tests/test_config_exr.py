"""Scene configuration (loadTOML, src/main.cpp:22-116) and EXR output
(Integrator::save -> saveEXR, src/core/utils.h:95-156) of the product library,
against fixtures the unmodified reference produced (tests/golden/
make_config_goldens.py): the parsed Config must match field for field (floats
bit for bit, errors where the reference throws) and the EXR bytes must be
identical. CPU only; the end-to-end CLI run is in test_gpu_parity.py."""
import glob
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import bdpt_amd

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
CONFIGS = sorted(glob.glob(os.path.join(GOLD, "config", "*.toml")))
INTEGRATORS = {"normal": 0, "simple": 1, "ao": 2, "ro": 3, "direct": 4, "path": 5, "bdpt": 7}


def hexf(x: float) -> str:
    return float(np.float32(x)).hex().replace("0x1.0000000000000p", "0x1p").replace("0x0.0p+0", "0x0p+0")


def c_hex(x: float) -> str:
    """printf("%a", (double)float) as glibc prints it."""
    v = float(np.float32(x))
    if v != v:
        return "nan" if struct.pack(">f", np.float32(x))[0] < 0x80 else "-nan"
    if v in (float("inf"), float("-inf")):
        return "inf" if v > 0 else "-inf"
    if v == 0:
        return "-0x0p+0" if str(v).startswith("-") else "0x0p+0"
    m, e = v.hex().split("p")
    m = m.rstrip("0").rstrip(".")
    return f"{m}p{e}"


@pytest.fixture(scope="module")
def expected():
    with open(os.path.join(GOLD, "config", "expected.json")) as f:
        return json.load(f)


def test_config_fixtures_cover_reference_scene_files(expected):
    assert len(CONFIGS) == len(expected) >= 12
    assert {"ref_cbox_bdpt_glass.toml", "ref_bonus_cbox_bdpt.toml"} <= set(expected)


@pytest.mark.parametrize("path", CONFIGS, ids=[os.path.basename(p) for p in CONFIGS])
def test_load_toml_matches_reference(path, expected):
    ref = expected[os.path.basename(path)]
    if ref["error"]:
        with pytest.raises(bdpt_amd.BdptError):
            bdpt_amd.load_toml(path)
        return
    sc = bdpt_amd.load_toml(path)
    c = sc.config
    assert sc.obj_file_raw.encode().hex() == ref["objfile_hex"]
    assert c_hex(c.camera.fov) == ref["fov"]
    for k, name in (("eye", "eye"), ("at", "at"), ("up", "up")):
        assert [c_hex(v) for v in getattr(c.camera, name)] == ref[k], k
    assert (c.width, c.height) == (ref["width"], ref["height"])
    assert int(sc.realtime) == ref["realtime"]
    if not ref["realtime"]:
        assert INTEGRATORS[sc.integrator] == ref["integrator"]
        if sc.integrator == "path":
            assert (sc.path.rr_depth, c_hex(sc.path.rr_prob)) == (ref["rrDepth"], ref["rrProb"])
            for k in ("isExplicit", "maxDepth", "emitterSamples", "bsdfSamples"):
                if k in ref:
                    got = {"isExplicit": int(sc.path.explicit), "maxDepth": sc.path.max_depth,
                           "emitterSamples": sc.path.emitter_samples, "bsdfSamples": sc.path.bsdf_samples}[k]
                    assert got == ref[k], k
        if sc.integrator == "direct":  # main.cpp:88-92
            d = sc.direct
            assert (d.emitter_samples, d.bsdf_samples, d.sampling_strategy) == (
                ref["emitterSamples"], ref["bsdfSamples"], ref["samplingStrategy"])
            assert d.c().sampling_strategy == bdpt_amd.DIRECT_STRATEGIES.get(ref["samplingStrategy"], 0)
        assert c.spp == ref["spp"]
        if "rrDepth" in ref:
            assert c.rr_depth == ref["rrDepth"]
            assert c_hex(c.rr_prob) == ref["rrProb"]


def test_objfile_resolves_against_toml_directory(tmp_path):
    p = tmp_path / "sub" / "scene.toml"
    p.parent.mkdir()
    p.write_text('[input]\nobjfile = "../mesh/x.obj"\n[camera]\n[film]\n[renderer]\ntype = "bdpt"\n')
    sc = bdpt_amd.load_toml(str(p))
    assert sc.obj_file == str(tmp_path / "sub" / "../mesh/x.obj")
    p.write_text('[input]\nobjfile = "/abs/x.obj"\n[camera]\n[film]\n[renderer]\ntype = "bdpt"\n')
    assert bdpt_amd.load_toml(str(p)).obj_file == "/abs/x.obj"


@pytest.mark.parametrize("text", [
    "[camera]\n[film]\n[renderer]\n",                                    # no [input] objfile
    '[input]\nobjfile = "a"\n[film]\n[renderer]\n',                      # no [camera]
    '[input]\nobjfile = "a"\nobjfile = "b"\n[camera]\n[film]\n[renderer]\n',  # duplicate key
    '[input]\nobjfile = "a\n[camera]\n[film]\n[renderer]\n',             # unterminated string
    '[input]\nobjfile = "a"\n[camera]\neye = [1.0, 2.0\n[film]\n[renderer]\n',  # unterminated array
    '[input]\nobjfile = "a"\n[camera]\n[film]\nwidth = 99999999999\n[renderer]\n',  # int overflow
])
def test_malformed_toml_is_an_error(tmp_path, text):
    p = tmp_path / "bad.toml"
    p.write_text(text)
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.load_toml(str(p))


def test_missing_toml_is_an_error(tmp_path):
    with pytest.raises(bdpt_amd.BdptError, match="cannot open"):
        bdpt_amd.load_toml(str(tmp_path / "nope.toml"))


@pytest.fixture(scope="module")
def exr_gold():
    return np.load(os.path.join(GOLD, "exr_goldens.npz"))


def test_exr_bytes_match_reference_on_g1_framebuffer(exr_gold):
    fb = np.load(os.path.join(GOLD, "G1_cbox_low_64x64_spp4.npz"))["fb"]
    assert bdpt_amd.encode_exr(fb, 64, 64) == exr_gold["e1_bytes"].tobytes()


def test_exr_bytes_match_reference_on_special_values(exr_gold):
    W, H = (int(v) for v in exr_gold["e2_shape"])
    assert bdpt_amd.encode_exr(exr_gold["e2_input"], W, H) == exr_gold["e2_bytes"].tobytes()


def decode_exr(blob: bytes):
    """Minimal reader for the uncompressed B/G/R half scanline files saveEXR writes."""
    assert blob[:4] == bytes([0x76, 0x2F, 0x31, 0x01])
    p, attrs = 8, {}
    while blob[p] != 0:
        e = blob.index(b"\0", p)
        name = blob[p:e].decode()
        t = blob.index(b"\0", e + 1)
        size = struct.unpack_from("<I", blob, t + 1)[0]
        attrs[name] = blob[t + 5:t + 5 + size]
        p = t + 5 + size
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    p += 1
    offsets = struct.unpack_from(f"<{H}Q", blob, p)
    img = np.zeros((H, W, 3), np.float16)
    for y, off in enumerate(offsets):
        line, n = struct.unpack_from("<iI", blob, off)
        assert line == y and n == W * 6
        planes = np.frombuffer(blob, np.float16, 3 * W, off + 8).reshape(3, W)
        img[y] = planes[::-1].T  # B, G, R -> RGB
    return img


def test_exr_roundtrip_is_half_of_the_framebuffer(tmp_path):
    rng = np.random.default_rng(1)
    fb = (rng.random((9, 13, 3)) * 40).astype(np.float32)
    path = str(tmp_path / "out.exr")
    bdpt_amd.save_exr(fb, 13, 9, path)
    img = decode_exr(open(path, "rb").read())
    # tinyexr rounds half-up on the first dropped bit: within 1 half ulp of the float
    ref = fb.astype(np.float16).astype(np.float32)
    assert np.allclose(img.astype(np.float32), ref, rtol=2 ** -10, atol=0)


def test_exr_rejects_bad_arguments(tmp_path):
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.encode_exr(np.zeros(5, np.float32), 2, 1)
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.save_exr(np.zeros(6, np.float32), 2, 1, str(tmp_path / "no" / "dir" / "x.exr"))


def test_cli_without_gpu_rejects_non_bdpt_scenes(tmp_path):
    """The CLI parses the TOML before touching the GPU: other integrators and
    realtime passes are refused with the reference's error style."""
    cli = os.path.join(os.path.dirname(bdpt_amd.LIB_PATH), "tinyrender_amd")
    assert os.path.exists(cli)
    r = subprocess.run([cli, os.path.join(GOLD, "config", "t04_realtime.toml")], capture_output=True, text=True)
    assert r.returncode != 0 and "realtime render passes are not part" in r.stderr
    r = subprocess.run([cli, os.path.join(GOLD, "config", "t05_bad_type.toml")], capture_output=True, text=True)
    assert r.returncode != 0 and "Error while parsing scene file" in r.stderr
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode != 0 and "Syntax" in r.stderr
