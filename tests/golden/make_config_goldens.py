"""Generates the scene-configuration and EXR fixtures from the UNMODIFIED reference.

Run in the development container (needs /root/reference):
    make -C oracle/ref            # oracle/_ref/ref_bdpt (reference sources + driver)
    python tests/golden/make_config_goldens.py

* config/expected.json: for every config/*.toml, the Config the reference's
  loadTOML (src/main.cpp:22-116, cpptoml) builds — `ref_bdpt toml FILE` — or
  {"error": true} when it throws. Floats as C99 hex strings, objfile as hex bytes.
  The ref_*.toml files are the reference's own scene files (data/a5/...); the
  t*.toml files are edge cases (int/float typing, defaults, escapes, rounding).
* exr_goldens.npz: the bytes the reference's saveEXR (src/core/utils.h:95-156,
  tinyexr) writes — `ref_bdpt exr` — for (e1) the G1 golden framebuffer and
  (e2) a 37x5 buffer of special values (zeros, denormals, half-rounding edges,
  overflow, inf, NaN, negatives) plus random floats over many exponents.
"""
from __future__ import annotations

import glob
import json
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "ref_bdpt")


def special_buffer() -> np.ndarray:
    W, H = 37, 5
    rng = np.random.default_rng(446)
    n = W * H * 3
    bits = [0x00000000, 0x80000000, 0x00000001, 0x007fffff, 0x00800000, 0x33000000, 0x33000001, 0x337fffff,
            0x33800000, 0x38800000, 0x387fffff, 0x387fe000, 0x387ff000, 0x38801000, 0x38800fff, 0x3f800000,
            0x3f801000, 0x3f800fff, 0x3f802000, 0x3f803000, 0x477fe000, 0x477fefff, 0x477ff000, 0x477fffff,
            0x47800000, 0x7f7fffff, 0x7f800000, 0xff800000, 0x7fc00000, 0x7f800001, 0xffc00001, 0xbf800000,
            0xc77ff000, 0xb3800000, 0x80000001, 0x3eaaaaab, 0x3dcccccd]
    special = np.array(bits, dtype=np.uint32).view(np.float32)
    rand = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 20, n))).astype(np.float32)
    buf = rand.copy()
    buf[:len(special)] = special
    buf[len(special):2 * len(special)] = -special
    return buf


def ref_exr(fb: np.ndarray, W: int, H: int) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "fb.f32"), os.path.join(d, "out.exr")
        fb.astype(np.float32).tofile(src)
        subprocess.run([REF, "exr", src, str(W), str(H), dst], check=True, capture_output=True)
        with open(dst, "rb") as f:
            return f.read()


def main() -> None:
    if not os.path.exists(REF):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle", "ref")], check=True)
    expected = {}
    for path in sorted(glob.glob(os.path.join(HERE, "config", "*.toml"))):
        out = subprocess.run([REF, "toml", path], check=True, capture_output=True, text=True).stdout
        expected[os.path.basename(path)] = json.loads(out.strip().splitlines()[-1])
    with open(os.path.join(HERE, "config", "expected.json"), "w") as f:
        json.dump(expected, f, indent=1, sort_keys=True)
        f.write("\n")
    g1 = np.load(os.path.join(HERE, "G1_cbox_low_64x64_spp4.npz"))["fb"]
    e2 = special_buffer()
    np.savez_compressed(os.path.join(HERE, "exr_goldens.npz"),
                        e1_bytes=np.frombuffer(ref_exr(g1, 64, 64), dtype=np.uint8),
                        e2_input=e2, e2_shape=np.array([37, 5]),
                        e2_bytes=np.frombuffer(ref_exr(e2, 37, 5), dtype=np.uint8))
    print(f"{len(expected)} configs, 2 EXR fixtures")


if __name__ == "__main__":
    main()
