"""Generates the golden fixtures in tests/golden/ from the UNMODIFIED reference.

Run in the development container (needs /root/reference):
    make -C oracle/ref            # builds oracle/_ref/ref_bdpt from the reference sources
    python tests/golden/make_goldens.py

Every framebuffer fixture is the output of oracle/_ref/ref_bdpt (reference
BDPTIntegrator::render + the per-(pixel, sample)-seeded driver of
oracle/ref/ref_driver.cpp), single-threaded so splats land in the reference's
own order. Scene fixtures are sha256 digests of the reference's triangle list
(BVH leaf order), flat BVH nodes and camera matrices (ref_bdpt dump).
"""
from __future__ import annotations

import hashlib
import json
import os
import platform
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "scenes"))
import variants  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "ref_bdpt")
# the reference built with its compile-time strategy switch (bdpt.h:16-17) flipped (oracle/ref/Makefile)
REF_STRATEGY = {"bdpt": REF, "lt": REF + "_lt", "pt": REF + "_pt"}
# the reference built with NO_RR = 0 (bdpt.h:18 flipped, oracle/ref/Makefile): Russian roulette past rrDepth
REF_RR = REF + "_rr"

# name: (scene, W, H, spp, rrDepth, row_stride[, strategy: bdpt | lt (LIGHT_TRACING) | pt (PATH_TRACING)])
FRAMEBUFFERS = {
    "G1_cbox_low_64x64_spp4": ("cbox_low", 64, 64, 4, 5, 1),
    "G2_caustic_64x64_spp16": ("caustic", 64, 64, 16, 8, 1),
    "G3_hardlight_64x64_spp16": ("hardlight", 64, 64, 16, 2, 1),
    "G4_hardlight_mirror_64x64_spp16": ("hardlight_mirror", 64, 64, 16, 5, 1),
    "G5_caustic_80x48_spp1": ("caustic", 80, 48, 1, 8, 1),
    # bench resolution: every 16th row of 512x512 at 4 spp (splats land everywhere)
    "G6_caustic_512x512_spp4_rows16": ("caustic", 512, 512, 4, 8, 16),
    "G7_hardlight_512x512_spp4_rows32": ("hardlight", 512, 512, 4, 2, 32),
    # synthetic 1M-triangle box (scenes/synth.py), BASELINE configs[4] at a small size
    "G8_synth1m_48x32_spp2": ("synth1m", 48, 32, 2, 8, 1),
    # the reference's single-strategy builds (LIGHT_TRACING / PATH_TRACING = 1, bdpt.h:16-17)
    "G9_caustic_lt_64x64_spp16": ("caustic", 64, 64, 16, 8, 1, "lt"),
    "G10_caustic_pt_64x64_spp16": ("caustic", 64, 64, 16, 8, 1, "pt"),
    "G11_hardlight_lt_64x64_spp16": ("hardlight", 64, 64, 16, 2, 1, "lt"),
    "G12_hardlight_pt_64x64_spp16": ("hardlight", 64, 64, 16, 2, 1, "pt"),
}

# The reference's Russian-roulette branch (NO_RR = 0): name: (scene, W, H, spp, rrDepth, row_stride)
RR_FRAMEBUFFERS = {
    "R1_caustic_rr_64x64_spp16": ("caustic", 64, 64, 16, 8, 1),
    "R2_hardlight_rr_64x64_spp16": ("hardlight", 64, 64, 16, 2, 1),
    "R3_cbox_low_rr_64x64_spp4": ("cbox_low", 64, 64, 4, 5, 1),
    # roulette from the first bounce on (rrDepth 1: every loop test draws)
    "R4_caustic_rr1_48x48_spp4": ("caustic", 48, 48, 4, 1, 1),
    "R5_hardlight_mirror_rr_48x48_spp4": ("hardlight_mirror", 48, 48, 4, 3, 1),
    "R6_caustic_rr_512x512_spp2_rows32": ("caustic", 512, 512, 2, 8, 32),
}

# PathTracerIntegrator (src/integrators/path.h) frames: name: (scene, W, H, spp, path settings)
PATH_FRAMEBUFFERS = {
    # the settings of the reference's data/a5/bonus_bdpt/tinyrender/cbox_bdpt_path.toml
    "P1_hardlight_path_64x64_spp4": ("hardlight", 64, 64, 4, {}),
    "P2_caustic_path_64x64_spp4": ("caustic", 64, 64, 4, {}),
    # multiple importance sampling of the direct light (emitter + BSDF samples)
    "P3_caustic_path_mis_48x48_spp4": ("caustic", 48, 48, 4, dict(emitter_samples=2, bsdf_samples=2)),
    "P4_cbox_low_path_implicit_64x64_spp4": ("cbox_low", 64, 64, 4, dict(explicit=False, max_depth=5)),
    "P5_hardlight_path_maxdepth3_48x48_spp4": ("hardlight", 48, 48, 4, dict(max_depth=3, bsdf_samples=1)),
}

# DirectIntegrator (src/integrators/direct.h) frames: name: (scene, W, H, spp, direct settings). Its
# emitters are treated as spheres (shape center, AABB half-width, renderer.cpp:349-358).
DIRECT_FRAMEBUFFERS = {
    "D1_caustic_direct_area_48x48_spp4": ("caustic", 48, 48, 4, dict(strategy="area", emitter_samples=2)),
    "D2_hardlight_direct_solidangle_48x48_spp4": ("hardlight", 48, 48, 4, dict(strategy="solidAngle",
                                                                                emitter_samples=2)),
    "D3_caustic_direct_cosine_48x48_spp4": ("caustic", 48, 48, 4, dict(strategy="cosineHemisphere",
                                                                        emitter_samples=3)),
    "D4_hardlight_direct_bsdf_48x48_spp4": ("hardlight", 48, 48, 4, dict(strategy="bsdf", bsdf_samples=3)),
    "D5_caustic_direct_mis_48x48_spp4": ("caustic", 48, 48, 4, dict(strategy="mis", emitter_samples=2,
                                                                     bsdf_samples=2)),
    "D6_hardlight_direct_mis_48x48_spp4": ("hardlight", 48, 48, 4, dict(strategy="mis", emitter_samples=1,
                                                                         bsdf_samples=1)),
}

# BASELINE configs[1] / [3] / [4] at their full size: the reference renders a few-row
# shard (8 threads); the fixture keeps the shard's own rows (eye estimates plus the
# splats that land on them) and block sums of the whole frame (every splat).
# name: (scene, W, H, spp, rrDepth, row_offset, row_stride, block)
LARGE_FRAMEBUFFERS = {
    # the bench workload (BASELINE configs[1], the metric's frame) at its own spp: eight rows
    "L0_caustic_512x512_spp256_rows8": ("caustic", 512, 512, 256, 8, 31, 64, 32),
    "L1_caustic_1024x1024_spp1024_rows2": ("caustic", 1024, 1024, 1024, 8, 300, 512, 32),
    "L2_synth1m_2048x2048_spp512_rows2": ("synth1m", 2048, 2048, 512, 8, 700, 1024, 64),
    # configs[2] at its own spp (HardLight, rrDepth 2: the short-subpath build)
    "L3_hardlight_512x512_spp1024_rows8": ("hardlight", 512, 512, 1024, 2, 17, 64, 32),
    # the bench workload with Russian roulette (the reference's NO_RR = 0 build, ref_bdpt_rr)
    "L4_caustic_rr_512x512_spp256_rows8": ("caustic", 512, 512, 256, 8, 45, 64, 32, 1),
}

SCENE_DUMPS = {"cbox_low": (64, 64), "caustic": (512, 512), "hardlight": (512, 512), "hardlight_mirror": (512, 512),
               "synth1m": (64, 64)}


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main() -> None:
    """python make_goldens.py [NAME ...]: regenerate everything, or only the named
    framebuffer / scene entries (merged into the existing manifest)."""
    only = set(sys.argv[1:])
    if not os.path.exists(REF):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle", "ref")], check=True)
    old = {}
    if only and os.path.exists(os.path.join(HERE, "manifest.json")):
        with open(os.path.join(HERE, "manifest.json")) as f:
            old = json.load(f)
    manifest = {
        "generator": "oracle/_ref/ref_bdpt (reference sources @ /root/reference, oracle/ref/Makefile)",
        "compiler": subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
        "glibc": platform.libc_ver()[1],
        "seed_convention": "Sampler((int)(260450963u + pixel*spp + k)); jitter next2D first when spp > 1",
        "framebuffers": dict(old.get("framebuffers", {})),
        "scenes": dict(old.get("scenes", {})),
    }
    for sect in ("rr_framebuffers", "path_framebuffers", "direct_framebuffers", "large_framebuffers"):
        if sect in old:
            manifest[sect] = dict(old[sect])
    tmp = tempfile.mkdtemp()
    for name, entry in FRAMEBUFFERS.items():
        if only and name not in only:
            continue
        scene, W, H, spp, rr, stride = entry[:6]
        strategy = entry[6] if len(entry) > 6 else "bdpt"
        toml = os.path.join(tmp, name + ".toml")
        with open(toml, "w") as f:
            f.write(variants.toml_text(scene, W, H, spp, rr))
        out = os.path.join(tmp, name + ".f32")
        cmd = [REF_STRATEGY[strategy], "render", toml, str(W), str(H), str(spp), "--rr", str(rr), "--out", out]
        if stride > 1:
            cmd += ["--row-stride", str(stride)]
        r = subprocess.run(cmd, capture_output=True, text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        fb = np.fromfile(out, np.float32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), fb=fb)
        manifest["framebuffers"][name] = dict(scene=scene, width=W, height=H, spp=spp, rr_depth=rr, row_stride=stride,
                                              strategy=strategy,
                                              samples=info["samples"], sha256=sha(fb.tobytes()),
                                              mean_rgb=[float(x) for x in fb.reshape(-1, 3).mean(0)],
                                              ref_seconds=info["seconds"])
        print(name, manifest["framebuffers"][name]["sha256"][:16], info)
    for name, (scene, W, H, spp, rr, stride) in RR_FRAMEBUFFERS.items():
        if only and name not in only:
            continue
        toml = os.path.join(tmp, name + ".toml")
        with open(toml, "w") as f:
            f.write(variants.toml_text(scene, W, H, spp, rr))
        out = os.path.join(tmp, name + ".f32")
        cmd = [REF_RR, "render", toml, str(W), str(H), str(spp), "--rr", str(rr), "--out", out]
        if stride > 1:
            cmd += ["--row-stride", str(stride)]
        r = subprocess.run(cmd, capture_output=True, text=True, check=True, timeout=3600)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        fb = np.fromfile(out, np.float32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), fb=fb)
        manifest.setdefault("rr_framebuffers", dict(old.get("rr_framebuffers", {})))
        manifest["rr_framebuffers"][name] = dict(scene=scene, width=W, height=H, spp=spp, rr_depth=rr,
                                                 row_stride=stride, russian_roulette=1, samples=info["samples"],
                                                 sha256=sha(fb.tobytes()),
                                                 mean_rgb=[float(x) for x in fb.reshape(-1, 3).mean(0)],
                                                 ref_seconds=info["seconds"])
        print(name, manifest["rr_framebuffers"][name]["sha256"][:16], info)
    for name, (scene, W, H, spp, path) in PATH_FRAMEBUFFERS.items():
        if only and name not in only:
            continue
        toml = os.path.join(tmp, name + ".toml")
        with open(toml, "w") as f:
            f.write(variants.path_toml_text(scene, W, H, spp, **path))
        out = os.path.join(tmp, name + ".f32")
        r = subprocess.run([REF, "render", toml, str(W), str(H), str(spp), "--out", out], capture_output=True,
                           text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        fb = np.fromfile(out, np.float32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), fb=fb)
        manifest.setdefault("path_framebuffers", dict(old.get("path_framebuffers", {})))
        manifest["path_framebuffers"][name] = dict(scene=scene, width=W, height=H, spp=spp, path=path,
                                                   samples=info["samples"], sha256=sha(fb.tobytes()),
                                                   mean_rgb=[float(x) for x in fb.reshape(-1, 3).mean(0)],
                                                   ref_seconds=info["seconds"])
        print(name, manifest["path_framebuffers"][name]["sha256"][:16], info)
    for name, (scene, W, H, spp, direct) in DIRECT_FRAMEBUFFERS.items():
        if only and name not in only:
            continue
        toml = os.path.join(tmp, name + ".toml")
        with open(toml, "w") as f:
            f.write(variants.direct_toml_text(scene, W, H, spp, **direct))
        out = os.path.join(tmp, name + ".f32")
        r = subprocess.run([REF, "render", toml, str(W), str(H), str(spp), "--out", out], capture_output=True,
                           text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        fb = np.fromfile(out, np.float32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), fb=fb)
        manifest.setdefault("direct_framebuffers", dict(old.get("direct_framebuffers", {})))
        manifest["direct_framebuffers"][name] = dict(scene=scene, width=W, height=H, spp=spp, direct=direct,
                                                     samples=info["samples"], sha256=sha(fb.tobytes()),
                                                     mean_rgb=[float(x) for x in fb.reshape(-1, 3).mean(0)],
                                                     ref_seconds=info["seconds"])
        print(name, manifest["direct_framebuffers"][name]["sha256"][:16], info)
    for name, entry in LARGE_FRAMEBUFFERS.items():
        if only and name not in only:
            continue
        scene, W, H, spp, rr, off, stride, blk = entry[:8]
        russian_roulette = entry[8] if len(entry) > 8 else 0
        toml = os.path.join(tmp, name + ".toml")
        with open(toml, "w") as f:
            f.write(variants.toml_text(scene, W, H, spp, rr))
        out = os.path.join(tmp, name + ".f32")
        r = subprocess.run([REF_RR if russian_roulette else REF, "render", toml, str(W), str(H), str(spp), "--rr", str(rr), "--out", out,
                            "--row-offset", str(off), "--row-stride", str(stride), "--threads", "8"],
                           capture_output=True, text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        fb = np.fromfile(out, np.float32).reshape(H, W, 3)
        rows = list(range(off, H, stride))
        blocks = fb.astype(np.float64).reshape(H // blk, blk, W // blk, blk, 3).sum(axis=(1, 3))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rows=np.array(rows, np.int32), fb_rows=fb[rows],
                            blocks=blocks)
        manifest.setdefault("large_framebuffers", dict(old.get("large_framebuffers", {})))
        manifest["large_framebuffers"][name] = dict(scene=scene, width=W, height=H, spp=spp, rr_depth=rr,
                                                    row_offset=off, row_stride=stride, block=blk,
                                                    russian_roulette=russian_roulette,
                                                    samples=info["samples"], threads=8,
                                                    sha256_rows=sha(fb[rows].tobytes()),
                                                    frame_sum=[float(x) for x in blocks.sum((0, 1))],
                                                    ref_seconds=info["seconds"])
        print(name, info)
    for scene, (W, H) in SCENE_DUMPS.items():
        if only and scene not in only:
            continue
        toml = os.path.join(tmp, scene + "_dump.toml")
        with open(toml, "w") as f:
            f.write(variants.toml_text(scene, W, H, 1))
        d = os.path.join(tmp, scene + "_dump")
        os.makedirs(d, exist_ok=True)
        r = subprocess.run([REF, "dump", toml, str(W), str(H), d], capture_output=True, text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        ent = dict(info)
        ent["width"], ent["height"] = W, H
        for fn in ("tri_f32", "tri_i32", "node_f32", "node_u32", "camera_f32"):
            with open(os.path.join(d, fn + ".bin"), "rb") as f:
                ent[fn + "_sha256"] = sha(f.read())
        cam = np.fromfile(os.path.join(d, "camera_f32.bin"), np.float32)
        ent["camera_f32"] = [float(x).hex() for x in cam]
        for fn in ("materials", "emitters", "shapes"):
            with open(os.path.join(d, fn + ".txt")) as f:
                ent[fn + "_txt"] = f.read().splitlines()
        manifest["scenes"][scene] = ent
        print(scene, info)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
