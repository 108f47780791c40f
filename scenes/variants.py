"""Scene catalogue for tests and the bench.

Each entry names an OBJ under scenes/ plus the camera / renderer settings of the
reference TOML it comes from. Variants that only change a material are
materialised into a scratch directory (the OBJ is symlinked, the MTL rewritten),
so the repository keeps one copy of each mesh.
"""
from __future__ import annotations

import os
import re
import shutil
import tempfile

ROOT = os.path.dirname(os.path.abspath(__file__))

# Camera of data/a5/cbox/tinyrender/cbox_bdpt_glass.toml and
# data/a5/bonus_bdpt/tinyrender/cbox_bdpt.toml (identical in both).
CBOX_CAMERA = dict(eye=[0.0, 0.8, 3.8], at=[0.0, 0.8, 0.0], up=[0.0, 1.0, 0.0], fov=30.0)

SCENES = {
    # BASELINE.json configs[0]: diffuse-only cbox_low, rrDepth default 5.
    "cbox_low": dict(obj="cbox/cbox_low.obj", camera=CBOX_CAMERA, rr_depth=5),
    # configs[1]/[3]: CausticSample (cbox_mirror: glass sphere, mixture wall), rrDepth 8.
    "caustic": dict(obj="cbox/cbox_mirror.obj", camera=CBOX_CAMERA, rr_depth=8),
    # configs[2]: HardLightSample (bonus_bdpt: tiny disc light, mixture sphere), rrDepth 2.
    "hardlight": dict(obj="bonus_bdpt/cbox.obj", camera=CBOX_CAMERA, rr_depth=2),
    # Perfect-mirror variant: the HardLight scene with the sphere switched to
    # illum 3 (MirrorBSDF). No shipped material uses illum 3.
    "hardlight_mirror": dict(obj="bonus_bdpt/cbox.obj", camera=CBOX_CAMERA, rr_depth=5,
                             mtl_patch={"rightSphere": {"illum": "3"}}),
}


def _patch_mtl(text: str, patch: dict) -> str:
    out, cur = [], None
    for line in text.splitlines():
        m = re.match(r"\s*newmtl\s+(.*)$", line)
        if m:
            cur = m.group(1).strip()
        key = line.strip().split(" ")[0] if line.strip() else ""
        if cur in patch and key in patch[cur]:
            line = f"{key} {patch[cur][key]}"
        out.append(line)
    return "\n".join(out) + "\n"


def obj_path(name: str, scratch: str | None = None) -> str:
    """Absolute OBJ path for a catalogue scene (materialising variants)."""
    sc = SCENES[name]
    src = os.path.join(ROOT, sc["obj"])
    if "mtl_patch" not in sc:
        return src
    scratch = scratch or os.path.join(tempfile.gettempdir(), "bdpt_scene_variants")
    d = os.path.join(scratch, name)
    os.makedirs(d, exist_ok=True)
    dst = os.path.join(d, os.path.basename(src))
    if not os.path.exists(dst):
        try:
            os.symlink(src, dst)
        except OSError:
            shutil.copyfile(src, dst)
    with open(src, "r") as f:
        mtllib = re.search(r"^mtllib\s+(\S+)", f.read(4096), re.M).group(1)
    with open(os.path.join(os.path.dirname(src), mtllib)) as f:
        text = _patch_mtl(f.read(), sc["mtl_patch"])
    with open(os.path.join(d, mtllib), "w") as f:
        f.write(text)
    return dst


def toml_text(name: str, width: int, height: int, spp: int, rr_depth: int | None = None) -> str:
    sc = SCENES[name]
    cam = sc["camera"]
    rr = sc["rr_depth"] if rr_depth is None else rr_depth
    f3 = lambda v: "[ " + ", ".join(repr(float(x)) for x in v) + " ]"
    return (f'[input]\nobjfile = "{obj_path(name)}"\n\n[camera]\neye = {f3(cam["eye"])}\nat = {f3(cam["at"])}\n'
            f'up = {f3(cam["up"])}\nfov = {float(cam["fov"])!r}\n\n[film]\nwidth = {width}\nheight = {height}\n\n'
            f'[renderer]\nrealtime = false\ntype = "bdpt"\nrrDepth = {rr}\nrrProb = 0.95\nspp = {spp}\n')
