"""Synthetic 1M-triangle scene (BASELINE.json configs[4]).

The Cornell box of data/a5/cbox/mesh/cbox_low.obj (walls, floor, ceiling,
light, left box — every shape but its low-poly sphere) plus two UV spheres of
708 x 354 segments (2 x 501 264 triangles, quads split into two triangles, the
pole rows kept as degenerate-free fans' quads so every segment is two faces):
one diffuse (the leftBox material), one glass (illum 6, Ni 1.5). About one
million triangles — a BVH-bandwidth stress case whose scene data (~100 MB with
the BVH) does not fit the 4 MB-per-XCD L2.

The OBJ is written deterministically into a scratch directory on first use
(`obj_path()`), with per-vertex normals and global vertex indices that stay
valid after the dropped shape.
"""
from __future__ import annotations

import os
import re
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
SRC_OBJ = os.path.join(ROOT, "cbox", "cbox_low.obj")
SRC_MTL = os.path.join(ROOT, "cbox", "cbox_low.mtl")
SEG_U, SEG_V = 708, 354
SPHERES = [  # (object name, material, centre, radius)
    ("diffuseSphere", "leftBox", (-0.42, 0.33, 0.25), 0.33),
    ("glassSphere", "glassSphere", (0.42, 0.33, -0.22), 0.33),
]
GLASS_MTL = "newmtl glassSphere\nNs 10\nKa 1 1 1\nKd 1 1 1\nKs 0 0 0\nKe 0 0 0\nTf 1 1 1\nNi 1.5\nd 1\nillum 6\n"


def _cbox_without_sphere():
    """(vertex lines, normal lines, shape blocks) of cbox_low.obj minus rightSphere,
    with face indices renumbered to the kept vertices/normals."""
    lines = open(SRC_OBJ).read().splitlines()
    verts, norms, shapes = [], [], []
    cur = None
    for ln in lines:
        if ln.startswith("v "):
            verts.append(ln)
        elif ln.startswith("vn "):
            norms.append(ln)
        elif ln.startswith("o "):
            cur = {"name": ln[2:].strip(), "lines": []}
            shapes.append(cur)
        elif cur is not None and (ln.startswith("f ") or ln.startswith("usemtl") or ln.startswith("s ")):
            cur["lines"].append(ln)
    keep = [s for s in shapes if s["name"] != "rightSphere"]
    used_v, used_n = set(), set()
    for s in keep:
        for ln in s["lines"]:
            if ln.startswith("f "):
                for c in ln.split()[1:]:
                    p = c.split("/")
                    used_v.add(int(p[0]))
                    if len(p) > 2 and p[2]:
                        used_n.add(int(p[2]))
    vmap = {old: i + 1 for i, old in enumerate(sorted(used_v))}
    nmap = {old: i + 1 for i, old in enumerate(sorted(used_n))}
    out_v = [verts[o - 1] for o in sorted(used_v)]
    out_n = [norms[o - 1] for o in sorted(used_n)]
    out_shapes = []
    for s in keep:
        body = []
        for ln in s["lines"]:
            if ln.startswith("f "):
                cs = []
                for c in ln.split()[1:]:
                    p = c.split("/")
                    cs.append(f"{vmap[int(p[0])]}//{nmap[int(p[2])]}")
                body.append("f " + " ".join(cs))
            else:
                body.append(ln)
        out_shapes.append((s["name"], body))
    return out_v, out_n, out_shapes


def _uv_sphere(center, radius):
    """Vertices/normals on a (SEG_V + 1) x SEG_U grid and 2 * SEG_U * SEG_V triangles."""
    th = np.pi * np.arange(SEG_V + 1) / SEG_V            # polar angle
    ph = 2 * np.pi * np.arange(SEG_U) / SEG_U            # azimuth
    st, ct = np.sin(th)[:, None], np.cos(th)[:, None]
    n = np.stack([st * np.cos(ph)[None, :], np.broadcast_to(ct, (SEG_V + 1, SEG_U)),
                  st * np.sin(ph)[None, :]], -1).reshape(-1, 3)
    v = np.asarray(center)[None, :] + radius * n
    i = np.arange(SEG_V)[:, None]
    j = np.arange(SEG_U)[None, :]
    a = i * SEG_U + j
    b = i * SEG_U + (j + 1) % SEG_U
    c = (i + 1) * SEG_U + j
    d = (i + 1) * SEG_U + (j + 1) % SEG_U
    tris = np.concatenate([np.stack([a, c, b], -1).reshape(-1, 3), np.stack([b, c, d], -1).reshape(-1, 3)])
    return v.astype(np.float32), n.astype(np.float32), tris


def write(dirpath: str) -> str:
    os.makedirs(dirpath, exist_ok=True)
    obj = os.path.join(dirpath, "synth1m.obj")
    if os.path.exists(obj) and os.path.getsize(obj) > 0:
        return obj
    verts, norms, shapes = _cbox_without_sphere()
    nv, nn = len(verts), len(norms)
    tmp = obj + f".{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        f.write("# synthetic 1M-triangle Cornell box (scenes/synth.py)\nmtllib synth1m.mtl\n")
        f.write("\n".join(verts) + "\n" + "\n".join(norms) + "\n")
        for name, body in shapes:
            f.write(f"o {name}\n" + "\n".join(body) + "\n")
        for name, mtl, center, radius in SPHERES:
            v, n, t = _uv_sphere(center, radius)
            f.write(f"o {name}\n")
            np.savetxt(f, v, fmt="v %.6f %.6f %.6f")
            np.savetxt(f, n, fmt="vn %.6f %.6f %.6f")
            f.write(f"usemtl {mtl}\ns off\n")
            tv = t + 1 + nv
            tn = t + 1 + nn
            faces = np.stack([tv[:, 0], tn[:, 0], tv[:, 1], tn[:, 1], tv[:, 2], tn[:, 2]], -1)
            np.savetxt(f, faces, fmt="f %d//%d %d//%d %d//%d")
            nv += len(v)
            nn += len(n)
    os.replace(tmp, obj)
    mtl = open(SRC_MTL).read()
    if not re.search(r"newmtl\s+glassSphere", mtl):
        mtl = mtl.rstrip("\n") + "\n\n" + GLASS_MTL
    with open(os.path.join(dirpath, "synth1m.mtl"), "w") as f:
        f.write(mtl)
    return obj


def obj_path() -> str:
    return write(os.path.join(tempfile.gettempdir(), "bdpt_synth"))


if __name__ == "__main__":
    print(obj_path())
