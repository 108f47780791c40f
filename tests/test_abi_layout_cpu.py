"""The ctypes mirror of include/bdpt_amd.h (bdpt_amd.py) against the header itself:
every struct the Python side passes across the C-ABI has the size and field
offsets gcc gives the C declaration (a field added on one side only would shift
everything after it without any error at the call). CPU only: a small C program
compiled against the header prints sizeof / offsetof."""
import ctypes
import os
import subprocess

import pytest

import bdpt_amd

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (C type, ctypes mirror)
STRUCTS = [
    ("bdpt_camera", bdpt_amd._Camera),
    ("bdpt_frame_params", bdpt_amd._FrameParams),
    ("bdpt_scene_info", bdpt_amd._SceneInfo),
    ("bdpt_path_params", bdpt_amd._PathParams),
    ("bdpt_direct_params", bdpt_amd._DirectParams),
    ("bdpt_config", bdpt_amd._Config),
    ("bdpt_splat", bdpt_amd._Splat),
    ("bdpt_multi_stats", bdpt_amd._MultiStats),
    ("bdpt_material_desc", bdpt_amd._MaterialDesc),
    ("bdpt_emitter_desc", bdpt_amd._EmitterDesc),
    ("bdpt_bvh_node_desc", bdpt_amd._BvhNodeDesc),
    ("bdpt_scene_desc", bdpt_amd._SceneDesc),
    ("bdpt_stats", bdpt_amd._Stats),
]


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "bdpt_amd.h"', "int main(void) {"]
    lines.append('    printf("bdpt_hit size %zu\\n", sizeof(bdpt_hit));')
    for fname in bdpt_amd.HIT_DTYPE.names:
        lines.append(f'    printf("bdpt_hit {fname} %zu\\n", offsetof(bdpt_hit, {fname}));')
    for cname, mirror in STRUCTS:
        lines.append(f'    printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in mirror._fields_:
            lines.append(f'    printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ["    return 0;", "}"]
    src = d / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = d / "layout"
    r = subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    layout = {}
    for ln in out.splitlines():
        cname, key, val = ln.split()
        layout[(cname, key)] = int(val)
    return layout


@pytest.mark.parametrize("cname,mirror", STRUCTS, ids=[c for c, _ in STRUCTS])
def test_ctypes_mirror_matches_header(c_layout, cname, mirror):
    assert ctypes.sizeof(mirror) == c_layout[(cname, "size")], cname
    for fname, _ in mirror._fields_:
        assert getattr(mirror, fname).offset == c_layout[(cname, fname)], (cname, fname)


def test_hit_dtype_matches_header(c_layout):
    """bdpt_intersect / bdpt_intersect_from fill a numpy array of HIT_DTYPE."""
    dt = bdpt_amd.HIT_DTYPE
    assert dt.itemsize == c_layout[("bdpt_hit", "size")]
    for fname in dt.names:
        assert dt.fields[fname][1] == c_layout[("bdpt_hit", fname)], fname
