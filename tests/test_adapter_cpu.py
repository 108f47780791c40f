"""The reference-side binding of INTEGRATION.md, compiled and checked without a GPU.

`make -C oracle/ref adapter` extracts the adapter header and the registration
edits verbatim from INTEGRATION.md (oracle/ref/make_adapter.py), compiles them
with the reference's own integrator.cpp / renderer.cpp / main.cpp and links the
product library. Here (CPU):
* the document's blocks apply to the reference (anchors found exactly once) and
  the binding compiles and links;
* the extraction refuses a missing or repeated anchor;
* the scene descriptor the adapter builds from the reference's in-memory Scene
  (bdpt_scene_create) gives device arrays bit-identical to bdpt_scene_load_obj
  on the same files, for all five catalogue scenes (`adapter_check layout`).
The GPU half (frames through Renderer::render, render(ray, sampler) against the
reference's BDPTIntegrator) is tests/test_gpu_adapter.py.
"""
import json
import os
import subprocess
import sys

import pytest

import bdpt_amd
import variants

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_ROOT = "/root/reference"
AD = os.path.join(REPO, "oracle", "_ref", "adapter")
CHECK = os.path.join(AD, "adapter_check")
MAKE_ADAPTER = os.path.join(REPO, "oracle", "ref", "make_adapter.py")

needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF_ROOT, "src")),
                               reason="reference sources not present (GPU box)")


@pytest.fixture(scope="module")
def built():
    if os.path.isdir(os.path.join(REF_ROOT, "src")):
        r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle", "ref"), "adapter"],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    if not os.path.exists(CHECK):
        pytest.skip("adapter_check not built")
    return CHECK


@needs_ref
def test_integration_md_blocks_apply_and_compile(built):
    hdr = os.path.join(AD, "src", "integrators", "bdpt_gpu.h")
    with open(hdr) as f:
        text = f.read()
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        doc = f.read()
    assert text.strip() in doc  # verbatim
    assert "struct GpuBDPTIntegrator : Integrator" in text
    assert "~GpuBDPTIntegrator" not in text  # Integrator has no virtual destructor (integrator.h:23-31)
    with open(os.path.join(AD, "src", "core", "core.h")) as f:
        core = f.read()
    assert core.index("EBDPTIntegrator,") < core.index("EBDPTGpuIntegrator,") < core.index("EIntegrators")
    with open(os.path.join(AD, "src", "core", "renderer.cpp")) as f:
        rend = f.read()
    assert "#include <integrators/bdpt_gpu.h>" in rend and "gpu->renderFrame();" in rend
    assert os.access(os.path.join(AD, "tinyrender"), os.X_OK)


@needs_ref
@pytest.mark.parametrize("anchor, count", [("NO SUCH LINE", 0), ("}", "many")])
def test_make_adapter_rejects_bad_anchor(tmp_path, anchor, count):
    doc = tmp_path / "doc.md"
    doc.write_text('<!-- adapter-file: src/x.h -->\n```cpp\nint x;\n```\n'
                   f'<!-- adapter-edit: src/core/core.h after {json.dumps(anchor)} -->\n```cpp\n// y\n```\n')
    r = subprocess.run([sys.executable, MAKE_ADAPTER, str(doc), REF_ROOT, str(tmp_path / "out")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "anchor" in (r.stdout + r.stderr)


def _toml(tmp_path, name):
    p = tmp_path / f"{name}.toml"
    p.write_text(variants.toml_text(name, 64, 64, 1, kind="bdpt_gpu"))
    return str(p)


@needs_ref
@pytest.mark.parametrize("name", ["cbox_low", "caustic", "hardlight", "hardlight_mirror", "synth1m"])
def test_scene_desc_from_reference_scene_equals_obj_ingest(built, tmp_path, name):
    """Every device array (tri, shade, both trees, leaf boxes, BSDF / emitter
    records, emitter faces and CDFs, shape map, roots) from the reference's own
    Scene through bdpt_scene_create equals the OBJ path's, bit for bit."""
    r = subprocess.run([built, "layout", _toml(tmp_path, name)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    assert out["mismatches"] == 0 and out["info_equal"]
    assert all(a["equal"] for a in out["arrays"]) and len(out["arrays"]) == len(bdpt_amd.LAYOUT_ARRAYS)
    assert out["triangles"] > 0 and out["bytes"] > 0
