"""The multi-device decomposition through the product library (SURVEY §5,
§8(e)): interleaved row shards rendered by libbdpt_amd.so, summed into one
frame, equal to the reference's frame.

* bdpt_multi_* (one process, one context + stream per device): devices [0] run
  the RCCL path (ncclCommInitAll + ncclReduce, a one-rank communicator on this
  one-GPU box); [0, 0] and [0, 0, 0] rehearse 2 / 3 shards on one GPU (local sum).
* torch.distributed (bench.py's path): two gloo ranks, both on GPU 0, each
  renders its shard with the product library; dist.reduce sums the frames.
* tinyrender_amd --devices 0,0: the CLI over bdpt_multi, EXR decoded against the golden.
"""
import os
import socket
import subprocess

import numpy as np
import pytest

import bdpt_amd
import bdpt_dist
import variants
from conftest import REPO, load_golden

pytestmark = pytest.mark.gpu
TOL = 1e-4  # per-pixel relative L2 (BASELINE north star)


def rel_l2(fb, ref):
    a, r = np.asarray(fb, np.float64).reshape(-1, 3), np.asarray(ref, np.float64).reshape(-1, 3)
    return float((np.linalg.norm(a - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)).max())


def config(m, rr=None):
    cam = bdpt_amd.Camera(**variants.SCENES[m["scene"]]["camera"])
    return bdpt_amd.Config(camera=cam, width=m["width"], height=m["height"], spp=m["spp"],
                           rr_depth=rr if rr is not None else m.get("rr_depth", variants.SCENES[m["scene"]]["rr_depth"]))


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_gpu_multi_device_bdpt_frame_equals_reference(golden_manifest, devices):
    name = "G2_caustic_64x64_spp16"
    m = golden_manifest["framebuffers"][name]
    sc = bdpt_amd.Scene(variants.obj_path(m["scene"]))
    r = bdpt_amd.MultiDeviceRenderer(sc, config(m, m["rr_depth"]), devices)
    fb = r.render_frame()
    st = r.stats()
    assert st["rccl"] == (len(set(devices)) == len(devices))
    assert st["samples"] == m["width"] * m["height"] * m["spp"]
    # every shard did its share (rows i, i + N, ...)
    rows = [len(bdpt_dist.shard_rows(i, len(devices), m["height"])) for i in range(len(devices))]
    assert st["device_samples"] == [k * m["width"] * m["spp"] for k in rows]
    assert rel_l2(fb, load_golden(name)) <= TOL


def test_gpu_multi_device_accumulates_onto_the_callers_frame(golden_manifest):
    """bdpt_multi_render_host ADDS, as bdpt_render_host does: two calls = 2x frame."""
    name = "G1_cbox_low_64x64_spp4"
    m = golden_manifest["framebuffers"][name]
    sc = bdpt_amd.Scene(variants.obj_path(m["scene"]))
    r = bdpt_amd.MultiDeviceRenderer(sc, config(m, m["rr_depth"]), [0, 0])
    a = r.render_frame()
    c = config(m, m["rr_depth"])
    p = bdpt_amd._FrameParams()
    p.camera, p.width, p.height, p.spp, p.rr_depth = c.camera.c(), c.width, c.height, c.spp, c.rr_depth
    p.seed_base, p.row_stride = c.seed_base, 1
    rgb = a.copy()
    bdpt_amd._check(bdpt_amd.lib().bdpt_multi_render_host(r._h, p, None, None, rgb.ctypes.data))
    assert rel_l2(rgb, 2 * load_golden(name)) <= TOL


@pytest.mark.parametrize("kind,name", [("path", "P3_caustic_path_mis_48x48_spp4"),
                                       ("direct", "D6_hardlight_direct_mis_48x48_spp4")])
def test_gpu_multi_device_other_integrators(golden_manifest, kind, name):
    m = golden_manifest[f"{kind}_framebuffers"][name]
    sc = bdpt_amd.Scene(variants.obj_path(m["scene"]))
    if kind == "path":
        kw = dict(path=bdpt_amd.PathSettings(**m["path"]))
    else:
        d = dict(m["direct"])
        kw = dict(direct=bdpt_amd.DirectSettings(sampling_strategy=d.pop("strategy"), **d))
    r = bdpt_amd.MultiDeviceRenderer(sc, config(m, 5), [0, 0], **kw)
    assert rel_l2(r.render_frame(), load_golden(name)) <= TOL


def test_gpu_multi_device_rejects_bad_arguments():
    sc = bdpt_amd.Scene(variants.obj_path("cbox_low"))
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**variants.SCENES["cbox_low"]["camera"]), width=8, height=8, spp=1)
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.MultiDeviceRenderer(sc, cfg, [bdpt_amd.device_count()])
    with pytest.raises(bdpt_amd.BdptError):
        bdpt_amd.MultiDeviceRenderer(sc, cfg, [])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, name, out):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json
        with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
            m = json.load(f)["framebuffers"][name]
        it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(m["scene"])), config(m, m["rr_depth"]), device=0)
        it.init()
        off, stride = bdpt_dist.row_shard(rank, world)
        fb = torch.from_numpy(it.render_frame(row_offset=off, row_stride=stride).copy())
        n = torch.tensor([it.stats()["samples"]], dtype=torch.int64)
        bdpt_dist.reduce_framebuffer(fb, dst=0)
        dist.all_reduce(n)
        if rank == 0:
            np.save(out, fb.numpy())
            np.save(out + ".n.npy", n.numpy())
    finally:
        dist.destroy_process_group()


def test_gpu_two_gloo_ranks_render_shards_with_the_product_library(golden_manifest, tmp_path):
    """bench.py's decomposition with the product library as the per-rank renderer
    (two processes on GPU 0), reduced over gloo: equals the reference frame."""
    import torch.multiprocessing as mp

    name = "G3_hardlight_64x64_spp16"
    m = golden_manifest["framebuffers"][name]
    out = str(tmp_path / "fb.npy")
    mp.spawn(_rank, args=(2, _free_port(), name, out), nprocs=2, join=True)
    assert int(np.load(out + ".n.npy")[0]) == m["width"] * m["height"] * m["spp"]
    assert rel_l2(np.load(out), load_golden(name)) <= TOL


def test_gpu_cli_devices_flag(golden_manifest, tmp_path):
    """tinyrender_amd <toml> nogui --devices 0,0: two shards + sum, EXR next to the TOML."""
    name = "G2_caustic_64x64_spp16"
    m = golden_manifest["framebuffers"][name]
    toml = tmp_path / "scene.toml"
    toml.write_text(variants.toml_text(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"]))
    exe = os.path.join(REPO, "bidirectional-path-tracing_amd", "lib", "tinyrender_amd")
    r = subprocess.run([exe, str(toml), "nogui", "--devices", "0,0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "2 devices (local sum)" in r.stdout
    from test_config_exr import decode_exr

    img = decode_exr((tmp_path / "scene.exr").read_bytes()).astype(np.float32)
    ref = load_golden(name).reshape(m["height"], m["width"], 3).astype(np.float16).astype(np.float32)
    assert np.allclose(img, ref, rtol=2 ** -10, atol=0)


@pytest.mark.parametrize("pipeline", ["1", "2"])
def test_gpu_bench_two_rank_rehearsal(tmp_path, pipeline):
    """bench.py's N > 1 path (torch.distributed.run, one rank per device, barrier +
    max-over-ranks timing, row shards, the framebuffer reduce, rank 0's JSON line), one and two frames in flight,
    rehearsed on this one-GPU box: BDPT_BENCH_REHEARSAL=1 puts both ranks on GPU 0
    and reduces over gloo instead of RCCL."""
    import json
    import sys

    env = dict(os.environ, BDPT_BENCH_REHEARSAL="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--width", "64", "--height", "64", "--spp", "4",
           "--no-cpu", "--pipeline", pipeline]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["samples_per_step"] == 64 * 64 * 4
    rk = out["ranks"]  # what a scaling run needs to be diagnosed
    assert rk["world_size"] == 2 and rk["backend"] == "gloo" and rk["rehearsal_one_device"]
    assert len(rk["kernel_ms"]) == 2 and min(rk["kernel_ms"]) > 0
    assert out["config"]["frames_in_flight"] == int(pipeline)
    if pipeline == "1":  # (frames in flight: the reduce runs on the frame's stream, untimed)
        assert len(rk["reduce_ms"]) == 2
    assert sum(rk["samples"]) == 64 * 64 * 4 and rk["kernel_ms_max"] >= rk["kernel_ms_min"]
