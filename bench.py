"""Benchmark of the MI355X BDPT hot path (BASELINE.json metric).

A step = one full frame of the CausticSample scene (cbox_mirror, rrDepth 8) at
512x512 and 256 spp = 67,108,864 camera samples (one eye + one light subpath
each), rendered by the HIP megakernel into a float32 framebuffer in HBM, plus
— with N > 1 ranks — the RCCL sum-reduce of the framebuffer to rank 0. Ranks
render interleaved rows of the same image (strong scaling); every rank splats
into its own full-frame buffer, so the reduce is the path's one exchange step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (metric, value = whole-job Msamples/s, roofline of
the render kernel, cpu_baseline = the reference CPU path timed on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "bidirectional-path-tracing_amd"), os.path.join(REPO, "scenes"),
          os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

# torch first: its HIP runtime is then the one the product library binds to
# (both carry SONAME libamdhip64.so.7), so framebuffer tensors and streams are shared.
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bdpt_amd  # noqa: E402
import bdpt_dist  # noqa: E402
import variants  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SCENE_LABEL = {
    "caustic": "CausticSample (cbox_mirror.obj)",
    "hardlight": "HardLightSample (bonus_bdpt cbox.obj)",
    "hardlight_mirror": "HardLightSample, sphere as perfect mirror (illum 3)",
    "cbox_low": "diffuse Cornell box (cbox_low.obj)",
    "synth1m": "synthetic 1M-triangle box (scenes/synth.py)",
}
METRIC = "Msamples/sec (whole node) at 256 spp, Cornell caustic 512², 1/2/4/8 GPUs"


def algorithmic_bytes_per_sample(c: dict, samples: int) -> float:
    """SURVEY.md §8(d) byte model on this build's data layout, evaluated on its
    own counting pass (DESIGN.md "Roofline"): 112 B per 4-wide node visit (six
    child-bound float4 + the link float4), 48 B per triangle test (v0, e1, e2),
    96 B per shaded closest hit (v0 + the 80-byte shading record), 64 B per
    light vertex written or read, 12 B per framebuffer add (camera splats and
    the per-sample eye estimate)."""
    b = (112 * c["interior_visits"] + 48 * c["tri_tests"] + 96 * c["closest_rays"]
         + 64 * (c["light_verts"] + c["light_vert_reads"]) + 12 * (c["splats"] + samples))
    return b / max(samples, 1)


def cpu_baseline(scene: str, W: int, H: int, spp: int, rr: int, integrator: str = "bdpt") -> dict:
    """The reference CPU path (oracle/_ref/ref_bdpt = the unmodified reference
    BDPT compiled from its sources) on a bounded sample of the same workload:
    every `stride`-th row of the 512x512 image at the bench spp, std::thread over
    the host's cores. Falls back to the C restatement (kind "port")."""
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    ref = os.path.join(REPO, "oracle", "_ref", "ref_bdpt")
    toml = os.path.join("/tmp", f"bench_{scene}_{os.getpid()}.toml")
    with open(toml, "w") as f:
        if integrator == "bdpt":
            f.write(variants.toml_text(scene, W, H, spp, rr))
        elif integrator == "path":
            f.write(variants.path_toml_text(scene, W, H, spp))
        else:
            f.write(variants.direct_toml_text(scene, W, H, spp))
    # ~6 rows per thread: 10-20 s of wall time at the reference's ~18 us per caustic sample-thread
    stride = max(1, H // (6 * threads))
    if os.path.exists(ref):
        rr_arg = ["--rr", str(rr)] if integrator == "bdpt" else []
        out = subprocess.run([ref, "render", toml, str(W), str(H), str(spp), *rr_arg, "--threads",
                              str(threads), "--row-stride", str(stride)], capture_output=True, text=True,
                             check=True, timeout=900)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        kind, val, secs, samples = "reference", r["msamples_per_s"], r["seconds"], r["samples"]
    else:
        import oracle as O
        sc = O.Scene(variants.obj_path(scene))
        cam = variants.SCENES[scene]["camera"]
        p = (O.make_params(cam, W, H, spp, rr) if integrator == "bdpt" else
             O.make_path_params(cam, W, H, spp) if integrator == "path" else O.make_direct_params(cam, W, H, spp))
        t = time.time()
        _, samples = sc.render(p, threads=threads, rows=list(range(0, H, stride)))
        secs = time.time() - t
        kind, val = "port", samples / secs * 1e-6
    os.unlink(toml)
    return {"value": round(val, 6), "unit": "Msamples/s", "cores": threads, "kind": kind,
            "sample": f"{scene} {W}x{H}, {spp} spp, every {stride}th row ({samples} camera samples, "
                      f"{secs:.1f} s wall, {threads} threads)"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="caustic")
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--rr-depth", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--integrator", choices=["bdpt", "path", "direct"], default="bdpt",
                    help="bdpt = the hot path (BASELINE metric); path = the reference's PathTracerIntegrator "
                         "(path.h, cbox_bdpt_path.toml settings), direct = its DirectIntegrator (direct.h, MIS, "
                         "1 emitter + 1 BSDF sample) on the same substrate, for comparison")
    ap.add_argument("--schedule", choices=["megakernel", "wavefront"], default="megakernel",
                    help="render schedule (BDPT_FLAG_WAVEFRONT for the shade/trace passes)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_caustic_512x512_256spp.json"),
                    help="measured HBM bytes per launch (rocprofv3 --pmc summary) for roofline.traffic")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    sc = variants.SCENES[args.scene]
    rr = args.rr_depth or sc["rr_depth"]
    W, H, spp = args.width, args.height, args.spp
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**sc["camera"]), width=W, height=H, spp=spp, rr_depth=rr)
    if args.integrator == "path":
        integ = bdpt_amd.PathTracerIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                              bdpt_amd.PathSettings(), device=local if world > 1 else 0)
    elif args.integrator == "direct":
        integ = bdpt_amd.DirectIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                          bdpt_amd.DirectSettings(sampling_strategy="mis"),
                                          device=local if world > 1 else 0)
    else:
        integ = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                        device=local if world > 1 else 0)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    kernel_ms = []
    sched_flags = bdpt_amd.FLAG_WAVEFRONT if args.schedule == "wavefront" else 0

    row_offset, row_stride = bdpt_dist.row_shard(rank, world)

    def step():
        fb.zero_()
        integ.render_device(fb.data_ptr(), stream, row_offset=row_offset, row_stride=row_stride, flags=sched_flags)
        kernel_ms.append(integ.stats()["kernel_ms"])  # waits for the render kernel's end event
        bdpt_dist.reduce_framebuffer(fb, dst=0)

    for _ in range(args.warmup):
        step()
    kernel_ms.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples_total = W * H * spp  # all ranks together, per step
    value = samples_total * args.steps / elapsed * 1e-6
    local_samples = integ.stats()["samples"]
    avg_kernel_ms = sum(kernel_ms) / max(len(kernel_ms), 1)

    if rank == 0 and args.integrator in ("path", "direct"):
        metric = ("Msamples/sec, PathTracerIntegrator (path.h, explicit, RR 0.95 past depth 5)"
                  if args.integrator == "path" else
                  "Msamples/sec, DirectIntegrator (direct.h, MIS, 1 emitter + 1 BSDF sample)")
        out = {"metric": metric,
               "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic camera samples",
               "config": {"workload": f"{args.integrator}_{args.scene}_{W}x{H}_{spp}spp",
                          "scene": SCENE_LABEL.get(args.scene),
                          "kernel_ms": round(avg_kernel_ms, 3)}}
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args.scene, W, H, spp, rr, integrator=args.integrator)
        print(json.dumps(out), flush=True)
    elif rank == 0:
        # algorithmic bytes per sample from a counting pass (untimed, same seeds, smaller spp)
        cnt_cfg = bdpt_amd.Config(camera=cfg.camera, width=W, height=H, spp=min(spp, 16), rr_depth=rr)
        cnt = bdpt_amd.BDPTIntegrator(integ.scene, cnt_cfg, device=local if world > 1 else 0)
        cbuf = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
        cnt.render_device(cbuf.data_ptr(), stream, flags=bdpt_amd.FLAG_COUNT | sched_flags)
        cst = cnt.stats()
        bps = algorithmic_bytes_per_sample(cst["counters"], cst["samples"])
        achieved = bps * local_samples / (avg_kernel_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.pmc):
            with open(args.pmc) as f:
                pm = json.load(f)
            if pm.get("config") == f"{args.scene}_{W}x{H}_{spp}spp":
                traffic = pm.get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic camera samples over the reference's own scene files" if args.scene != "synth1m"
                     else "synthetic camera samples over a generated 1M-triangle scene"),
            "config": {"workload": f"{args.scene}_{W}x{H}_{spp}spp", "scene": SCENE_LABEL.get(args.scene, args.scene),
                       "width": W, "height": H, "spp": spp, "rr_depth": rr, "samples_per_step": samples_total,
                       "parallelism": f"{world}-way row-interleaved shards + RCCL sum-reduce"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "kernel": "bdpt_frame_kernel" if args.schedule == "megakernel"
                         else "bdpt_shade_kernel + bdpt_trace_kernel",
                         "schedule": args.schedule, "kernel_ms": round(avg_kernel_ms, 3),
                         "bytes_per_sample": round(bps, 1),
                         "counts_per_sample": {k: round(v / cst["samples"], 3) for k, v in cst["counters"].items()}},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args.scene, W, H, spp, rr)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
