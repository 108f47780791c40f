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


# SURVEY.md §8(d) byte model (the figure `roofline.achieved` is priced on):
# 64 B per interior node visit, 36 B per triangle test (3 float3 vertices), 40 B
# per closest hit (3 normals + matID for shading), 64 B per light vertex written
# or read, 12 B per framebuffer add (camera splats + the per-sample eye estimate).
SURVEY_BYTES = dict(node=64, tri=36, hit=40, vertex=64, fb=12)
# This build's own layout: 112 B per 4-wide node visit (six child-bound float4 +
# the link float4), 48 B per triangle test (v0, e1, e2), 96 B per shaded closest
# hit (v0 + the 80-byte shading record); vertices and framebuffer as above.
LAYOUT_BYTES = dict(node=112, tri=48, hit=96, vertex=64, fb=12)


def algorithmic_bytes_per_sample(c: dict, samples: int, m: dict = SURVEY_BYTES) -> float:
    """Bytes per camera sample under byte model `m`, evaluated on the build's own
    counting pass (same seeds): counters interior_visits, tri_tests,
    closest_rays, light_verts + light_vert_reads, splats (+1 eye add)."""
    b = (m["node"] * c["interior_visits"] + m["tri"] * c["tri_tests"] + m["hit"] * c["closest_rays"]
         + m["vertex"] * (c["light_verts"] + c["light_vert_reads"]) + m["fb"] * (c["splats"] + samples))
    return b / max(samples, 1)


def algorithmic_write_bytes(c: dict, samples: int) -> float:
    """Bytes per camera sample the algorithm must write: every light-vertex
    record (64 B) and every framebuffer add (12 B: camera splats + the eye add)."""
    return (64 * c["light_verts"] + 12 * (c["splats"] + samples)) / max(samples, 1)


# Reference CPU cost per camera sample and thread (measured on the GPU box's host,
# round 1) — only sizes the bounded CPU sample.
CPU_US_PER_SAMPLE = {"caustic": 18.0, "hardlight": 5.0, "hardlight_mirror": 9.0, "cbox_low": 9.0, "synth1m": 35.0}
RR_CPU_FACTOR = 3.5  # Russian roulette: subpaths continue past rrDepth (Caustic 512², 8 threads: 3.5x)


def host_cpus() -> dict:
    """The host cores this job may use: the scheduler affinity set, capped by the
    cgroup CPU quota (on the GPU box the job's share of a larger machine; nproc
    there reports the whole machine), plus the machine's CPU count and model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "model": model}


def cpu_baseline(scene: str, W: int, H: int, spp: int, rr: int, integrator: str = "bdpt",
                 frame_out: str | None = None, russian_roulette: bool = False) -> dict:
    """The reference CPU path (oracle/_ref/ref_bdpt = the unmodified reference
    BDPT compiled from its sources) on a bounded sample of the same workload:
    every `stride`-th row of the image at the bench spp, std::thread over every
    host core this job may use. With `frame_out`, the reference's framebuffer of
    that row shard is written there (for the in-run parity check). Falls back to
    the C restatement (kind "port") when the reference binary is absent. With
    russian_roulette the reference is the NO_RR = 0 build (oracle/_ref/ref_bdpt_rr,
    bdpt.h:18 flipped)."""
    cpus = host_cpus()
    threads = cpus["usable"]
    ref = os.path.join(REPO, "oracle", "_ref", "ref_bdpt_rr" if russian_roulette else "ref_bdpt")
    toml = os.path.join("/tmp", f"bench_{scene}_{os.getpid()}.toml")
    with open(toml, "w") as f:
        if integrator == "bdpt":
            f.write(variants.toml_text(scene, W, H, spp, rr))
        elif integrator == "path":
            f.write(variants.path_toml_text(scene, W, H, spp))
        else:
            f.write(variants.direct_toml_text(scene, W, H, spp))
    # about 15 s of wall time at the reference's per-sample cost on one thread
    us = CPU_US_PER_SAMPLE.get(scene, 20.0) * (RR_CPU_FACTOR if russian_roulette else 1.0)
    target_samples = 15.0 * threads / (us * 1e-6)
    stride = max(1, int(round(H * W * spp / max(target_samples, 1.0))))
    stride = min(stride, H)
    if os.path.exists(ref):
        rr_arg = ["--rr", str(rr)] if integrator == "bdpt" else []
        out_arg = ["--out", frame_out] if frame_out else []
        out = subprocess.run([ref, "render", toml, str(W), str(H), str(spp), *rr_arg, "--threads",
                              str(threads), "--row-stride", str(stride), *out_arg], capture_output=True, text=True,
                             check=True, timeout=900)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        kind, val, secs, samples = "reference", r["msamples_per_s"], r["seconds"], r["samples"]
    else:
        import numpy as np
        import oracle as O
        sc = O.Scene(variants.obj_path(scene))
        cam = variants.SCENES[scene]["camera"]
        p = (O.make_params(cam, W, H, spp, rr, russian_roulette=int(russian_roulette)) if integrator == "bdpt" else
             O.make_path_params(cam, W, H, spp) if integrator == "path" else O.make_direct_params(cam, W, H, spp))
        t = time.time()
        fbo, samples = sc.render(p, threads=threads, rows=list(range(0, H, stride)))
        secs = time.time() - t
        kind, val = "port", samples / secs * 1e-6
        if frame_out:
            np.asarray(fbo, np.float32).tofile(frame_out)
    os.unlink(toml)
    return {"value": round(val, 6), "unit": "Msamples/s", "cores": threads, "kind": kind,
            "sample": f"{scene} {W}x{H}, {spp} spp, every {stride}th row from row 0 ({samples} camera samples, "
                      f"{secs:.1f} s wall, {threads} threads)",
            "row_stride": stride, "host": cpus}


def frame_parity(gpu, ref) -> dict:
    """Per-pixel relative L2 ||g - r|| / max(||r||, 1e-8) (north star: <= 1e-4)."""
    import numpy as np

    g = np.asarray(gpu, np.float64).reshape(-1, 3)
    r = np.asarray(ref, np.float64).reshape(-1, 3)
    err = np.linalg.norm(g - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)
    return {"max_rel_l2": float(err.max()), "frac_pixels_over_1e-4": float((err > 1e-4).mean()),
            "image_rel_l2": float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)),
            "pixels": int(len(err)), "nonzero_pixels": int((np.abs(r).sum(1) > 0).sum())}


def stamped(path: str, build: str) -> dict | None:
    """A committed profile summary, only if it was measured on this kernel build."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d if d.get("kernel_build") == build else None


def pm_scale(pm: dict, samples: int) -> float:
    """Launch-size ratio of a profiled launch to this run's (the stamped files are
    per launch of the same workload; 1.0 when the sample counts agree)."""
    return pm["samples_per_launch"] / max(samples, 1)


def issue_roofline(deep: dict, kernel_s: float) -> dict | None:
    """The issue roofline the frame kernel is under, from the
    build-stamped pmc_deep counters of one launch and that launch's duration:
      clock           = GRBM_GUI_ACTIVE / XCDs / kernel_s (effective shader clock)
      valu_issue_frac = SQ_INSTS_VALU / (CUs * 4 SIMDs * clock / 2 * kernel_s)
                        (a wave64 VALU instruction issues over 2 cycles)
      lane_frac       = valu_issue_frac * active_lane_frac (of the FP32 vector lane peak)
    plus VALU / SALU wave instructions per sample."""
    c = deep.get("counters_per_launch") or {}
    gui, valu = c.get("GRBM_GUI_ACTIVE"), c.get("SQ_INSTS_VALU")
    if not gui or not valu or kernel_s <= 0:
        return None
    xcds, cus = 8, deep.get("cus", 256)
    clock = gui / xcds / kernel_s
    issue_frac = valu / (cus * 4 * clock / 2 * kernel_s)
    lanes = deep.get("active_lane_frac")
    out = {"bound": "VALU issue", "clock_ghz": round(clock * 1e-9, 3), "valu_issue_frac": round(issue_frac, 4),
           "active_lane_frac": lanes, "lane_frac": round(issue_frac * lanes, 4) if lanes else None,
           "valu_insts_per_sample": deep.get("valu_insts_per_sample"),
           "salu_insts_per_sample": deep.get("salu_insts_per_sample"),
           "wait_frac": deep.get("wait_frac"), "source": deep.get("source"),
           "formula": "lane_frac = SQ_INSTS_VALU / (CUs * 4 * clock / 2 * s) * active_lane_frac, "
                      "clock = GRBM_GUI_ACTIVE / 8 / s"}
    return out


def heartbeat(period: float = 30.0) -> None:
    """A line on stderr every `period` s while the process runs (a Russian-roulette
    frame is one kernel of a minute or more: without output it looks hung)."""
    import threading

    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench] running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main() -> None:
    heartbeat()
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
    ap.add_argument("--count-spp", type=int, default=None,
                    help="spp of the untimed counting pass (default min(spp, 16); 1 with --russian-roulette, where "
                         "a trapped subpath's chain runs at the lone lane's pace in that pass)")
    ap.add_argument("--russian-roulette", action="store_true",
                    help="the reference's NO_RR = 0 branch (bdpt.h:18, :68, :129-132, :188, :201-204): subpaths "
                         "continue past rrDepth by roulette; the bdpt_frame_kernel_rr build, checked against "
                         "oracle/_ref/ref_bdpt_rr")
    ap.add_argument("--integrator", choices=["bdpt", "path", "direct"], default="bdpt",
                    help="bdpt = the hot path (BASELINE metric); path = the reference's PathTracerIntegrator "
                         "(path.h, cbox_bdpt_path.toml settings), direct = its DirectIntegrator (direct.h, MIS, "
                         "1 emitter + 1 BSDF sample) on the same substrate, for comparison")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the in-run parity check of the GPU row shard against the CPU reference frame")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="BDPT frames in flight: 1 (default) = each step waits for its frame; 2 = consecutive "
                         "steps' frames overlap (two contexts, streams and framebuffers): the next frame's blocks "
                         "start on the CUs the previous frame's draining blocks leave, hiding most of the "
                         "persistent grid's end tail, which each of N ranks pays per frame (1/8 row shard: 0.961 "
                         "-> 0.981 of full/8, DESIGN.md §5). Every frame is still rendered whole, into its own "
                         "framebuffer, and reduced; the clock brackets all K steps. (Each launch's event time then "
                         "includes the overlap with its neighbour, so it exceeds the per-step time.)")
    ap.add_argument("--profiles", default=os.path.join(REPO, "profiles"),
                    help="directory of kernel-build-stamped PMC summaries (pmc_<workload>.json, "
                         "pmc_deep_<workload>.json) for roofline.traffic / limiter")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N > 1 path on a one-GPU box (never the driver's runs):
    # BDPT_BENCH_REHEARSAL=1 puts every rank on device 0 and reduces over gloo
    # (RCCL cannot form a communicator with one device twice).
    rehearsal = os.environ.get("BDPT_BENCH_REHEARSAL") == "1"
    gpu = 0 if rehearsal else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu if world > 1 else 0)

    sc = variants.SCENES[args.scene]
    rr = args.rr_depth or sc["rr_depth"]
    W, H, spp = args.width, args.height, args.spp
    rrm = bdpt_amd.RR_LUMINANCE if args.russian_roulette else bdpt_amd.RR_NONE
    if args.russian_roulette and args.integrator != "bdpt":
        sys.exit("--russian-roulette is the BDPT integrator's NO_RR switch")
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**sc["camera"]), width=W, height=H, spp=spp, rr_depth=rr,
                          russian_roulette=rrm)
    if args.integrator == "path":
        integ = bdpt_amd.PathTracerIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                              bdpt_amd.PathSettings(), device=gpu if world > 1 else 0)
    elif args.integrator == "direct":
        integ = bdpt_amd.DirectIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                          bdpt_amd.DirectSettings(sampling_strategy="mis"),
                                          device=gpu if world > 1 else 0)
    else:
        integ = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(args.scene)), cfg,
                                        device=gpu if world > 1 else 0)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    kernel_ms, reduce_ms, tail_ms, capped, parked, longs, express = [], [], [], [], [], [], []

    row_offset, row_stride = bdpt_dist.row_shard(rank, world)

    def step():
        fb.zero_()
        integ.render_device(fb.data_ptr(), stream, row_offset=row_offset, row_stride=row_stride)
        st = integ.stats()  # waits for the render kernel's end event
        kernel_ms.append(st["kernel_ms"])
        tail_ms.append(st.get("tail_ms", 0.0))
        capped.append(st.get("capped_samples", 0))
        parked.append(st.get("parked_samples", 0))
        longs.append(st.get("rr_long_walks_max", 0))
        express.append(st.get("rr_express_iters", [0, 0, 0]))
        if st.get("schedule_errors"):  # draws past the generated MT19937 ring, or a continuation walk out of stack
            raise RuntimeError(f"{st['schedule_errors']} schedule errors in the render")
        if args.integrator == "path":
            integ.check_levels()  # a sample past the 512-level stack would not be the reference's
        if world > 1:  # the exchange step, timed on its own (host wall: it includes waiting for slower ranks)
            r0 = time.perf_counter()
            bdpt_dist.reduce_framebuffer(fb, dst=0)
            torch.cuda.synchronize(dev)
            reduce_ms.append((time.perf_counter() - r0) * 1e3)

    # Pipelined frames (--pipeline 2): step i renders on context / stream / framebuffer i mod 2;
    # a context's stats are read (which waits for its frame) only when it is reused two steps
    # later, so the other stream's frame is already queued behind it.
    nctx = max(1, args.pipeline) if args.integrator == "bdpt" else 1
    if nctx > 1:
        integs = [integ] + [bdpt_amd.BDPTIntegrator(integ.scene, cfg, device=gpu if world > 1 else 0)
                            for _ in range(nctx - 1)]
        fbs = [fb] + [torch.zeros_like(fb) for _ in range(nctx - 1)]
        tstreams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nctx - 1)]
        pending = [False] * nctx
        nstep = [0]

        def collect(j):
            st = integs[j].stats()  # waits for context j's frame
            kernel_ms.append(st["kernel_ms"])
            tail_ms.append(st.get("tail_ms", 0.0))
            capped.append(st.get("capped_samples", 0))
            parked.append(st.get("parked_samples", 0))
            longs.append(st.get("rr_long_walks_max", 0))
            express.append(st.get("rr_express_iters", [0, 0, 0]))
            if st.get("schedule_errors"):
                raise RuntimeError(f"{st['schedule_errors']} schedule errors in the render")
            pending[j] = False

        def step():  # noqa: F811 (the pipelined step)
            j = nstep[0] % nctx
            nstep[0] += 1
            if pending[j]:
                collect(j)
            with torch.cuda.stream(tstreams[j]):
                fbs[j].zero_()
                integs[j].render_device(fbs[j].data_ptr(), tstreams[j].cuda_stream, row_offset=row_offset,
                                        row_stride=row_stride)
                if world > 1:  # the exchange step, on the frame's own stream
                    bdpt_dist.reduce_framebuffer(fbs[j], dst=0)
            pending[j] = True

        def drain():
            for j in range(nctx):
                if pending[j]:
                    collect(j)
    else:
        def drain():
            pass

    for _ in range(args.warmup):
        step()
    drain()
    kernel_ms.clear()
    reduce_ms.clear()
    tail_ms.clear()
    capped.clear()
    parked.clear()
    longs.clear()
    express.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples_total = W * H * spp  # all ranks together, per step
    value = samples_total * args.steps / elapsed * 1e-6
    local_samples = integ.stats()["samples"]
    avg_kernel_ms = sum(kernel_ms) / max(len(kernel_ms), 1)
    ranks = None
    if world > 1:
        # what every rank saw: its render-kernel time, its reduce time, its samples
        mine = torch.tensor([avg_kernel_ms, sum(reduce_ms) / max(len(reduce_ms), 1), float(local_samples)],
                            dtype=torch.float64, device="cpu" if rehearsal else dev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        per = [v.cpu().tolist() for v in allv]
        ranks = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                 "rehearsal_one_device": rehearsal,
                 "kernel_ms": [round(k, 3) for k, _, _ in per],
                 # (with frames in flight the reduce runs on the frame's stream, untimed)
                 "reduce_ms": [round(r, 3) for _, r, _ in per] if nctx == 1 else None,
                 "samples": [int(n) for _, _, n in per],
                 "kernel_ms_min": round(min(k for k, _, _ in per), 3), "kernel_ms_max": round(max(k for k, _, _ in per), 3),
                 "reduce_bytes": W * H * 3 * 4}

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
        if ranks:
            out["ranks"] = ranks
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args.scene, W, H, spp, rr, integrator=args.integrator)
        print(json.dumps(out), flush=True)
    elif rank == 0:
        # algorithmic bytes per sample from a counting pass (untimed, same seeds, smaller spp)
        # (Russian roulette: 1 spp by default — the counting pass keeps every walk in the
        # megakernel, so a trapped subpath's chain there runs at the lone lane's pace; at 1 spp
        # every lane holds one sample, so its SIMD-efficiency counters measure a frame that is
        # all drain: --count-spp 16 for scenes without trapped subpaths)
        count_spp = args.count_spp or (1 if args.russian_roulette else min(spp, 16))
        cnt_cfg = bdpt_amd.Config(camera=cfg.camera, width=W, height=H, spp=count_spp,
                                  rr_depth=rr,
                                  russian_roulette=rrm)
        cnt = bdpt_amd.BDPTIntegrator(integ.scene, cnt_cfg, device=gpu if world > 1 else 0)
        cbuf = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
        cnt.render_device(cbuf.data_ptr(), stream, flags=bdpt_amd.FLAG_COUNT)
        cst = cnt.stats()
        cts = cst["counters"]
        bps = algorithmic_bytes_per_sample(cts, cst["samples"], SURVEY_BYTES)
        bps_layout = algorithmic_bytes_per_sample(cts, cst["samples"], LAYOUT_BYTES)
        kernel_s = avg_kernel_ms * 1e-3
        achieved = bps * local_samples / kernel_s / 1e9
        workload = f"{args.scene}_{W}x{H}_{spp}spp" + ("_rr" if args.russian_roulette else "")
        build = bdpt_amd.kernel_build_hash()
        # measured memory-side traffic and issue counters of THIS kernel build
        # (rocprofv3 --pmc passes, tools/profile_round.sh / tools/pmc_deep.sh)
        pm = stamped(os.path.join(args.profiles, f"pmc_{workload}.json"), build)
        deep = stamped(os.path.join(args.profiles, f"pmc_deep_{workload}.json"), build)
        traffic = pm["hbm_bytes_per_launch"] * local_samples / pm["samples_per_launch"] if pm else None
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                "kernel": cst.get("kernel") or "bdpt_frame_kernel",
                "kernel_build": build, "schedule": "megakernel", "kernel_ms": round(avg_kernel_ms, 3),
                "samples_per_launch": local_samples,
                "byte_model": "SURVEY.md 8(d): 64 B/node visit, 36 B/triangle test, 40 B/closest hit, "
                              "64 B/light vertex written or read, 12 B/framebuffer add",
                "bytes_per_sample": round(bps, 1),
                "bytes_per_sample_layout_model": round(bps_layout, 1),
                "achieved_layout_model": round(bps_layout * local_samples / kernel_s / 1e9, 2),
                "counts_per_sample": {k: round(v / cst["samples"], 3) for k, v in cts.items()},
                # the counting pass's schedule counters (bdpt_stats.sched; Counts::q), per sample
                "sched_per_sample": {k: round(v / cst["samples"], 4) for k, v in cst["sched"].items()},
                # the persistent grid's end tail (device clock: the frame's last 64-sample chunk
                # claimed -> last wave done), what a 1/N row shard pays again per rank
                "tail_ms": round(sum(tail_ms) / max(len(tail_ms), 1), 3)}
        if traffic is not None:
            roof["dram_achieved"] = round(traffic / kernel_s / 1e9, 2)
            roof["dram_frac"] = round(traffic / kernel_s / 1e9 / HBM_PEAK_GBPS, 5)
            roof["traffic_over_algorithmic"] = round(traffic / (bps * local_samples), 4)
            roof["traffic_source"] = pm.get("source")
            # FETCH_SIZE's x2 (MI355X_MICROARCH.md: 128-B requests tallied at 64 B) is calibrated on
            # wide streaming reads only; this kernel's reads are 16-B gathers, so both readings are
            # reported: `traffic` takes the doubled one (the upper bound)
            scale = local_samples / pm["samples_per_launch"]
            roof["traffic_bounds"] = {
                "fetch_x1": round((pm["fetch_size_kib_raw"] * 1024 + pm["write_bytes"]) * scale),
                "fetch_x2": round(traffic),
                "write": round(pm["write_bytes"] * scale),
                "write_over_algorithmic_writes": round(pm["write_bytes"] * scale / max(
                    1.0, algorithmic_write_bytes(cts, cst["samples"]) * local_samples), 3)}
        if deep is not None:
            roof["limiter"] = deep.get("limiter")
            for k in ("active_lane_frac", "valu_issue_frac", "wait_frac", "valu_insts_per_sample"):
                roof[k] = deep.get(k)
            roof["issue_source"] = deep.get("source")
            issue = issue_roofline(deep, kernel_s * pm_scale(deep, local_samples))
            if issue:
                roof["issue"] = issue
                roof["binding"] = issue["bound"]
        default_workload = (args.scene, W, H, spp) == ("caustic", 512, 512, 256) and not args.russian_roulette
        out = {
            "metric": METRIC if default_workload else f"Msamples/sec (whole node), {SCENE_LABEL.get(args.scene, args.scene)} "
                                                      f"{W}x{H} at {spp} spp",
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
            "config": {"workload": workload, "scene": SCENE_LABEL.get(args.scene, args.scene),
                       "width": W, "height": H, "spp": spp, "rr_depth": rr, "samples_per_step": samples_total,
                       "frames_in_flight": nctx,
                       "parallelism": (f"{world}-way row-interleaved shards + one framebuffer sum-reduce "
                                       f"({ranks['backend']})" if ranks else "one GPU, whole image (no reduce)")},
            "roofline": roof,
        }
        if args.russian_roulette:
            # Russian roulette: subpath depth is unbounded (bdpt.h:68, :188); the timed frames'
            # samples that met the store / bounce bounds (must be 0) and the counting pass's maxima
            out["config"]["russian_roulette"] = "NO_RR = 0 (bdpt.h:18)"
            out["russian_roulette"] = {"capped_samples_per_step": capped, "counting_pass_spp": cnt_cfg.spp,
                                       "parked_walks_per_step": parked,
                                       # walks deeper than 512 bounces one wave held at once (max), and the
                                       # express-mode loop iterations of waves holding 1 / 2..4 / more of them
                                       "long_walks_per_wave_max_per_step": longs,
                                       "express_iters_1_2to4_more_per_step": express,
                                       "continuation": "walks past BDPT_PARK_DEPTH bounces finished by the chain kernel "
                                                       "(one wave per walk) and resume launches",
                                       "max_light_depth": cst.get("max_light_depth"),
                                       "max_eye_depth": cst.get("max_eye_depth"),
                                       "max_queries_per_sample": cst.get("max_queries"),
                                       # SIMD efficiency of the counting pass (lane iterations / 64 x wave iterations)
                                       "trav_simd_eff": round(cts["trav_lane_iters"] / max(64 * cts["trav_wave_iters"], 1), 4),
                                       "shade_simd_eff": round(cts["shade_lane_actions"] / max(64 * cts["shade_wave_actions"], 1), 4),
                                       "tail_ms": roof["tail_ms"], "kernel": cst.get("kernel")}
        if ranks:
            out["ranks"] = ranks
        if world == 1 and not args.no_cpu:
            ref_fb = None if args.no_parity else os.path.join("/tmp", f"bench_ref_fb_{os.getpid()}.f32")
            cb = cpu_baseline(args.scene, W, H, spp, rr, frame_out=ref_fb, russian_roulette=args.russian_roulette)
            out["cpu_baseline"] = {k: v for k, v in cb.items() if k != "row_stride"}
            if ref_fb is not None:
                import numpy as np

                # the same row shard on the GPU, same seeds: framebuffer parity in this run
                pbuf = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
                integ.render_device(pbuf.data_ptr(), stream, row_offset=0, row_stride=cb["row_stride"])
                torch.cuda.synchronize(dev)
                ref = np.fromfile(ref_fb, np.float32)
                os.unlink(ref_fb)
                par = frame_parity(pbuf.cpu().numpy(), ref)
                par.update({"rows": f"every {cb['row_stride']}th row from 0", "spp": spp,
                            "reference": cb["kind"], "tolerance": 1e-4})
                out["parity"] = par
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
