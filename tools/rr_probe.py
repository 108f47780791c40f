"""Russian-roulette probe (the reference's NO_RR = 0 branch): frame time, the
persistent grid's end tail, samples that met the bounds, and the counting pass's
per-sample maxima (subpath depths, queries) of one render.

    python tools/rr_probe.py [scene] [W] [H] [spp] [row_offset] [row_stride]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bidirectional-path-tracing_amd"), os.path.join(REPO, "scenes")]
import torch  # noqa: E402

import bdpt_amd  # noqa: E402
import variants  # noqa: E402

def _beat():  # a line every 30 s: one Russian-roulette frame can run for minutes
    import threading

    t0 = time.time()

    def run():
        while True:
            time.sleep(30)
            print(f"[rr_probe] running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


_beat()
a = sys.argv[1:]
name = a[0] if a else "caustic"
W, H, spp = (int(x) for x in (a[1:4] if len(a) >= 4 else (512, 512, 4)))
off, stride = (int(x) for x in (a[4:6] if len(a) >= 6 else (0, 1)))
sc = variants.SCENES[name]
cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**sc["camera"]), width=W, height=H, spp=spp, rr_depth=sc["rr_depth"],
                      russian_roulette=bdpt_amd.RR_LUMINANCE)
it = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(name)), cfg)
it.init()
passes = ((0, "render"),) if os.environ.get("RR_PROBE_NO_COUNT") else ((0, "render"), (bdpt_amd.FLAG_COUNT, "counting"))
for flags, label in passes:
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    t = time.time()
    it.render_device(fb.data_ptr(), torch.cuda.current_stream().cuda_stream, row_offset=off, row_stride=stride,
                     flags=flags)
    st = it.stats()  # waits for the kernel
    out = {"pass": label, "scene": name, "W": W, "H": H, "spp": spp, "rows": [off, stride], "samples": st["samples"],
           "kernel_ms": round(st["kernel_ms"], 3), "span_ms": round(st["span_ms"], 3),
           "tail_ms": round(st["tail_ms"], 3), "capped": st["capped_samples"],
           "parked": st.get("parked_samples"), "launches": st.get("launches"),
           "long_walks_max": st.get("rr_long_walks_max"), "express_iters_1_2to4_more": st.get("rr_express_iters"),
           "wall_s": round(time.time() - t, 3),
           # BDPT_EXPRESS_PROBE builds: express iterations with one busy lane, their clocks in the
           # cooperative walk block, and in the whole loop iteration (bdpt_stats.sched)
           "sched": st.get("sched"),
           "kernel": st["kernel"]}
    if flags:
        out.update(max_light_depth=st["max_light_depth"], max_eye_depth=st["max_eye_depth"],
                   max_queries=st["max_queries"], counters=st["counters"],
                   trav_simd_eff=round(st["counters"]["trav_lane_iters"] / max(64 * st["counters"]["trav_wave_iters"], 1), 4),
                   shade_simd_eff=round(st["counters"]["shade_lane_actions"] / max(64 * st["counters"]["shade_wave_actions"], 1), 4))
    print(json.dumps(out), flush=True)
