"""Kernel time of one rank's row shard (row_stride N) against the full frame on
one GPU: the strong-scaling tail a persistent grid pays when each of N ranks
renders 1/N of the frame (lanes idle once the shard's work counter runs out).

    python tools/shard_tail.py [scene W H spp] [N...]

Each shard is measured twice: rows claimed top to bottom, and costly rows first
(bdpt_set_row_order with the queries per row of a 4-spp counting pass of the
same shard, bdpt_amd.cost_row_order).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("bidirectional-path-tracing_amd", "scenes"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

import bdpt_amd  # noqa: E402
import variants  # noqa: E402


def main():
    a = sys.argv[1:]
    scene, W, H, spp = (a[0], int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else ("caustic", 512, 512, 256)
    ns = [int(x) for x in a[4:]] or [1, 2, 4, 8]
    sc = variants.SCENES[scene]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**sc["camera"]), width=W, height=H, spp=spp,
                          rr_depth=sc["rr_depth"])
    integ = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(scene)), cfg, device=0)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    ccfg = bdpt_amd.Config(camera=cfg.camera, width=W, height=H, spp=min(spp, 4), rr_depth=cfg.rr_depth)
    counter = bdpt_amd.BDPTIntegrator(integ.scene, ccfg, device=0)
    cfb = torch.zeros_like(fb)
    full = {}
    for n in ns:
        nrows = len(range(0, H, n))
        counter.render_device(cfb.data_ptr(), stream, row_offset=0, row_stride=n, flags=bdpt_amd.FLAG_COUNT)
        order = bdpt_amd.cost_row_order(counter.row_costs(nrows))
        for kind in ("top-down", "cost"):
            integ.set_row_order(order if kind == "cost" else None)
            ms, tails = [], []
            for rep in range(3):
                fb.zero_()
                integ.render_device(fb.data_ptr(), stream, row_offset=0, row_stride=n)
                st = integ.stats()
                ms.append(st["kernel_ms"])
                tails.append(st.get("tail_ms", 0.0))
            t = min(ms[1:])
            tail = min(tails[1:])
            if n == 1:
                full[kind] = t
            f = full.get(kind)
            ideal = f / n if f else float("nan")
            print(f"row_stride {n} ({kind} rows): kernel {t:.2f} ms, full/{n} = {ideal:.2f} ms, "
                  f"efficiency {ideal / t:.3f}, end tail {tail:.2f} ms", flush=True)
        integ.set_row_order(None)
    # Throughput form: K frames of the shard back to back with two frames in flight (two
    # contexts and streams, bench.py --pipeline 2), wall time per frame against the full
    # frame's the same way.
    ctxs = [integ, bdpt_amd.BDPTIntegrator(integ.scene, cfg, device=0)]
    fbs = [fb, torch.zeros_like(fb)]
    ss = [torch.cuda.current_stream(), torch.cuda.Stream()]
    import time
    pfull = None
    for n in ns:
        def run(k):
            for i in range(k):
                j = i % 2
                with torch.cuda.stream(ss[j]):
                    fbs[j].zero_()
                    ctxs[j].render_device(fbs[j].data_ptr(), ss[j].cuda_stream, row_offset=0, row_stride=n)
            torch.cuda.synchronize()
        K = 4 * n
        run(2)
        t0 = time.perf_counter()
        run(K)
        per = (time.perf_counter() - t0) / K * 1e3
        if n == 1:
            pfull = per
        ideal = pfull / n if pfull else float("nan")
        print(f"row_stride {n} (2 frames in flight, {K} frames): {per:.2f} ms per frame, full/{n} = {ideal:.2f} ms, "
              f"efficiency {ideal / per:.3f}", flush=True)


if __name__ == "__main__":
    main()
