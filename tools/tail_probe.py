"""The drain phase of a row shard, from a BDPT_TAIL_PROBE=1 variant library
(tools/build_variant.sh tailprobe -DBDPT_TAIL_PROBE=1; BDPT_AMD_LIB selects it):
per wave, the time from its first drain iteration (no sample left to claim) and
from the first iteration with at most 4 busy lanes to its end. The probe reuses
the Russian-roulette diag words (s_memrealtime ticks, 100 MHz).

    BDPT_AMD_LIB=.../libbdpt_amd_tailprobe.so python tools/tail_probe.py [scene W H spp] [N...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("bidirectional-path-tracing_amd", "scenes"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

import bdpt_amd  # noqa: E402
import variants  # noqa: E402

TICKS_PER_MS = 1.0e5


def main():
    a = sys.argv[1:]
    scene, W, H, spp = (a[0], int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else ("caustic", 512, 512, 256)
    ns = [int(x) for x in a[4:]] or [1, 8]
    sc = variants.SCENES[scene]
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**sc["camera"]), width=W, height=H, spp=spp,
                          rr_depth=sc["rr_depth"])
    integ = bdpt_amd.BDPTIntegrator(bdpt_amd.Scene(variants.obj_path(scene)), cfg, device=0)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for n in ns:
        for rep in range(2):
            fb.zero_()
            integ.render_device(fb.data_ptr(), stream, row_offset=0, row_stride=n)
            st = integ.stats()
        few_max, drain_max = st["rr_long_walks_max"], st["rr_express_iters"][0]
        few_sum, few_waves = st["rr_express_iters"][1], st["rr_express_iters"][2]
        print(f"row_stride {n}: kernel {st['kernel_ms']:.2f} ms, end tail {st.get('tail_ms', 0.0):.2f} ms, "
              f"longest drain {drain_max / TICKS_PER_MS:.3f} ms, longest <=4-lane drain {few_max / TICKS_PER_MS:.3f} ms, "
              f"mean <=4-lane drain {few_sum / max(few_waves, 1) / TICKS_PER_MS:.3f} ms over {few_waves} waves",
              flush=True)


if __name__ == "__main__":
    main()
