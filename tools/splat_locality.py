"""Camera-splat pixel locality (CPU, the C oracle): would a per-wave cache of
recent splat pixels aggregate the float atomics of connectToCamera? A wave runs
64-sample chunks of one pixel each (spp 256); this replays 8 consecutive chunks
at random image spots, takes each sample's splatted pixels (bdpt.h:295-371,
oracle sample()) in order, and reports the hit rate of an LRU cache of E pixels.

    python tools/splat_locality.py [scene] [trials]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "scenes")]
import oracle as O  # noqa: E402
import variants  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "caustic"
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    sc = variants.SCENES[name]
    scene = O.Scene(variants.obj_path(name))
    W = H = 512
    p = O.make_params(sc["camera"], W, H, 256, sc["rr_depth"])
    rng = np.random.default_rng(1)
    t0, res, total = time.time(), {}, 0
    for _ in range(trials):
        px0 = int(rng.integers(0, W * H - 64))
        stream = []
        for c in range(8):
            for k in range(64):
                _, fb = scene.sample(p, px0 + c, k)
                stream += [int(x) for x in np.nonzero(fb.reshape(-1, 3).any(axis=1))[0]]
        total += len(stream)
        for E in (4, 8, 16, 64, 256):
            cache, hits = [], 0
            for q in stream:
                if q in cache:
                    hits += 1
                    cache.remove(q)
                else:
                    if len(cache) >= E:
                        cache.pop(0)
                cache.append(q)
            h, n = res.get(E, (0, 0))
            res[E] = (h + hits, n + len(stream))
    print(f"{name}: splats per sample {total / (trials * 8 * 64):.3f}; LRU hit rate by entries "
          f"{ {E: round(h / n, 4) for E, (h, n) in res.items()} } ({time.time() - t0:.1f} s)")


if __name__ == "__main__":
    main()
