"""Dumps the GPU's closest hits / occlusion on the adversarial fixtures (diagnostics).
usage: python tools/adv_dump.py OUTDIR"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("bidirectional-path-tracing_amd", "scenes"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: F401,E402
import bdpt_amd  # noqa: E402
import variants  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
for scene in ("caustic", "hardlight", "synth1m"):
    g = np.load(os.path.join(REPO, "tests", "golden", f"kat_adversarial_{scene}.npz"))
    sc = bdpt_amd.Scene(variants.obj_path(scene))
    cfg = bdpt_amd.Config(camera=bdpt_amd.Camera(**variants.SCENES[scene]["camera"]), width=64, height=64, spp=1,
                          rr_depth=8)
    it = bdpt_amd.BDPTIntegrator(sc, cfg)
    it.init()
    rays, kind = g["rays"], g["kind"]
    res = {}
    for name, sel, rule in (("near", kind != 4, False), ("far", kind == 4, False), ("all", kind >= 0, False),
                            ("near_rule", kind != 4, True), ("all_rule", kind >= 0, True)):
        nrm = g["onrm"][sel] if rule else None
        h = it.intersect(rays[sel], origin_normals=nrm)
        o = it.intersect(rays[sel], occlusion=True, origin_normals=nrm)
        res[name + "_t"], res[name + "_u"], res[name + "_v"] = h["t"], h["u"], h["v"]
        res[name + "_hit"], res[name + "_tri"], res[name + "_occ"] = h["hit"], h["tri"], o["hit"]
        res[name + "_shape"], res[name + "_prim"] = h["shape_id"], h["prim_id"]
        k = g["hit"][sel] == 1
        bad = (h["t"][k].view(np.uint32) != g["t"][sel][k].view(np.uint32))
        obad = o["hit"] != g["occluded"][sel]
        print(scene, name, "hits", int(k.sum()), "t mismatches", int(bad.sum()), "per kind",
              np.bincount(kind[sel][k][bad], minlength=6).tolist(), "occlusion mismatches", int(obad.sum()),
              np.bincount(kind[sel][obad], minlength=6).tolist(), flush=True)
    np.savez_compressed(os.path.join(out, f"adv_{scene}.npz"), **res)
