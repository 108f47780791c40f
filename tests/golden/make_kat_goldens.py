"""Per-function known-answer fixtures from the UNMODIFIED reference.

Run in the development container (needs oracle/_ref/ref_bdpt, built from
/root/reference by oracle/ref/Makefile):
    python tests/golden/make_kat_goldens.py

Each fixture holds seeded inputs and the reference's own outputs for one piece
of the BDPT path (ref_bdpt kat / sample_state, oracle/ref/ref_driver.cpp):
  kat_bsdf_<scene>.npz      BSDF::eval / pdf / sample (core.h:308-310) of every material
  kat_fresnel.npz           GlassBSDF::FresnelDielectric (glass.h:40-53)
  kat_triangle.npz          rayTriangleIntersect (core.h:379-400)
  kat_intersect_<scene>.npz AcceleratorBVH::intersect + the any-hit query (accel.h:125-172, bvh.h:259-352)
  kat_splat.npz             BDPTIntegrator::splatToImagePlane (bdpt.h:485-496)
  kat_adversarial_<scene>.npz  AcceleratorBVH::intersect + the any-hit query on rays where the
                            product traversal's exactness argument is thinnest (grazing, ties,
                            surface origins, origins beyond 100 scene diagonals)
  kat_sampler_<integ>.npz   Integrator::render(ray, sampler) from arbitrary std::mt19937 states
                            (integrator.h:31; bdpt.h:219, path.h:235, direct.h:449)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "scenes"))
import variants  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "ref_bdpt")
TMP = tempfile.mkdtemp()
f32 = np.float32


def run(args):
    subprocess.run([REF, *args], check=True, capture_output=True, text=True)


def toml(scene, W=64, H=64, spp=1, rr=None, kind="bdpt", **kw):
    path = os.path.join(TMP, f"{scene}_{kind}_{W}x{H}.toml")
    with open(path, "w") as f:
        if kind == "bdpt":
            f.write(variants.toml_text(scene, W, H, spp, rr))
        elif kind == "path":
            f.write(variants.path_toml_text(scene, W, H, spp, **kw))
        else:
            f.write(variants.direct_toml_text(scene, W, H, spp, **kw))
    return path


def kat(scene_toml, W, H, kind, records: np.ndarray, width: int) -> np.ndarray:
    fin, fout = os.path.join(TMP, kind + ".in"), os.path.join(TMP, kind + ".out")
    records.astype(f32).tofile(fin)
    run(["kat", scene_toml, str(W), str(H), kind, fin, fout])
    return np.fromfile(fout, f32).reshape(-1, width)


def unit(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(f32)


def directions(rng, n):
    """Local-frame directions: mostly upper hemisphere, some lower, some grazing."""
    d = unit(rng, n)
    up = rng.random(n) < 0.7
    d[up, 2] = np.abs(d[up, 2])
    g = rng.random(n) < 0.1  # grazing
    d[g, 2] = (rng.random(g.sum()) * 1e-3 * np.sign(rng.random(g.sum()) - 0.3)).astype(f32)
    d[g] /= np.linalg.norm(d[g], axis=1, keepdims=True)
    return d.astype(f32)


def bsdf_fixture(scene, n_per=800, seed=1):
    rng = np.random.default_rng(seed)
    t = toml(scene)
    sys.path.insert(0, os.path.join(REPO, "bidirectional-path-tracing_amd"))
    import bdpt_amd  # host-only scene ingest: the material count

    nmat = bdpt_amd.Scene(variants.obj_path(scene)).info()["materials"]
    mats, recs = [], []
    for m in range(nmat):
        wo, wi = directions(rng, n_per), directions(rng, n_per)
        u = rng.random((n_per, 2)).astype(f32)
        u[:8] = np.array([[0, 0], [0.5, 0.5], [0.999999, 0.999999], [1e-7, 0.3], [0.3, 1e-7], [0.25, 0.75],
                          [0.9, 0.1], [0.1, 0.9]], f32)
        recs.append(np.concatenate([np.full((n_per, 1), m, np.int32).view(f32), wo, wi, u], axis=1))
        mats.append(m)
    rec = np.concatenate(recs)
    out = kat(t, 64, 64, "bsdf", rec, 14)
    np.savez_compressed(os.path.join(HERE, f"kat_bsdf_{scene}.npz"), mat=rec[:, 0].view(np.int32), wo=rec[:, 1:4],
                        wi=rec[:, 4:7], u=rec[:, 7:9], eval=out[:, 0:3], pdf=out[:, 3], sample_f=out[:, 4:7],
                        sample_wi=out[:, 7:10], sample_pdf=out[:, 10], type=out[:, 11].view(np.int32),
                        null=out[:, 13])
    print("bsdf", scene, rec.shape[0], "records,", len(mats), "materials")


def fresnel_fixture(n=6000, seed=2):
    rng = np.random.default_rng(seed)
    eta = np.where(rng.random(n)[:, None] < 0.5, [[1.0, 1.5]], [[1.5, 1.0]]).astype(f32)
    cos_i = rng.random(n).astype(f32)
    cos_i[:6] = [0, 1, 1e-6, 0.5, 0.7453560, 0.7453559]  # around the critical angle from inside
    e = eta[:, 0] / eta[:, 1]
    sin2_t = e * e * np.maximum(0, 1 - cos_i * cos_i)
    cos_t = np.sqrt(np.maximum(0, 1 - sin2_t)).astype(f32)
    cos_t = np.where(rng.random(n) < 0.1, rng.random(n), cos_t).astype(f32)
    rec = np.concatenate([eta, cos_i[:, None], cos_t[:, None]], axis=1).astype(f32)
    out = kat(toml("caustic"), 64, 64, "fresnel", rec, 1)[:, 0]
    np.savez_compressed(os.path.join(HERE, "kat_fresnel.npz"), inp=rec, out=out)
    print("fresnel", n)


def triangle_fixture(n=10000, seed=3):
    rng = np.random.default_rng(seed)
    v = (rng.normal(size=(n, 9)) * rng.choice([0.01, 1.0, 100.0], size=(n, 1))).astype(f32)
    o = (rng.normal(size=(n, 3)) * 3).astype(f32)
    b = rng.random((n, 3))
    b[: n // 4] = np.stack([rng.random(n // 4) * 1.2 - 0.1, rng.random(n // 4) * 1.2 - 0.1,
                            np.zeros(n // 4)], 1)  # near and across the edges
    b[:, 2] = 1 - b[:, 0] - b[:, 1]
    target = b[:, 2:3] * v[:, 0:3] + b[:, 0:1] * v[:, 3:6] + b[:, 1:2] * v[:, 6:9]
    d = target - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    par = rng.random(n) < 0.05  # rays parallel to the triangle plane (|det| < 1e-8)
    e1, e2 = v[par, 3:6] - v[par, 0:3], v[par, 6:9] - v[par, 0:3]
    d[par] = e1 / np.linalg.norm(e1, axis=1, keepdims=True) + 0 * e2
    rays = np.concatenate([o, d.astype(f32), np.full((n, 1), 1e-8, f32), np.full((n, 1), 3.4e38, f32)], 1)
    rec = np.concatenate([rays, v], 1).astype(f32)
    out = kat(toml("caustic"), 64, 64, "tri", rec, 4)
    np.savez_compressed(os.path.join(HERE, "kat_triangle.npz"), rays=rec[:, :8], verts=rec[:, 8:], out=out)
    print("triangle", n, "hits", int(out[:, 0].sum()))


def scene_rays(rng, scene, n):
    """Camera rays, rays from inside the box in every direction (incl. axis-parallel),
    and shadow-ray segments between points inside the box."""
    eye = np.array(variants.SCENES[scene]["camera"]["eye"], f32)
    k = n // 4
    lo, hi = np.array([-1.0, 0.0, -1.0]), np.array([1.0, 1.6, 1.0])
    # 1: camera rays toward the box (min_t 1, max_t 1000: renderer.cpp:192)
    tgt = lo + rng.random((k, 3)) * (hi - lo)
    d = tgt - eye
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r1 = np.concatenate([np.repeat(eye[None], k, 0), d, np.ones((k, 1)), np.full((k, 1), 1000.0)], 1)
    # 2: from inside the box, random directions (Epsilon / FLT_MAX, ContinuePathRandomWalk)
    o = lo + rng.random((k, 3)) * (hi - lo)
    d = unit(rng, k)
    r2 = np.concatenate([o, d, np.full((k, 1), 1e-8), np.full((k, 1), 3.402823466e38)], 1)
    # 3: axis-parallel directions (zero reciprocal components: the exact binary-tree path)
    o = lo + rng.random((k, 3)) * (hi - lo)
    d = np.zeros((k, 3))
    d[np.arange(k), rng.integers(0, 3, k)] = rng.choice([-1.0, 1.0], k)
    half = k // 2
    d[:half, (np.arange(half) + 1) % 3] = rng.normal(size=half)  # one zero component only
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r3 = np.concatenate([o, d, np.full((k, 1), 1e-8), np.full((k, 1), 3.402823466e38)], 1)
    # 4: shadow segments (visibilityQuery: [Epsilon, dist - 1e-5], bdpt.h:498-505)
    m = n - 3 * k
    a = lo + rng.random((m, 3)) * (hi - lo)
    b = lo + rng.random((m, 3)) * (hi - lo)
    d = b - a
    dist = np.linalg.norm(d, axis=1, keepdims=True)
    r4 = np.concatenate([a, d / dist, np.full((m, 1), 1e-8), dist - 1e-5], 1)
    return np.concatenate([r1, r2, r3, r4]).astype(f32)


def intersect_fixture(scene, n, seed):
    rng = np.random.default_rng(seed)
    rays = scene_rays(rng, scene, n)
    out = kat(toml(scene), 64, 64, "intersect", rays, 21)
    np.savez_compressed(os.path.join(HERE, f"kat_intersect_{scene}.npz"), rays=rays, out=out)
    print("intersect", scene, n, "hits", int(out[:, 0].sum()), "occluded", int(out[:, 20].sum()))


def _normalize(v):
    return (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(f32)


def _surface_points(rng, tri, idx, nrm=None):
    """Points on triangles idx as the path computes hit points (shade_hit /
    SurfaceInteraction: (v0 w + v1 u) + v2 v in float32), with a share exactly on
    edges and vertices. With nrm (the corner normals, [ntri, 9]) also the
    interpolated shading normals there (normalize((n0 w + n1 u) + n2 v), float32)."""
    n = idx.size
    u = rng.random(n).astype(f32)
    v = (rng.random(n) * (1 - u)).astype(f32)
    k = rng.random(n)
    u[k < 0.1] = 0
    v[(k >= 0.1) & (k < 0.2)] = 0
    e = (k >= 0.2) & (k < 0.3)
    v[e] = (f32(1) - u[e]).astype(f32)
    c = (k >= 0.3) & (k < 0.35)
    u[c], v[c] = 0, 0
    w = (f32(1) - u - v).astype(f32)
    v0, v1, v2 = tri[idx, 0:3], tri[idx, 3:6], tri[idx, 6:9]
    p = ((v0 * w[:, None] + v1 * u[:, None]) + v2 * v[:, None]).astype(f32)
    if nrm is None:
        return p
    n0, n1, n2 = nrm[idx, 0:3], nrm[idx, 3:6], nrm[idx, 6:9]
    sn = ((n0 * w[:, None] + n1 * u[:, None]) + n2 * v[:, None]).astype(f32)
    sn = (sn / np.sqrt(np.sum(sn.astype(f32) * sn, 1, keepdims=True, dtype=f32))).astype(f32)
    return p, sn


def adversarial_rays(scene, n, seed):
    """Rays chosen where the product traversal's exactness argument is thinnest
    (DESIGN.md §2 items 5-6): the computed hit of Moller-Trumbore near |det| = 1e-8,
    ties between triangles sharing an edge or a vertex, origins on surfaces, and
    origins beyond 100 scene diagonals, and (kinds 6, 7) grazing rays leaving the
    curved mesh, whose interpolated shading normal is not the triangle's plane
    normal. Returns (rays [n', 8] float32, kind [n'], the geometric normal of the
    triangle a ray leaves [n', 3] (0 for camera / free / far origins), that
    triangle [n'] (-1: none) and the shading normal the path holds there [n', 3])."""
    sys.path.insert(0, os.path.join(REPO, "bidirectional-path-tracing_amd"))
    import bdpt_amd

    rng = np.random.default_rng(seed)
    tf, ti, nf, _ = bdpt_amd.Scene(variants.obj_path(scene)).export()
    tri = tf[:, :9].astype(f32)
    cnrm = tf[:, 9:18].astype(f32)
    e1, e2 = tri[:, 3:6] - tri[:, 0:3], tri[:, 6:9] - tri[:, 0:3]
    cr = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    area = 0.5 * np.linalg.norm(cr, axis=1)
    ok = area > 0
    ng = np.zeros_like(cr)
    ng[ok] = cr[ok] / np.linalg.norm(cr[ok], axis=1, keepdims=True)
    lo, hi = nf[0, :3].astype(np.float64), nf[0, 3:].astype(np.float64)
    diag = float(np.linalg.norm(hi - lo))
    centre = (lo + hi) / 2
    big = np.argsort(-area)[:64]  # walls, floor, ceiling, box faces, light
    shapes, counts = np.unique(ti[:, 0], return_counts=True)
    curved = np.flatnonzero(ti[:, 0] == shapes[np.argmax(counts)])  # the tessellated sphere(s)
    FLT_MAX = 3.402823466e38
    k = n // 6
    out, kind, onrm, otri, osn = [], [], [], [], []

    def add(o, d, mn, mx, tag, nrm=None, tri_idx=None, sn=None):
        ok = np.isfinite(o).all(1) & np.isfinite(d).all(1)  # degenerate triangles of a generated mesh
        if not ok.all():
            o, d = o[ok], d[ok]
            mn, mx = (mn if np.isscalar(mn) else mn[ok]), (mx if np.isscalar(mx) else mx[ok])
            nrm, tri_idx, sn = (None if x is None else np.asarray(x)[ok] for x in (nrm, tri_idx, sn))
        m = o.shape[0]
        onrm.append(np.zeros((m, 3), f32) if nrm is None else np.asarray(nrm, f32))
        otri.append(np.full(m, -1, np.int32) if tri_idx is None else np.asarray(tri_idx, np.int32))
        osn.append(np.zeros((m, 3), f32) if sn is None else np.asarray(sn, f32))
        out.append(np.concatenate([o, _normalize(d), np.broadcast_to(np.float32(mn), (m, 1)) if np.isscalar(mn)
                                   else mn[:, None], np.broadcast_to(np.float32(mx), (m, 1)) if np.isscalar(mx)
                                   else mx[:, None]], 1).astype(f32))
        kind.append(np.full(m, tag, np.int32))

    # 0: grazing continuation rays from points on the large triangles, |sin| from 0 to 1e-2
    idx = rng.choice(big, k)
    o, sn = _surface_points(rng, tri, idx, cnrm)
    t1 = _normalize(e1[idx])
    t2 = _normalize(np.cross(ng[idx], t1))
    phi = rng.random(k) * 2 * np.pi
    delta = rng.choice([0.0, 1e-9, 3e-9, 1e-8, 3e-8, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 0.015, 0.02, 0.03, 0.05],
                       k) * rng.choice([-1, 1], k)
    d = t1 * np.cos(phi)[:, None] + t2 * np.sin(phi)[:, None] + ng[idx] * delta[:, None]
    h = rng.choice([0.0, 0.0, 1e-7, -1e-7, 1e-6, -1e-6, 1e-5, 1e-4], k)
    add((o + ng[idx] * h[:, None]).astype(f32), d, 1e-8, FLT_MAX, 0, ng[idx], idx, sn)
    # 1: grazing shadow segments between two points of the same large triangle (visibilityQuery)
    idx = rng.choice(big, k)
    (a, sn), b = _surface_points(rng, tri, idx, cnrm), _surface_points(rng, tri, idx)
    lift = rng.choice([0.0, 1e-7, 1e-5, 1e-3], k)[:, None] * ng[idx]
    a, b = (a + lift).astype(f32), (b + lift).astype(f32)
    dd = (b - a).astype(f32)
    dist = np.sqrt((dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]) + dd[:, 2] * dd[:, 2]).astype(f32)
    keep = dist > 1e-4
    add(a[keep], dd[keep], 1e-8, (dist[keep] - f32(1e-5)).astype(f32), 1, ng[idx][keep], idx[keep], sn[keep])
    # 2: rays through the curved mesh's vertices and edges (ties between neighbours, silhouettes)
    idx = rng.choice(curved, k)
    w = rng.choice(4, k)
    tgt = np.where((w == 0)[:, None], tri[idx, 0:3], np.where((w == 1)[:, None], (tri[idx, 0:3] + tri[idx, 3:6]) / 2,
                   _surface_points(rng, tri, idx)))
    eye = np.array(variants.SCENES[scene]["camera"]["eye"], np.float64)
    inner = lo + rng.random((k, 3)) * (hi - lo)
    o = np.where((rng.random(k) < 0.5)[:, None], eye, inner).astype(f32)
    add(o, tgt - o, 1e-8, FLT_MAX, 2)
    # 3: continuation rays from surface points of any triangle, both hemispheres, near-tangent included
    idx = rng.integers(0, tri.shape[0], k)
    o, sn = _surface_points(rng, tri, idx, cnrm)
    d = rng.normal(size=(k, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    flat = rng.random(k) < 0.3
    d[flat] -= ng[idx][flat] * np.sum(d[flat] * ng[idx][flat], 1, keepdims=True) * (1 - rng.choice(
        [1e-6, 1e-4, 1e-2], flat.sum()))[:, None]
    add(o, d, 1e-8, FLT_MAX, 3, ng[idx], idx, sn)
    # 4: origins 100 - 10000 scene diagonals away, aimed at surface points (the slack-test regime)
    dirn = rng.normal(size=(k, 3))
    dirn /= np.linalg.norm(dirn, axis=1, keepdims=True)
    far = diag * np.exp(rng.uniform(np.log(100.0), np.log(10000.0), k))
    o = (centre + dirn * far[:, None]).astype(f32)
    tgt = _surface_points(rng, tri, rng.integers(0, tri.shape[0], k))
    mx = np.where(rng.random(k) < 0.5, FLT_MAX, far * 1.5).astype(f32)
    add(o, tgt - o, np.where(rng.random(k) < 0.5, 1.0, 1e-8).astype(f32), mx, 4)
    # 5: shadow segments between surface points of any two triangles
    m = n - 5 * k
    ia = rng.integers(0, tri.shape[0], m)
    a, sn = _surface_points(rng, tri, ia, cnrm)
    b = _surface_points(rng, tri, rng.integers(0, tri.shape[0], m))
    dd = (b - a).astype(f32)
    dist = np.sqrt((dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]) + dd[:, 2] * dd[:, 2]).astype(f32)
    keep = dist > 1e-4
    add(a[keep], dd[keep], 1e-8, (dist[keep] - f32(1e-5)).astype(f32), 5, ng[ia][keep], ia[keep], sn[keep])
    # 6: grazing continuation rays leaving the curved mesh: |cos| to the
    # triangle's plane from 0 to 0.1, while the interpolated shading normal the path
    # tests against (cull_near_for) is tilted from that plane's normal
    idx = rng.choice(curved, k)
    o, sn = _surface_points(rng, tri, idx, cnrm)
    t1 = _normalize(e1[idx])
    t2 = _normalize(np.cross(ng[idx], t1))
    phi = rng.random(k) * 2 * np.pi
    delta = rng.choice([0.0, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 3e-3, 1e-2, 0.015, 0.019, 0.021, 0.03, 0.05, 0.1],
                       k) * rng.choice([-1, 1], k)
    d = t1 * np.cos(phi)[:, None] + t2 * np.sin(phi)[:, None] + ng[idx] * delta[:, None]
    h = rng.choice([0.0, 0.0, 1e-7, -1e-7, 1e-6, -1e-6], k)
    add((o + ng[idx] * h[:, None]).astype(f32), d, 1e-8, FLT_MAX, 6, ng[idx], idx, sn)
    # 7: grazing shadow segments from the curved mesh along its triangles' planes
    idx = rng.choice(curved, k)
    a, sn = _surface_points(rng, tri, idx, cnrm)
    t1 = _normalize(e1[idx])
    t2 = _normalize(np.cross(ng[idx], t1))
    phi = rng.random(k) * 2 * np.pi
    delta = rng.choice([0.0, 1e-6, 1e-4, 1e-2, 0.019, 0.03, 0.1], k) * rng.choice([-1, 1], k)
    d = _normalize(t1 * np.cos(phi)[:, None] + t2 * np.sin(phi)[:, None] + ng[idx] * delta[:, None])
    ln = np.exp(rng.uniform(np.log(1e-3), np.log(2.0), k))
    b = (a + d * ln[:, None]).astype(f32)
    dd = (b - a).astype(f32)
    dist = np.sqrt((dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]) + dd[:, 2] * dd[:, 2]).astype(f32)
    keep = dist > 1e-4
    add(a[keep], dd[keep], 1e-8, (dist[keep] - f32(1e-5)).astype(f32), 7, ng[idx][keep], idx[keep], sn[keep])
    return (np.concatenate(out), np.concatenate(kind), np.concatenate(onrm), np.concatenate(otri),
            np.concatenate(osn))


def adversarial_fixture(scene, n, seed):
    rays, kind, onrm, otri, osn = adversarial_rays(scene, n, seed)
    out = kat(toml(scene), 64, 64, "intersect", rays, 21)
    np.savez_compressed(os.path.join(HERE, f"kat_adversarial_{scene}.npz"), rays=rays, kind=kind, onrm=onrm,
                        otri=otri, osn=osn,
                        hit=out[:, 0].astype(np.int8), t=out[:, 1], u=out[:, 2], v=out[:, 3],
                        shape=out[:, 4].view(np.int32), prim=out[:, 5].view(np.int32),
                        occluded=out[:, 20].astype(np.int8))
    print("adversarial", scene, rays.shape[0], "rays; hits", int(out[:, 0].sum()), "occluded",
          int(out[:, 20].sum()), "per kind", np.bincount(kind))


def splat_fixture(seed=5):
    rng = np.random.default_rng(seed)
    res = {}
    for (W, H) in [(64, 64), (512, 512), (80, 48)]:
        n = 4000
        p = (np.array([-1.2, -0.2, -1.2]) + rng.random((n, 3)) * np.array([2.4, 2.0, 6.0])).astype(f32)
        out = kat(toml("caustic", W, H), W, H, "splat", p, 2).view(np.int32)
        res[f"p_{W}x{H}"] = p
        res[f"xy_{W}x{H}"] = out
    np.savez_compressed(os.path.join(HERE, "kat_splat.npz"), **res)
    print("splat")


def states(rng, n):
    """std::mt19937 states: seeded and advanced (across the first twist, the lazy
    window's end, a whole state) and arbitrary words with arbitrary positions."""
    out = []
    for i in range(n):
        if i < n * 3 // 4:
            rs = np.random.RandomState(int(rng.integers(0, 2**32)))  # init_genrand == std::mt19937(seed)
            skip = int(rng.choice([0, 1, 2, 100, 225, 226, 227, 400, 623, 624, 625, 1000, 5000]))
            if skip:
                rs.randint(0, 2**32, size=skip, dtype=np.uint32)
            _, key, pos = rs.get_state()[:3]
            out.append(np.concatenate([key.astype(np.uint32), [np.uint32(pos)]]))
        else:
            key = rng.integers(0, 2**32, size=624, dtype=np.uint64).astype(np.uint32)
            out.append(np.concatenate([key, [np.uint32(rng.integers(0, 625))]]))
    return np.array(out, np.uint32)


def sampler_fixture(name, scene, toml_path, W, H, spp, rr, n, seed):
    rng = np.random.default_rng(seed)
    eye = np.array(variants.SCENES[scene]["camera"]["eye"], f32)
    tgt = np.array([-1.0, 0.0, -1.0]) + rng.random((n, 3)) * np.array([2.0, 1.6, 2.0])
    d = tgt - eye
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([np.repeat(eye[None], n, 0), d, np.ones((n, 1)), np.full((n, 1), 1000.0)], 1).astype(f32)
    st = states(rng, n)
    rec = np.concatenate([rays, st.view(f32)], 1)
    fin, fout = os.path.join(TMP, name + ".in"), os.path.join(TMP, name + ".out")
    rec.astype(f32).tofile(fin)
    # rr only for the BDPT scenes: ref_driver's setup() writes it to Config's
    # pt.rrDepth, which shares a union with di.bsdfSamples (core.h:201-240)
    run(["sample_state", toml_path, str(W), str(H), str(spp), str(rr if "bdpt" in name else 0), fin, fout, "-"])
    out = np.fromfile(fout, f32).reshape(n, 3 + 625 + 1 + 64)
    np.savez_compressed(os.path.join(HERE, f"kat_sampler_{name}.npz"), rays=rays, state_in=st, Li=out[:, :3],
                        state_out=out[:, 3:628].view(np.uint32), nsplat=out[:, 628].view(np.int32),
                        splats=out[:, 629:].reshape(n, 16, 4), width=W, height=H, spp=spp, rr=rr)
    print("sampler", name, n, "records; splat counts", np.bincount(out[:, 628].view(np.int32)))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "adversarial":  # only these fixtures
        for i, (sc, n) in enumerate([("caustic", 48000), ("hardlight", 48000), ("synth1m", 30000)]):
            adversarial_fixture(sc, n, seed=40 + i)
        return
    if not os.path.exists(REF):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle", "ref")], check=True)
    for i, sc in enumerate(["caustic", "hardlight", "hardlight_mirror", "hardlight_phong", "cbox_low"]):
        bsdf_fixture(sc, seed=10 + i)
    fresnel_fixture()
    triangle_fixture()
    for i, (sc, n) in enumerate([("caustic", 12000), ("hardlight", 8000), ("cbox_low", 4000)]):
        intersect_fixture(sc, n, seed=20 + i)
    splat_fixture()
    for i, (sc, n) in enumerate([("caustic", 48000), ("hardlight", 48000), ("synth1m", 30000)]):
        adversarial_fixture(sc, n, seed=40 + i)
    sampler_fixture("bdpt_caustic", "caustic", toml("caustic", 64, 64, 16, 8), 64, 64, 16, 8, 160, 30)
    sampler_fixture("bdpt_hardlight_rr12", "hardlight", toml("hardlight", 64, 64, 16, 12), 64, 64, 16, 12, 100, 31)
    sampler_fixture("path_caustic", "caustic", toml("caustic", 64, 64, 16, kind="path"), 64, 64, 16, 5, 80, 32)
    sampler_fixture("direct_hardlight", "hardlight",
                    toml("hardlight", 64, 64, 16, kind="direct", strategy="mis", emitter_samples=2, bsdf_samples=2),
                    64, 64, 16, 5, 80, 33)


if __name__ == "__main__":
    main()
