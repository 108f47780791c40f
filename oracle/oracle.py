"""TEST INFRASTRUCTURE ONLY: ctypes binding for the C oracle (oracle/src).

Used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Never imported by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_bdpt")


class Params(ctypes.Structure):
    _fields_ = [
        ("eye", ctypes.c_float * 3),
        ("at", ctypes.c_float * 3),
        ("up", ctypes.c_float * 3),
        ("fov", ctypes.c_float),
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("spp", ctypes.c_int),
        ("rr_depth", ctypes.c_int),
        ("strategy", ctypes.c_int),  # 0 BDPT, 1 LIGHT_TRACING, 2 PATH_TRACING (bdpt.h:16-17)
        ("integrator", ctypes.c_int),  # 0 BDPTIntegrator, 1 PathTracerIntegrator (path.h)
        ("pt_explicit", ctypes.c_int),
        ("pt_max_depth", ctypes.c_int),
        ("pt_rr_depth", ctypes.c_int),
        ("pt_rr_prob", ctypes.c_float),
        ("pt_emitter_samples", ctypes.c_int),
        ("pt_bsdf_samples", ctypes.c_int),
        ("di_strategy", ctypes.c_int),  # DirectIntegrator samplingStrategy (DIRECT_STRATEGIES)
        ("di_emitter_samples", ctypes.c_int),
        ("di_bsdf_samples", ctypes.c_int),
        ("seed_base", ctypes.c_uint32),
        ("russian_roulette", ctypes.c_int),  # 0: NO_RR = 1 (bdpt.h:18, as shipped); 1: its NO_RR = 0 branch
    ]


DIRECT_STRATEGIES = {"area": 1, "solidAngle": 2, "cosineHemisphere": 3, "bsdf": 4, "mis": 5}


def make_direct_params(cam: dict, width: int, height: int, spp: int, strategy: str = "mis", emitter_samples: int = 1,
                       bsdf_samples: int = 1) -> "Params":
    """Params for DirectIntegrator (direct.h); defaults of main.cpp:90-92 except the strategy."""
    p = make_params(cam, width, height, spp, 1)
    p.integrator = 2
    p.di_strategy = DIRECT_STRATEGIES[strategy]
    p.di_emitter_samples, p.di_bsdf_samples = emitter_samples, bsdf_samples
    return p


# [renderer] defaults of a type = "path" scene (main.cpp:96-101)
PATH_DEFAULTS = dict(explicit=True, max_depth=-1, rr_depth=5, rr_prob=0.95, emitter_samples=1, bsdf_samples=0)


def make_path_params(cam: dict, width: int, height: int, spp: int, **path) -> "Params":
    """Params for PathTracerIntegrator (path.h) with PATH_DEFAULTS overridden by `path`."""
    s = dict(PATH_DEFAULTS, **path)
    p = make_params(cam, width, height, spp, s["rr_depth"])
    p.integrator = 1
    p.pt_explicit, p.pt_max_depth, p.pt_rr_depth = int(s["explicit"]), s["max_depth"], s["rr_depth"]
    p.pt_rr_prob, p.pt_emitter_samples, p.pt_bsdf_samples = s["rr_prob"], s["emitter_samples"], s["bsdf_samples"]
    return p


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.tro_scene_load.restype = ctypes.c_void_p
        L.tro_scene_load.argtypes = [ctypes.c_char_p]
        L.tro_scene_free.argtypes = [ctypes.c_void_p]
        L.tro_last_error.restype = ctypes.c_char_p
        L.tro_scene_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.tro_scene_dump.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 4
        L.tro_camera.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p]
        L.tro_render_row_samples.restype = ctypes.c_int64
        L.tro_render_row_samples.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int64, ctypes.c_int64]
        L.tro_render.restype = ctypes.c_int64
        L.tro_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.tro_sample.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
        L.tro_counters.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        L.tro_rr_overflow.restype = ctypes.c_int64
        L.tro_rr_overflow.argtypes = [ctypes.c_int]
        L.tro_walk_stats.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        L.tro_mt19937_nth.restype = ctypes.c_uint32
        L.tro_mt19937_nth.argtypes = [ctypes.c_uint32, ctypes.c_int]
        L.tro_sampler_nth.restype = ctypes.c_float
        L.tro_sampler_nth.argtypes = [ctypes.c_uint32, ctypes.c_int]
        for fn in ("tro_sinf", "tro_cosf"):
            getattr(L, fn).restype = ctypes.c_float
            getattr(L, fn).argtypes = [ctypes.c_float]
        L.tro_powf.restype = ctypes.c_float
        L.tro_powf.argtypes = [ctypes.c_float, ctypes.c_float]
        _lib = L
    return _lib


def make_params(cam: dict, width: int, height: int, spp: int, rr_depth: int, strategy: int = 0,
                russian_roulette: int = 0) -> Params:
    p = Params()
    p.eye[:] = [float(x) for x in cam["eye"]]
    p.at[:] = [float(x) for x in cam["at"]]
    p.up[:] = [float(x) for x in cam["up"]]
    p.fov = float(cam["fov"])
    p.width, p.height, p.spp, p.rr_depth = width, height, spp, rr_depth
    p.strategy = strategy
    p.russian_roulette = russian_roulette
    p.seed_base = 260450963  # the reference's Sampler seed (renderer.cpp:155)
    return p


class Scene:
    def __init__(self, obj_path: str):
        L = lib()
        self._h = L.tro_scene_load(obj_path.encode())
        if not self._h:
            raise RuntimeError("oracle scene load failed: " + L.tro_last_error().decode())

    def __del__(self):
        if getattr(self, "_h", None):
            lib().tro_scene_free(self._h)
            self._h = None

    def stats(self) -> dict:
        out = (ctypes.c_int64 * 6)()
        lib().tro_scene_stats(self._h, out)
        return dict(zip(["triangles", "nodes", "shapes", "materials", "emitters", "max_depth"], list(out)))

    def dump(self):
        st = self.stats()
        nt, nn = st["triangles"], st["nodes"]
        tf = np.zeros((nt, 18), np.float32)
        ti = np.zeros((nt, 3), np.int32)
        nf = np.zeros((nn, 6), np.float32)
        nu = np.zeros((nn, 3), np.uint32)
        lib().tro_scene_dump(self._h, tf.ctypes.data, ti.ctypes.data, nf.ctypes.data, nu.ctypes.data)
        return tf, ti, nf, nu

    def render(self, p: Params, threads: int = 1, rows: list[int] | None = None) -> tuple[np.ndarray, int]:
        """Returns (framebuffer [H*W*3] float32, samples). threads > 1 splits
        rows round-robin over threads with private framebuffers summed at the
        end (same per-sample work; splat sums reassociate)."""
        L = lib()
        W, H = p.width, p.height
        if rows is None:
            rows = list(range(H))
        if threads <= 1:
            fb = np.zeros(W * H * 3, np.float32)
            n = 0
            # contiguous single-threaded pass in pixel order == reference order
            if rows == list(range(H)):
                n = L.tro_render(self._h, ctypes.byref(p), fb.ctypes.data, 0, H, 1)
            else:
                for r in rows:
                    n += L.tro_render(self._h, ctypes.byref(p), fb.ctypes.data, r, r + 1, 1)
            return fb, n
        fbs = [np.zeros(W * H * 3, np.float32) for _ in range(threads)]
        counts = [0] * threads

        def work(t):
            for r in rows[t::threads]:
                counts[t] += L.tro_render(self._h, ctypes.byref(p), fbs[t].ctypes.data, r, r + 1, 1)

        ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        fb = fbs[0]
        for f in fbs[1:]:
            fb += f
        return fb, sum(counts)

    def render_row_samples(self, p: Params, row: int, s_lo: int, s_hi: int, fb: np.ndarray | None = None) -> np.ndarray:
        """Samples [s_lo, s_hi) of one row (s = j * spp + k), each added as Li / spp,
        into fb (a new zero framebuffer by default). A debugging aid (tools/rr_find.py)."""
        if fb is None:
            fb = np.zeros(p.width * p.height * 3, np.float32)
        lib().tro_render_row_samples(self._h, ctypes.byref(p), fb.ctypes.data, row, s_lo, s_hi)
        return fb

    def sample(self, p: Params, pixel: int, k: int):
        fb = np.zeros(p.width * p.height * 3, np.float32)
        Li = np.zeros(3, np.float32)
        lib().tro_sample(self._h, ctypes.byref(p), pixel, k, Li.ctypes.data, fb.ctypes.data)
        return Li, fb


def camera(p: Params) -> np.ndarray:
    out = np.zeros(72, np.float32)
    lib().tro_camera(ctypes.byref(p), out.ctypes.data)
    return out


def walk_stats(reset: bool = True) -> dict:
    """Deepest light / eye subpath and most stored light vertices of one sample (this thread)."""
    out = (ctypes.c_int64 * 3)()
    lib().tro_walk_stats(out, 1 if reset else 0)
    return dict(zip(["max_light_depth", "max_eye_depth", "max_light_verts"], list(out)))


def counters(reset: bool = True) -> dict:
    out = (ctypes.c_int64 * 9)()
    lib().tro_counters(out, 1 if reset else 0)
    keys = ["closest_rays", "shadow_rays", "interior_visits", "tri_tests", "light_verts",
            "light_vert_reads", "splats", "rng_draws", "eye_retraces"]
    return dict(zip(keys, list(out)))
