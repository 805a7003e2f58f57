"""ctypes wrapper of the CPU oracle (oracle/liboracle_bre.so) — test infrastructure only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_bre.so")


def _p(a):
    return None if a is None else a.ctypes.data


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        P, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
        lib.ora_slab_pad.restype = F
        lib.ora_beam_bounds.argtypes = [I64, P, P, P, I32, P]
        lib.ora_closest_points.argtypes = [P, P, P, P, P, P]
        lib.ora_closest_points.restype = I32
        lib.ora_intersect_box.argtypes = [P, P, P, F]
        lib.ora_intersect_box.restype = I32
        lib.ora_radius_at.argtypes = [F, F, I32]
        lib.ora_radius_at.restype = F
        lib.ora_bvh_build.argtypes = [I64, P, P, P, P, I32]
        lib.ora_bvh_build.restype = P
        lib.ora_bvh_node_count.argtypes = [P]
        lib.ora_bvh_node_count.restype = I64
        lib.ora_bvh_max_leaf.argtypes = [P]
        lib.ora_bvh_max_leaf.restype = I32
        lib.ora_bvh_free.argtypes = [P]
        lib.ora_gather.argtypes = [P, I64, P, P, P, P, P, F, P, P, P, P, P, I32, I64]
        lib.ora_gather_skip.argtypes = [P, I64, P, P, P, P, F, P, P, P, P, I32]
        lib.ora_gather_bruteforce.argtypes = [I64, P, P, P, P, I32, I64, P, P, P, P, F, P, P, P, I32, P]
        U64 = ctypes.c_uint64
        lib.ora_trace_photons.argtypes = [P, I64, I32, I32, F, I64, P, P, P, P, P]
        lib.ora_trace_photons.restype = I64
        lib.ora_pcg32.argtypes = [U64, I64, I32, P]
        lib.ora_pcg32_srandom.argtypes = [U64, U64, I64, P]
        lib.ora_hg_sample.argtypes = [F, I64, P, P, P, P]
        lib.ora_hg_p.argtypes = [F, I64, P, P, P]
        lib.ora_homogeneous_tr.argtypes = [P, P, I64, P, P, P]
        lib.ora_cosine_hemisphere.argtypes = [I64, P, P]
        lib.ora_fmath.argtypes = [I32, I64, P, P]
        lib.ora_camera_pass.argtypes = [P, I32, I32, I32, I32, I32, I32, I64, P, P, P, P, P, P, P]
        lib.ora_camera_pass.restype = I64
        lib.ora_halton.argtypes = [I32, I32, I64, P, P, P, P, P]
        lib.ora_radical_inverse.argtypes = [I32, U64]
        lib.ora_radical_inverse.restype = F
        lib.ora_scrambled_radical_inverse.argtypes = [I32, U64, P]
        lib.ora_scrambled_radical_inverse.restype = F
        lib.ora_shuffle.argtypes = [U64, I32, P]
        lib.ora_grid_density.argtypes = [P, I64, P, P]
        lib.ora_set_libm.argtypes = [I32]
        lib.ora_grid_eval.argtypes = [P, I32, I64, P, P, P, U64, P, P]
        lib.ora_tri_hits.argtypes = [P, I64, P, P, P]
        lib.ora_tri_sample.argtypes = [P, I32, I64, P, P, P, P]
        lib.ora_distribution1d.argtypes = [P, I32, I64, P, P, P, P, P]
        lib.ora_distribution1d_continuous.argtypes = [P, I32, I64, P, P, P, P]
        lib.ora_pcg32_default.argtypes = [I64, P]
        lib.ora_next_float.argtypes = [I32, I64, P, P]
        lib.ora_float_bits.argtypes = [I64, P, P]
        lib.ora_find_interval.argtypes = [P, I32, I64, P, P]
        lib.ora_tri_reintersect.argtypes = [I32, I32, P, P]
        lib.ora_scene_intersect.argtypes = [P, I64, P, P, I32, P, P, P]
        lib.ora_tri_reintersect.restype = I64

    # -- primitives --
    def set_libm(self, on: bool):
        """The host libm's std::exp / std::log / std::sin / std::cos (as pbrt calls them) instead of the
        restatement the GPU shares (include/bre_fmath.h; since round 6 the same bits for every input)."""
        self.lib.ora_set_libm(int(bool(on)))

    def slab_pad(self) -> float:
        return float(self.lib.ora_slab_pad())

    def beam_bounds(self, start, end, radius, sqrt_mode=0):
        start, end, radius = (np.ascontiguousarray(x, np.float32) for x in (start, end, radius))
        n = radius.shape[0]
        box = np.zeros((n, 6), np.float32)
        self.lib.ora_beam_bounds(n, _p(start), _p(end), _p(radius), sqrt_mode, _p(box))
        return box

    def closest_points(self, a0, a1, b0, b1):
        a0, a1, b0, b1 = (np.ascontiguousarray(x, np.float32) for x in (a0, a1, b0, b1))
        ac = np.zeros(3, np.float32)
        bc = np.zeros(3, np.float32)
        ok = self.lib.ora_closest_points(_p(a0), _p(a1), _p(b0), _p(b1), _p(ac), _p(bc))
        return bool(ok), ac, bc

    def intersect_box(self, box, o, d, tmax):
        box, o, d = (np.ascontiguousarray(x, np.float32) for x in (box, o, d))
        return bool(self.lib.ora_intersect_box(_p(box), _p(o), _p(d), float(tmax)))

    def radius_at(self, r0, alpha, it):
        return float(self.lib.ora_radius_at(r0, alpha, it))

    # -- photon pass (oracle/bre_oracle_photon.cpp) --
    def trace_photons(self, scene, n_photons, iteration=0, max_depth=5, radius=0.01):
        """Recursive restatement of the photon pass: beams in the reference's order + per-photon counts."""
        sp = ctypes.addressof(scene)
        counts = np.zeros(n_photons, np.int32)
        n = int(self.lib.ora_trace_photons(sp, n_photons, iteration, max_depth, float(radius), 0,
                                           None, None, None, None, _p(counts)))
        out = {"start": np.zeros((n, 3), np.float32), "end": np.zeros((n, 3), np.float32),
               "radius": np.zeros(n, np.float32), "power": np.zeros((n, 3), np.float32)}
        n2 = self.lib.ora_trace_photons(sp, n_photons, iteration, max_depth, float(radius), n, _p(out["start"]),
                                        _p(out["end"]), _p(out["radius"]), _p(out["power"]), None)
        assert n2 == n
        out["counts"] = counts
        return out

    def pcg32(self, seq, n, as_float=False):
        out = np.zeros(n, np.uint32)
        self.lib.ora_pcg32(seq, n, int(as_float), _p(out))
        return out.view(np.float32) if as_float else out

    def pcg32_srandom(self, initstate, initseq, n):
        out = np.zeros(n, np.uint32)
        self.lib.ora_pcg32_srandom(initstate, initseq, n, _p(out))
        return out

    def hg_sample(self, g, wo, u):
        wo, u = (np.ascontiguousarray(x, np.float32) for x in (wo, u))
        n = wo.shape[0]
        wi = np.zeros((n, 3), np.float32)
        pdf = np.zeros(n, np.float32)
        self.lib.ora_hg_sample(float(g), n, _p(wo), _p(u), _p(wi), _p(pdf))
        return wi, pdf

    def hg_p(self, g, wo, wi):
        wo, wi = (np.ascontiguousarray(x, np.float32) for x in (wo, wi))
        p = np.zeros(wo.shape[0], np.float32)
        self.lib.ora_hg_p(float(g), wo.shape[0], _p(wo), _p(wi), _p(p))
        return p

    def homogeneous_tr(self, sigma_a, sigma_s, d, tmax):
        sa, ss, d, tmax = (np.ascontiguousarray(x, np.float32) for x in (sigma_a, sigma_s, d, tmax))
        tr = np.zeros((d.shape[0], 3), np.float32)
        self.lib.ora_homogeneous_tr(_p(sa), _p(ss), d.shape[0], _p(d), _p(tmax), _p(tr))
        return tr

    def cosine_hemisphere(self, u):
        u = np.ascontiguousarray(u, np.float32)
        w = np.zeros((u.shape[0], 3), np.float32)
        self.lib.ora_cosine_hemisphere(u.shape[0], _p(u), _p(w))
        return w

    def fmath(self, kind, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros_like(x)
        self.lib.ora_fmath({"log": 0, "exp": 1, "sin": 2, "cos": 3}[kind], x.shape[0], _p(x), _p(y))
        return y

    # -- GridDensityMedium (oracle/ora_pbrt.h) --
    # -- the reference's own shape / sampling tests (tests/test_ref_tests.py) --
    def tri_hits(self, scene, o, d):
        """Per ray (tMax = inf): how many of the scene's triangles Triangle::Intersect hits."""
        o, d = (np.ascontiguousarray(x, np.float32) for x in (o, d))
        out = np.zeros(o.shape[0], np.int32)
        self.lib.ora_tri_hits(ctypes.addressof(scene), o.shape[0], _p(o), _p(d), _p(out))
        return out

    def scene_intersect(self, scene, o, d, bvh=True):
        """Scene::Intersect per ray (tMax = inf): (t, triangle or -1, BVH depth)."""
        o, d = (np.ascontiguousarray(x, np.float32) for x in (o, d))
        n = o.shape[0]
        t, tri, depth = np.zeros(n, np.float32), np.zeros(n, np.int32), ctypes.c_int32(0)
        self.lib.ora_scene_intersect(ctypes.addressof(scene), n, _p(o), _p(d), int(bool(bvh)), _p(t), _p(tri),
                                     ctypes.byref(depth))
        return t, tri, depth.value

    def tri_sample(self, scene, tri, u):
        """Triangle::Sample(u) of triangle `tri` (area measure): points, normals, pdfs."""
        u = np.ascontiguousarray(u, np.float32)
        n = u.shape[0]
        p, nrm, pdf = np.zeros((n, 3), np.float32), np.zeros((n, 3), np.float32), np.zeros(n, np.float32)
        self.lib.ora_tri_sample(ctypes.addressof(scene), int(tri), n, _p(u), _p(p), _p(nrm), _p(pdf))
        return p, nrm, pdf

    def distribution1d(self, func, u):
        """Distribution1D(func): SampleDiscrete(u) -> (index, pdf, uRemapped), and DiscretePDF."""
        func, u = np.ascontiguousarray(func, np.float32), np.ascontiguousarray(u, np.float32)
        m = u.shape[0]
        idx, pdf, urem = np.zeros(m, np.int32), np.zeros(m, np.float32), np.zeros(m, np.float32)
        dpdf = np.zeros(func.shape[0], np.float32)
        self.lib.ora_distribution1d(_p(func), func.shape[0], m, _p(u), _p(idx), _p(pdf), _p(urem), _p(dpdf))
        return idx, pdf, urem, dpdf

    def distribution1d_continuous(self, func, u):
        """Distribution1D(func).SampleContinuous(u) -> (x, pdf, offset)."""
        func, u = np.ascontiguousarray(func, np.float32), np.ascontiguousarray(u, np.float32)
        m = u.shape[0]
        x, pdf, off = np.zeros(m, np.float32), np.zeros(m, np.float32), np.zeros(m, np.int32)
        self.lib.ora_distribution1d_continuous(_p(func), func.shape[0], m, _p(u), _p(x), _p(pdf), _p(off))
        return x, pdf, off

    def pcg32_default(self, n):  # RNG() (rng.h:129)
        out = np.zeros(n, np.uint32)
        self.lib.ora_pcg32_default(n, _p(out))
        return out

    def next_float(self, x, up=True):  # NextFloatUp / NextFloatDown (pbrt.h:215-239)
        x = np.ascontiguousarray(x, dtype=np.float32)
        y = np.zeros_like(x)
        self.lib.ora_next_float(int(up), x.shape[0], _p(x), _p(y))
        return y

    def float_bits(self, u):  # FloatToBits(BitsToFloat(u)) (pbrt.h:191-202)
        u = np.ascontiguousarray(u, dtype=np.uint32)
        out = np.zeros_like(u)
        self.lib.ora_float_bits(u.shape[0], _p(u), _p(out))
        return out

    def find_interval(self, a, x):  # FindInterval(n, a[i] <= x) (pbrt.h:377-389)
        a = np.ascontiguousarray(a, dtype=np.float32)
        x = np.ascontiguousarray(x, dtype=np.float32)
        out = np.zeros(x.shape[0], np.int32)
        self.lib.ora_find_interval(_p(a), a.shape[0], x.shape[0], _p(x), _p(out))
        return out

    def tri_reintersect(self, n_tris=1000, rays_per_tri=10000):
        """Triangle.Reintersect (shapes.cpp:154-208): (re-intersections, rays tested, triangles used)."""
        tested, used = ctypes.c_int64(0), ctypes.c_int32(0)
        bad = int(self.lib.ora_tri_reintersect(int(n_tris), int(rays_per_tri), ctypes.byref(tested),
                                               ctypes.byref(used)))
        return bad, tested.value, used.value

    def grid_density(self, scene, p):
        p = np.ascontiguousarray(p, np.float32)
        out = np.zeros(p.shape[0], np.float32)
        self.lib.ora_grid_density(ctypes.addressof(scene), p.shape[0], _p(p), _p(out))
        return out

    def grid_eval(self, scene, kind, o, d, tmax, seq0=1):
        """kind 'tr' -> Tr per ray; 'sample' -> medium-space t or -1; plus sampler draws used."""
        o, d, tmax = (np.ascontiguousarray(x, np.float32) for x in (o, d, tmax))
        n = tmax.shape[0]
        out = np.zeros(n, np.float32)
        draws = np.zeros(n, np.int32)
        self.lib.ora_grid_eval(ctypes.addressof(scene), {"tr": 0, "sample": 1}[kind], n, _p(o), _p(d), _p(tmax),
                               seq0, _p(out), _p(draws))
        return out, draws

    # -- camera pass (oracle/bre_oracle_camera.cpp) --
    def camera_pass(self, scene, width, height, iteration=0, max_depth=5, render_surfaces=True, render_media=True):
        """Segments in row-major pixel order (depth order within a pixel) + surface radiance (W*H, 3)."""
        sp = ctypes.addressof(scene)
        args = (sp, width, height, iteration, max_depth, int(render_surfaces), int(render_media))
        n = int(self.lib.ora_camera_pass(*args, 0, None, None, None, None, None, None, None))
        assert n >= 0, "camera path ran out of Halton dimensions"
        out = {"o": np.zeros((n, 3), np.float32), "p": np.zeros((n, 3), np.float32), "d": np.zeros((n, 3), np.float32),
               "tmax": np.zeros(n, np.float32), "pixel": np.zeros(n, np.int32), "depth": np.zeros(n, np.int32)}
        ld = np.zeros((width * height, 3), np.float32)
        n2 = self.lib.ora_camera_pass(*args, n, _p(out["o"]), _p(out["p"]), _p(out["d"]), _p(out["tmax"]),
                                      _p(out["pixel"]), _p(out["depth"]), _p(ld))
        assert n2 == n
        out["surface"] = ld
        return out

    def halton(self, width, height, px, py, num, dim):
        px, py, dim = (np.ascontiguousarray(x, np.int32) for x in (px, py, dim))
        num = np.ascontiguousarray(num, np.int64)
        out = np.zeros(px.shape[0], np.float32)
        self.lib.ora_halton(width, height, px.shape[0], _p(px), _p(py), _p(num), _p(dim), _p(out))
        return out

    def radical_inverse(self, base_index, a):
        return np.float32(self.lib.ora_radical_inverse(base_index, a))

    def scrambled_radical_inverse(self, base_index, a, perm):
        perm = np.ascontiguousarray(perm, np.uint16)
        return np.float32(self.lib.ora_scrambled_radical_inverse(base_index, a, _p(perm)))

    def shuffle(self, seq, perm):
        perm = np.array(perm, np.uint16)
        self.lib.ora_shuffle(seq, perm.shape[0], _p(perm))
        return perm

    # -- gather through the reference SAH tree --
    def build(self, beams, sqrt_mode=0):
        return OracleBVH(self, beams, sqrt_mode)

    def bruteforce(self, beams, segs, R, sqrt_mode=0, nthreads=1):
        b = {k: np.ascontiguousarray(beams[k], np.float32) for k in ("start", "end", "radius", "power")}
        s = {k: np.ascontiguousarray(segs[k], np.float32) for k in ("o", "p", "d", "tmax")}
        nb, ns = b["radius"].shape[0], s["tmax"].shape[0]
        rgb = np.zeros((ns, 3), np.float32)
        rgb_exact = np.zeros((ns, 3), np.float64)
        cand = np.zeros(ns, np.int64)
        contrib = np.zeros(ns, np.int64)
        self.lib.ora_gather_bruteforce(nb, _p(b["start"]), _p(b["end"]), _p(b["radius"]), _p(b["power"]), sqrt_mode,
                                       ns, _p(s["o"]), _p(s["p"]), _p(s["d"]), _p(s["tmax"]), float(R), _p(rgb),
                                       _p(cand), _p(contrib), int(nthreads), _p(rgb_exact))
        # seg_rgb: the reference's float sum in beam order; seg_rgb_exact: the same terms in double
        return {"seg_rgb": rgb, "seg_rgb_exact": rgb_exact, "cand": cand, "contrib": contrib}


class OracleBVH:
    def __init__(self, ora: Oracle, beams, sqrt_mode=0):
        self.ora = ora
        self.b = {k: np.ascontiguousarray(beams[k], np.float32) for k in ("start", "end", "radius", "power")}
        n = self.b["radius"].shape[0]
        self.h = ora.lib.ora_bvh_build(n, _p(self.b["start"]), _p(self.b["end"]), _p(self.b["radius"]),
                                       _p(self.b["power"]), sqrt_mode)

    def node_count(self):
        return int(self.ora.lib.ora_bvh_node_count(self.h))

    def max_leaf(self):
        return int(self.ora.lib.ora_bvh_max_leaf(self.h))

    def gather(self, segs, R, npix=None, nthreads=1, chunk=256):
        s = {k: np.ascontiguousarray(segs[k], np.float32) for k in ("o", "p", "d", "tmax")}
        ns = s["tmax"].shape[0]
        pix = np.ascontiguousarray(segs["pixel"], np.int32) if "pixel" in segs else None
        rgb = np.zeros((ns, 3), np.float32)
        cand = np.zeros(ns, np.int64)
        vis = np.zeros(ns, np.int64)
        contrib = np.zeros(ns, np.int64)
        accum = None
        if npix is not None:
            accum = np.zeros((npix, 3), np.float32)
        self.ora.lib.ora_gather(self.h, ns, _p(s["o"]), _p(s["p"]), _p(s["d"]), _p(s["tmax"]), _p(pix), float(R),
                                _p(rgb), _p(accum), _p(cand), _p(vis), _p(contrib), int(nthreads), int(chunk))
        out = {"seg_rgb": rgb, "cand": cand, "visit": vis, "contrib": contrib}
        if accum is not None:
            out["accum"] = accum
        return out

    def gather_skip(self, segs, R, npix=None, nthreads=1):
        """Image-parity gather (ora_gather_skip): gather()'s per-segment sums and counts bit for bit,
        with candidates that provably cannot contribute skipped before ComputeClosestPoints; the film
        (npix) is composed here from the per-segment sums, in segment order."""
        s = {k: np.ascontiguousarray(segs[k], np.float32) for k in ("o", "p", "d", "tmax")}
        ns = s["tmax"].shape[0]
        rgb = np.zeros((ns, 3), np.float32)
        cand = np.zeros(ns, np.int64)
        contrib = np.zeros(ns, np.int64)
        skip = np.zeros(ns, np.int64)
        self.ora.lib.ora_gather_skip(self.h, ns, _p(s["o"]), _p(s["p"]), _p(s["d"]), _p(s["tmax"]), float(R),
                                     _p(rgb), _p(cand), _p(contrib), _p(skip), int(nthreads))
        out = {"seg_rgb": rgb, "cand": cand, "contrib": contrib, "skipped": skip}
        if npix is not None:
            accum = np.zeros((npix, 3), np.float32)
            np.add.at(accum, np.asarray(segs["pixel"], np.int64), rgb)  # sequential, segment order
            out["accum"] = accum
        return out

    def close(self):
        if self.h:
            self.ora.lib.ora_bvh_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_ORACLE = None


def load_oracle() -> Oracle:
    global _ORACLE
    if _ORACLE is None:
        srcs = [os.path.join(ORACLE_DIR, f) for f in ("bre_oracle.cpp", "bre_oracle_photon.cpp",
                                                      "bre_oracle_camera.cpp", "ora_pbrt.h")]
        srcs += [os.path.join(ROOT, "include", f) for f in ("bre_fmath.h", "bre_scene.h")]
        if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < max(os.path.getmtime(f) for f in srcs):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        _ORACLE = Oracle(ctypes.CDLL(ORACLE_SO))
    return _ORACLE
