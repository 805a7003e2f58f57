"""Independent pure-Python restatement of the photon pass (test infrastructure).

Written from the reference text (src/integrators/photonbeam.cpp:258-325, 383-421 and the pbrt
functions they call), NOT from oracle/bre_oracle_photon.cpp, with every float operation done on
numpy float32 scalars (IEEE single, like the reference's `Float`) and `Cross` in Python floats
(double, geometry.h:957-963).  The transcendentals are the host libm's expf / logf / sinf / cosf,
called through ctypes, as the reference calls them.  Slow (pure Python): used on a few hundred
photons to pin the C++ oracle.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import math
import struct

import numpy as np

f32 = np.float32
ONE_MINUS_EPS = f32(struct.unpack("<f", struct.pack("<I", 0x3F7FFFFF))[0])
INF = f32(np.inf)
MAXF = f32(3.402823466e38)
PI = f32(3.14159265358979323846)
INV_PI = f32(0.31830988618379067154)
PI_OVER_2 = f32(1.57079632679489661923)
PI_OVER_4 = f32(0.78539816339744830961)
MASK64 = (1 << 64) - 1


def _bits(x):
    return int(np.array(x, np.float32).view(np.uint32))


def _from_bits(u):
    return np.array(u & 0xFFFFFFFF, np.uint32).view(np.float32)[()]


# ---- transcendentals: the host libm itself, as the reference calls it (std::exp / std::log /
# std::sin / std::cos on a Float: expf, logf, sinf, cosf; spectrum.h:222-224, homogeneous.cpp:47,74,
# sampling.cpp:127, medium.cpp:194-213).  include/bre_fmath.h, which the oracle and the GPU use,
# returns these bits for every float input (tests/fmath_libm_check.c). ----
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _name in ("expf", "logf", "sinf", "cosf"):
    getattr(_libm, _name).argtypes = [ctypes.c_float]
    getattr(_libm, _name).restype = ctypes.c_float


def logf(x):
    return f32(_libm.logf(float(f32(x))))


def expf(x):
    return f32(_libm.expf(float(f32(x))))


def sincosf(x):
    x = float(f32(x))
    return f32(_libm.sinf(x)), f32(_libm.cosf(x))


# ---- PCG32 (rng.h) ----
class RNG:
    def __init__(self, seq):
        self.state = 0
        self.inc = ((seq << 1) | 1) & MASK64
        self.u32()
        self.state = (self.state + 0x853C49E6748FEA9B) & MASK64
        self.u32()

    def u32(self):
        old = self.state
        self.state = (old * 0x5851F42D4C957F2D + self.inc) & MASK64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF

    def uniform(self):
        v = f32(f32(self.u32()) * f32(2.0 ** -32))
        return v if v < ONE_MINUS_EPS else ONE_MINUS_EPS

    def get2d(self):
        first = self.uniform()
        second = self.uniform()
        return second, first  # g++: Point2f(Get1D(), Get1D()) evaluated right to left


# ---- vectors: tuples of float32 ----
def add(a, b):
    return tuple(f32(x + y) for x, y in zip(a, b))


def sub(a, b):
    return tuple(f32(x - y) for x, y in zip(a, b))


def mul(a, s):
    return tuple(f32(s * x) for x in a)


def div(a, s):
    inv = f32(f32(1) / s)
    return tuple(f32(x * inv) for x in a)


def dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def length(a):
    return f32(np.sqrt(dot(a, a)))


def normalize(a):
    return div(a, length(a))


def cross(a, b):
    ax, ay, az = (float(x) for x in a)
    bx, by, bz = (float(x) for x in b)
    return (f32(ay * bz - az * by), f32(az * bx - ax * bz), f32(ax * by - ay * bx))


def vabs(a):
    return tuple(f32(abs(x)) for x in a)


def coordinate_system(v1):
    if abs(v1[0]) > abs(v1[1]):
        v2 = div((-v1[2], f32(0), v1[0]), f32(np.sqrt(f32(f32(v1[0] * v1[0]) + f32(v1[2] * v1[2])))))
    else:
        v2 = div((f32(0), v1[2], -v1[1]), f32(np.sqrt(f32(f32(v1[1] * v1[1]) + f32(v1[2] * v1[2])))))
    return v2, cross(v1, v2)


def next_up(v):
    if v == INF:
        return v
    if v == 0:
        v = f32(0)
    u = _bits(v)
    return _from_bits(u + 1 if v >= 0 else u - 1)


def next_down(v):
    if v == -INF:
        return v
    if v == 0:
        v = f32(-0.0)
    u = _bits(v)
    return _from_bits(u - 1 if v > 0 else u + 1)


def offset_origin(p, perr, n, w):
    d = dot(vabs(n), perr)
    off = mul(n, d)
    if dot(w, n) < 0:
        off = tuple(-x for x in off)
    po = list(add(p, off))
    for i in range(3):
        if off[i] > 0:
            po[i] = next_up(po[i])
        elif off[i] < 0:
            po[i] = next_down(po[i])
    return tuple(po)


def gamma(n):
    e = f32(2.0 ** -24)
    return f32(f32(n * e) / f32(f32(1) - f32(n * e)))


def cosine_hemisphere(ux, uy):
    ox, oy = f32(f32(2 * ux) - f32(1)), f32(f32(2 * uy) - f32(1))
    if ox == 0 and oy == 0:
        dx = dy = f32(0)
    else:
        if abs(ox) > abs(oy):
            r, theta = ox, f32(PI_OVER_4 * f32(oy / ox))
        else:
            r, theta = oy, f32(PI_OVER_2 - f32(PI_OVER_4 * f32(ox / oy)))
        s, c = sincosf(theta)
        dx, dy = f32(c * r), f32(s * r)
    t = f32(f32(f32(1) - f32(dx * dx)) - f32(dy * dy))
    return (dx, dy, f32(np.sqrt(t if t > 0 else f32(0))))


def hg_sample(g, wo, u0, u1):
    g = f32(g)
    if abs(float(g)) < 1e-3:
        cos_t = f32(f32(1) - f32(2 * u0))
    else:
        sq = f32(f32(f32(1) - f32(g * g)) / f32(f32(f32(1) - g) + f32(f32(2 * g) * u0)))
        cos_t = f32(f32(f32(f32(1) + f32(g * g)) - f32(sq * sq)) / f32(2 * g))
    m = f32(f32(1) - f32(cos_t * cos_t))
    sin_t = f32(np.sqrt(m if m > 0 else f32(0)))
    phi = f32(f32(2 * PI) * u1)
    v1, v2 = coordinate_system(wo)
    sp, cp = sincosf(phi)
    return add(add(mul(v1, f32(sin_t * cp)), mul(v2, f32(sin_t * sp))), mul(tuple(-x for x in wo), cos_t))


def _gam(n):
    return gamma(n)


class Scene:
    def __init__(self, s):
        # one dict per pbrt Triangle (shapes/triangle.cpp)
        self.tris = []
        self.lights = []
        for i in range(s.n_triangles):
            t = s.triangles[i]
            p0, p1, p2 = (tuple(f32(x) for x in t.p[k]) for k in range(3))
            dp02, dp12 = sub(p0, p2), sub(p1, p2)
            # dpdu = (duv12[1] * dp02 - duv02[1] * dp12) * invdet with -1, -1, 1 (triangle.cpp:276-285)
            dpdu = mul(sub(mul(dp02, f32(-1)), mul(dp12, f32(-1))), f32(1))
            n = normalize(cross(dp02, dp12))
            ns = normalize(cross(sub(p1, p0), sub(p2, p0)))
            if t.flip:
                n = tuple(-x for x in n)
                ns = tuple(-x for x in ns)
            ss = normalize(dpdu)
            area = f32(0.5 * float(length(cross(sub(p1, p0), sub(p2, p0)))))
            self.tris.append(dict(p=(p0, p1, p2), n=n, ns=ns, ss=ss, ts=cross(n, ss), area=area,
                                  kd=tuple(f32(x) for x in t.kd), Le=tuple(f32(x) for x in t.Le)))
            if t.emit:
                self.lights.append(i)
        # ComputeLightPowerDistribution: Power() = 1 * Lemit * area * Pi, its y() (diffuse.cpp:64-66)
        func = []
        for li in self.lights:
            T = self.tris[li]
            pw = tuple(f32(f32(f32(c * f32(1)) * T["area"]) * PI) for c in T["Le"])
            func.append(f32(f32(f32(f32(0.212671) * pw[0]) + f32(f32(0.715160) * pw[1])) + f32(f32(0.072169) * pw[2])))
        nl = len(func)
        cdf = [f32(0)] * (nl + 1)
        for i in range(1, nl + 1):
            cdf[i] = f32(cdf[i - 1] + f32(func[i - 1] / f32(nl)))
        fint = cdf[nl]
        if fint == 0:
            cdf = [f32(f32(i) / f32(nl)) for i in range(nl + 1)]
        else:
            cdf = [cdf[0]] + [f32(c / fint) for c in cdf[1:]]
        self.lfunc, self.lcdf, self.lint = func, cdf, fint
        self.medium = bool(s.has_medium)
        self.sigma_t = tuple(f32(f32(a) + f32(b)) for a, b in zip(s.sigma_a, s.sigma_s))
        self.g = f32(s.g)
        self.grid = s.has_medium == 2
        if self.grid:  # GridDensityMedium ctor, grid.h:58-77
            self.n = tuple(int(v) for v in s.grid_n)
            self.m = [[f32(s.world_to_medium[4 * i + j]) for j in range(4)] for i in range(4)]
            cnt = self.n[0] * self.n[1] * self.n[2]
            self.density = np.ctypeslib.as_array((ctypes.c_float * cnt).from_address(s.grid_density)).copy()
            self.gsig = f32(f32(s.sigma_a[0]) + f32(s.sigma_s[0]))
            mx = f32(0)
            for v in self.density:
                mx = v if mx < v else mx
            self.inv_max = f32(f32(1) / mx)

    def sample_light(self, u):
        """Distribution1D::SampleDiscrete (sampling.h:90-100) with FindInterval (pbrt.h:377-389)."""
        size = len(self.lcdf)
        first, ln = 0, size
        while ln > 0:
            half = ln >> 1
            mid = first + half
            if self.lcdf[mid] <= u:
                first = mid + 1
                ln -= half + 1
            else:
                ln = half
        off = min(max(first - 1, 0), size - 2)
        pdf = f32(self.lfunc[off] / f32(self.lint * f32(len(self.lfunc)))) if self.lint > 0 else f32(0)
        return off, pdf

    @staticmethod
    def hit_tri(T, o, d, tmax):
        """Triangle::Intersect (triangle.cpp:177-300): watertight test; (t, p, pError) or None."""
        p0, p1, p2 = T["p"]
        ad = vabs(d)
        kz = (0 if ad[0] > ad[2] else 2) if ad[0] > ad[1] else (1 if ad[1] > ad[2] else 2)
        kx = 0 if kz + 1 == 3 else kz + 1
        ky = 0 if kx + 1 == 3 else kx + 1

        def perm(v):
            return [v[kx], v[ky], v[kz]]

        dd = perm(d)
        a, b, c = perm(sub(p0, o)), perm(sub(p1, o)), perm(sub(p2, o))
        sx = f32(-dd[0] / dd[2])
        sy = f32(-dd[1] / dd[2])
        sz = f32(f32(1) / dd[2])
        for v in (a, b, c):
            v[0] = f32(v[0] + f32(sx * v[2]))
            v[1] = f32(v[1] + f32(sy * v[2]))
        e0 = f32(f32(b[0] * c[1]) - f32(b[1] * c[0]))
        e1 = f32(f32(c[0] * a[1]) - f32(c[1] * a[0]))
        e2 = f32(f32(a[0] * b[1]) - f32(a[1] * b[0]))
        if e0 == 0 or e1 == 0 or e2 == 0:
            e0 = f32(float(c[1]) * float(b[0]) - float(c[0]) * float(b[1]))
            e1 = f32(float(a[1]) * float(c[0]) - float(a[0]) * float(c[1]))
            e2 = f32(float(b[1]) * float(a[0]) - float(b[0]) * float(a[1]))
        if (e0 < 0 or e1 < 0 or e2 < 0) and (e0 > 0 or e1 > 0 or e2 > 0):
            return None
        det = f32(f32(e0 + e1) + e2)
        if det == 0:
            return None
        for v in (a, b, c):
            v[2] = f32(v[2] * sz)
        ts = f32(f32(f32(e0 * a[2]) + f32(e1 * b[2])) + f32(e2 * c[2]))
        if det < 0 and (ts >= 0 or ts < f32(tmax * det)):
            return None
        if det > 0 and (ts <= 0 or ts > f32(tmax * det)):
            return None
        inv = f32(f32(1) / det)
        b0, b1, b2 = f32(e0 * inv), f32(e1 * inv), f32(e2 * inv)
        t = f32(ts * inv)
        mz = max(abs(a[2]), max(abs(b[2]), abs(c[2])))
        mx = max(abs(a[0]), max(abs(b[0]), abs(c[0])))
        my = max(abs(a[1]), max(abs(b[1]), abs(c[1])))
        dz = f32(_gam(3) * mz)
        dx = f32(_gam(5) * f32(mx + mz))
        dy = f32(_gam(5) * f32(my + mz))
        de = f32(f32(2) * f32(f32(f32(f32(_gam(2) * mx) * my) + f32(dy * mx)) + f32(dx * my)))
        me = max(abs(e0), max(abs(e1), abs(e2)))
        dt = f32(f32(f32(3) * f32(f32(f32(f32(_gam(3) * me) * mz) + f32(de * mz)) + f32(dz * me))) * abs(inv))
        if t <= dt:
            return None
        sums = [f32(f32(abs(f32(b0 * p0[k])) + abs(f32(b1 * p1[k]))) + abs(f32(b2 * p2[k]))) for k in range(3)]
        perr = mul(tuple(sums), _gam(7))
        p = add(add(mul(p0, b0), mul(p1, b1)), mul(p2, b2))
        return t, p, perr

    def intersect(self, o, d):
        best = None
        tmax = INF
        for i, T in enumerate(self.tris):
            h = self.hit_tri(T, o, d, tmax)
            if h is None:
                continue
            tmax = h[0]
            best = (h[1], h[2], i)
        return best, tmax

    def sample_tri(self, T, u0, u1):
        """Triangle::Sample (triangle.cpp:543-568): point, pError, normal, area pdf."""
        su0 = f32(np.sqrt(u0))
        b0, b1 = f32(f32(1) - su0), f32(u1 * su0)
        b2 = f32(f32(f32(1) - b0) - b1)
        p0, p1, p2 = T["p"]
        a, b, c = mul(p0, b0), mul(p1, b1), mul(p2, b2)
        p = add(add(a, b), c)
        perr = mul(add(add(vabs(a), vabs(b)), vabs(c)), _gam(6))
        return p, perr, T["ns"], f32(f32(1) / T["area"])

    def tr(self, d, tmax):
        x = f32(tmax * length(d))
        x = MAXF if MAXF < x else x
        return tuple(expf(f32(f32(-st) * x)) for st in self.sigma_t)


# ---- GridDensityMedium (grid.cpp:46-118; grid.h:84-88) ----
def _lerp(t, a, b):
    return f32(f32(f32(f32(1) - t) * a) + f32(t * b))


def _grid_d(sc, x, y, z):
    nx, ny, nz = sc.n
    if not (0 <= x < nx and 0 <= y < ny and 0 <= z < nz):
        return f32(0)
    return sc.density[(z * ny + y) * nx + x]


def _grid_density(sc, p):
    ps = [f32(f32(p[i] * f32(sc.n[i])) - f32(0.5)) for i in range(3)]
    pi = [int(math.floor(v)) for v in ps]
    d = [f32(ps[i] - f32(pi[i])) for i in range(3)]
    x, y, z = pi
    d00 = _lerp(d[0], _grid_d(sc, x, y, z), _grid_d(sc, x + 1, y, z))
    d10 = _lerp(d[0], _grid_d(sc, x, y + 1, z), _grid_d(sc, x + 1, y + 1, z))
    d01 = _lerp(d[0], _grid_d(sc, x, y, z + 1), _grid_d(sc, x + 1, y, z + 1))
    d11 = _lerp(d[0], _grid_d(sc, x, y + 1, z + 1), _grid_d(sc, x + 1, y + 1, z + 1))
    return _lerp(d[2], _lerp(d[1], d00, d10), _lerp(d[1], d01, d11))


def _grid_ray(sc, o, d, tmax):
    """WorldToMedium(Ray(o, Normalize(d), tMax*|d|)) (transform.h:251-299) and the unit-box
    IntersectP with t0/t1 (geometry.h:1386-1408); None on a miss."""
    dn = normalize(d)
    tm = f32(tmax * length(d))
    m = sc.m
    row = [f32(f32(f32(f32(m[i][0] * o[0]) + f32(m[i][1] * o[1])) + f32(m[i][2] * o[2])) + m[i][3]) for i in range(4)]
    err = [f32(f32(f32(abs(f32(m[i][0] * o[0])) + abs(f32(m[i][1] * o[1]))) + abs(f32(m[i][2] * o[2]))) + abs(m[i][3]))
           for i in range(3)]
    g3 = gamma(3)
    oerr = tuple(f32(g3 * e) for e in err)
    po = tuple(row[:3])
    if not (row[3] == 1):
        inv = f32(f32(1) / row[3])
        po = tuple(f32(inv * v) for v in po)
    dv = tuple(f32(f32(f32(m[i][0] * dn[0]) + f32(m[i][1] * dn[1])) + f32(m[i][2] * dn[2])) for i in range(3))
    l2 = dot(dv, dv)
    if l2 > 0:
        dt = f32(dot(vabs(dv), oerr) / l2)
        po = add(po, mul(dv, dt))
        tm = f32(tm - dt)
    t0, t1 = f32(0), tm
    pad = f32(f32(1) + f32(f32(2) * g3))
    for i in range(3):
        inv = f32(f32(1) / dv[i]) if dv[i] != 0 else f32(math.copysign(np.inf, dv[i]))
        with np.errstate(invalid="ignore"):
            tn = f32(f32(f32(0) - po[i]) * inv)
            tf = f32(f32(f32(1) - po[i]) * inv)
        if tn > tf:
            tn, tf = tf, tn
        tf = f32(tf * pad)
        t0 = tn if tn > t0 else t0
        t1 = tf if tf < t1 else t1
        if t0 > t1:
            return None
    return po, dv, t0, t1


def grid_sample(sc, rng, o, d, tmax):
    """Delta tracking (grid.cpp:62-89): the medium-space t of the interaction, or None."""
    r = _grid_ray(sc, o, d, tmax)
    if r is None:
        return None
    mo, md, t, tm = r
    while True:
        t = f32(t - f32(f32(logf(f32(f32(1) - rng.uniform())) * sc.inv_max) / sc.gsig))
        if t >= tm:
            return None
        if f32(_grid_density(sc, add(mo, mul(md, t))) * sc.inv_max) > rng.uniform():
            return t


def grid_tr(sc, rng, o, d, tmax):
    """Ratio tracking with Russian roulette below 0.1 (grid.cpp:91-118)."""
    r = _grid_ray(sc, o, d, tmax)
    if r is None:
        return f32(1)
    mo, md, t, tm = r
    tr = f32(1)
    while True:
        t = f32(t - f32(f32(logf(f32(f32(1) - rng.uniform())) * sc.inv_max) / sc.gsig))
        if t >= tm:
            return tr
        dens = _grid_density(sc, add(mo, mul(md, t)))
        x = f32(dens * sc.inv_max)
        tr = f32(tr * f32(f32(1) - (x if f32(0) < x else f32(0))))
        if tr < f32(0.1):
            q = f32(f32(1) - tr)
            q = q if f32(0.05) < q else f32(0.05)
            if rng.uniform() < q:
                return f32(0)
            tr = f32(tr / f32(f32(1) - q))


def trace_photon(sc: Scene, seq: int, max_depth: int, radius: float):
    """Beams of one photon, in the reference's push order: list of (start, end, radius, power)."""
    rng = RNG(seq)
    out = []
    ln, light_pdf = sc.sample_light(rng.uniform())  # lightDistr->SampleDiscrete
    u0 = rng.get2d()
    u1 = rng.get2d()
    rng.uniform()  # time
    L = sc.tris[sc.lights[ln]]
    p, perr, nl, pdf_pos = sc.sample_tri(L, *u0)
    wl = cosine_hemisphere(*u1)
    pdf_dir = f32(wl[2] * INV_PI)
    v1, v2 = coordinate_system(nl)
    w = add(add(mul(v1, wl[0]), mul(v2, wl[1])), mul(nl, wl[2]))
    o = offset_origin(p, perr, nl, w)
    Le = L["Le"] if dot(nl, w) > 0 else (f32(0),) * 3
    if pdf_pos == 0 or pdf_dir == 0 or all(x == 0 for x in Le):
        return out
    ad = f32(abs(dot(nl, w)))
    den = f32(f32(light_pdf * pdf_pos) * pdf_dir)
    beta = tuple(f32(f32(ad * x) / den) for x in Le)
    if all(x == 0 for x in beta):
        return out

    def rec(o, d, depth, beta):
        while depth < max_depth:
            hit, tmax = sc.intersect(o, d)
            if hit is None:
                return
            scattered = False
            if sc.medium and sc.grid:
                t = grid_sample(sc, rng, o, d, tmax)
                scattered = t is not None
            elif sc.medium:
                ch = min(int(f32(rng.uniform() * f32(3))), 2)
                dist = f32(-logf(f32(f32(1) - rng.uniform())) / sc.sigma_t[ch])
                dl = f32(dist * length(d))
                t = tmax if tmax < dl else dl
                scattered = bool(t < tmax)
            if all(x == 0 for x in beta):
                return
            if scattered:
                hx, hy = rng.get2d()
                wi = hg_sample(sc.g, tuple(-x for x in d), hx, hy)
                trv = (grid_tr(sc, rng, o, d, tmax),) * 3 if sc.grid else sc.tr(d, tmax)
                rec(add(o, mul(d, t)), wi, depth + 1, tuple(f32(b * x) for b, x in zip(beta, trv)))
            if sc.medium and sc.grid:
                bm = (grid_tr(sc, rng, o, d, tmax),) * 3
            else:
                bm = sc.tr(d, tmax) if sc.medium else (f32(1),) * 3
            out.append((o, hit[0], f32(radius), tuple(f32(a * b) for a, b in zip(bm, beta))))
            q = sc.tris[hit[2]]
            ux, uy = rng.get2d()
            if all(x == 0 for x in q["kd"]):
                return
            wo = tuple(-x for x in d)
            woz = dot(wo, q["n"])
            if woz == 0:
                return
            wil = list(cosine_hemisphere(ux, uy))
            if woz < 0:
                wil[2] = f32(wil[2] * f32(-1))
            pdf = f32(abs(wil[2]) * INV_PI) if f32(woz * wil[2]) > 0 else f32(0)
            fr = tuple(f32(k * INV_PI) for k in q["kd"])
            if pdf == 0 or all(x == 0 for x in fr):
                return
            ss, ts, n = q["ss"], q["ts"], q["n"]
            wi = tuple(f32(f32(f32(ss[i] * wil[0]) + f32(ts[i] * wil[1])) + f32(n[i] * wil[2])) for i in range(3))
            adw = f32(abs(dot(wi, n)))
            bn = tuple(f32(f32(f32(f32(bm[c] * beta[c]) * fr[c]) * adw) / pdf) for c in range(3))
            o = offset_origin(hit[0], hit[1], n, wi)
            d = wi

            def y(s):
                return f32(f32(f32(f32(0.212671) * s[0]) + f32(f32(0.715160) * s[1])) + f32(f32(0.072169) * s[2]))

            ratio = f32(f32(1) - f32(y(bn) / y(beta)))
            qrr = ratio if f32(0) < ratio else f32(0)
            if rng.uniform() < qrr:
                return
            beta = tuple(f32(x / f32(f32(1) - qrr)) for x in bn)
            depth += 1

    rec(o, w, 0, beta)
    return out


def trace_photons(scene_struct, n_photons, iteration=0, max_depth=5, radius=0.01, first=None):
    """Photons [0, first or n_photons) of a pass of n_photons (sequences iteration*N + i + 1)."""
    sc = Scene(scene_struct)
    beams = []
    counts = []
    for i in range(first if first is not None else n_photons):
        b = trace_photon(sc, iteration * n_photons + i + 1, max_depth, radius)
        counts.append(len(b))
        beams.extend(b)
    n = len(beams)
    arr = {"start": np.zeros((n, 3), np.float32), "end": np.zeros((n, 3), np.float32),
           "radius": np.zeros(n, np.float32), "power": np.zeros((n, 3), np.float32)}
    for k, (s, e, r, pw) in enumerate(beams):
        arr["start"][k] = s
        arr["end"][k] = e
        arr["radius"][k] = r
        arr["power"][k] = pw
    arr["counts"] = np.array(counts, np.int32)
    return arr



# ---- HaltonSampler restated (src/samplers/halton.cpp:63-127, lowdiscrepancy.cpp) ----
class DefaultRNG(RNG):
    """RNG() with PCG32_DEFAULT_STATE / PCG32_DEFAULT_STREAM (rng.h:145)."""

    def __init__(self):
        self.state = 0x853C49E6748FEA9B
        self.inc = 0xDA3E39CB94B95BDB


def uniform_u32_bounded(rng, b):
    threshold = ((~b + 1) & 0xFFFFFFFF) % b
    while True:
        r = rng.u32()
        if r >= threshold:
            return r % b


def shuffle(perm, rng):
    n = len(perm)
    for i in range(n):
        other = i + uniform_u32_bounded(rng, n - i)
        perm[i], perm[other] = perm[other], perm[i]
    return perm


def primes(n):
    out = []
    c = 2
    while len(out) < n:
        if all(c % q for q in out if q * q <= c):
            out.append(c)
        c += 1
    return out


class Halton:
    def __init__(self, width, height, ndims=16):
        self.primes = primes(ndims)
        rng = DefaultRNG()
        self.perms = [shuffle(list(range(p)), rng) for p in self.primes]
        self.scales, self.exps = [], []
        for res, base in ((width, 2), (height, 3)):
            scale, e = 1, 0
            while scale < min(res, 128):
                scale *= base
                e += 1
            self.scales.append(scale)
            self.exps.append(e)
        self.stride = self.scales[0] * self.scales[1]
        self.minv = [pow(self.scales[1], -1, self.scales[0]) if self.scales[0] > 1 else 0,
                     pow(self.scales[0], -1, self.scales[1]) if self.scales[1] > 1 else 0]

    def index(self, px, py, num):
        off = 0
        if self.stride > 1:
            for i, (p, base) in enumerate(((px % 128, 2), (py % 128, 3))):
                digits, inv = 0, p
                for _ in range(self.exps[i]):
                    digits = digits * base + inv % base
                    inv //= base
                off += digits * (self.stride // self.scales[i]) * self.minv[i]
            off %= self.stride
        return off + num * self.stride

    def sample(self, index, dim):
        if dim == 0:
            a = index >> self.exps[0]
            rev = int("{:064b}".format(a)[::-1], 2)
            return f32(rev * 2.0 ** -64)
        base = self.primes[dim]
        perm = self.perms[dim] if dim >= 2 else list(range(base))
        a = index if dim >= 2 else index // self.scales[1]
        inv_base = f32(f32(1) / f32(base))
        rev, inv_n = 0, f32(1)
        while a:
            rev = rev * base + perm[a % base]
            inv_n = f32(inv_n * inv_base)
            a //= base
        if dim == 1:
            v = f32(f32(rev) * inv_n)
        else:
            v = f32(inv_n * f32(f32(rev) + f32(f32(inv_base * f32(perm[0])) / f32(f32(1) - inv_base))))
        return v if v < ONE_MINUS_EPS else ONE_MINUS_EPS
