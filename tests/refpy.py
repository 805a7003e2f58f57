"""Independent pure-Python restatement of the reference's per-pair arithmetic (test infrastructure).

Written separately from oracle/bre_oracle.cpp so the two restatements check each other.  Every
operation is a numpy float32 scalar op (IEEE single, one rounding per op, no FMA), except where the
reference uses double (Cross, geometry.h:957-963; WorldBound's ::sqrt(double) reading).
For small cases only (pure-Python loops).
"""
import math

import numpy as np

f = np.float32


def v(x, y, z):
    return (f(x), f(y), f(z))


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def scale(a, s):  # Vector3::operator*(s) = (s*x, s*y, s*z)
    return (s * a[0], s * a[1], s * a[2])


def divv(a, d):  # Vector3::operator/(d): multiply by (Float)1/d
    inv = f(1) / f(d)
    return (a[0] * inv, a[1] * inv, a[2] * inv)


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def length(a):
    return np.sqrt(dot(a, a), dtype=np.float32)


def cross(a, b):
    ax, ay, az = (float(t) for t in a)
    bx, by, bz = (float(t) for t in b)
    return (f(ay * bz - az * by), f(az * bx - ax * bz), f(ax * by - ay * bx))


def det(a, b, c):
    return (a[0] * b[1] * c[2] + a[1] * b[2] * c[0] + a[2] * b[0] * c[1]) - (
        a[2] * b[1] * c[0] + a[1] * b[0] * c[2] + a[0] * b[2] * c[1])


def clamp(x, lo, hi):
    return lo if x < lo else (hi if x > hi else x)


def smin(a, b):
    return b if b < a else a


def smax(a, b):
    return b if a < b else a


def slab_pad():
    eps = f(2.0**-24)
    g3 = (f(3) * eps) / (f(1) - f(3) * eps)
    return f(1) + f(2) * g3


def world_bound(start, end, radius):
    """photonbeambvh.h:60-72 with the libstdc++ (double sqrt) reading."""
    start, end, radius = v(*start), v(*end), f(radius)
    d = sub(end, start)
    center = add(start, divv(d, 2))
    ln = length(d)
    d = divv(d, ln)
    tr = f(2) * radius
    size = tuple(f(float(d[i] * ln) + float(tr) * math.sqrt(float(f(1) - d[i] * d[i]))) for i in range(3))
    half = divv(size, 2)
    p1, p2 = sub(center, half), add(center, half)
    lo = tuple(smin(p1[i], p2[i]) for i in range(3))
    hi = tuple(smax(p1[i], p2[i]) for i in range(3))
    return lo, hi


def intersect_p(lo, hi, o, d, tmax):
    """geometry.h:1410-1436 (invDir = 1/d, dirIsNeg = invDir < 0)."""
    o, d = v(*o), v(*d)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = tuple(f(1) / d[i] for i in range(3))
        neg = [int(inv[i] < 0) for i in range(3)]
        b = (tuple(f(x) for x in lo), tuple(f(x) for x in hi))
        pad = slab_pad()
        tMin = (b[neg[0]][0] - o[0]) * inv[0]
        tMax = (b[1 - neg[0]][0] - o[0]) * inv[0]
        tyMin = (b[neg[1]][1] - o[1]) * inv[1]
        tyMax = (b[1 - neg[1]][1] - o[1]) * inv[1]
        tMax = tMax * pad
        tyMax = tyMax * pad
        if tMin > tyMax or tyMin > tMax:
            return False
        if tyMin > tMin:
            tMin = tyMin
        if tyMax < tMax:
            tMax = tyMax
        tzMin = (b[neg[2]][2] - o[2]) * inv[2]
        tzMax = (b[1 - neg[2]][2] - o[2]) * inv[2]
        tzMax = tzMax * pad
        if tMin > tzMax or tzMin > tMax:
            return False
        if tzMin > tMin:
            tMin = tzMin
        if tzMax < tMax:
            tMax = tzMax
        return bool((tMin < f(tmax)) and (tMax > 0))


def closest_points(a0, a1, b0, b1):
    """photonbeam.cpp:87-186.  Returns (ok, aClosest, bClosest)."""
    a0, a1, b0, b1 = v(*a0), v(*a1), v(*b0), v(*b1)
    A, B = sub(a1, a0), sub(b1, b0)
    magA, magB = length(A), length(B)
    if magA == 0:
        if magB == 0:
            return True, a0, b0
        B = divv(B, magB)
        A = sub(a0, b0)
        return True, a0, add(b0, scale(B, clamp(dot(A, B), f(0), magB)))
    if magB == 0:
        A = divv(A, magA)
        B = sub(b0, a0)
        return True, add(a0, scale(A, clamp(dot(A, B), f(0), magA))), b0
    A, B = divv(A, magA), divv(B, magB)
    c = cross(A, B)
    denom = dot(c, c)
    if denom == 0:
        return False, a0, b1
    t = sub(b0, a0)
    t0 = det(t, B, c) / denom
    t1 = det(t, A, c) / denom
    pA = add(a0, scale(A, t0))
    pB = add(b0, scale(B, t1))
    if t0 < 0:
        pA = a0
    elif t0 > magA:
        pA = a1
    if t0 < 0 or t0 > magA:
        pB = add(b0, scale(B, clamp(dot(B, sub(pA, b0)), f(0), magB)))
    if t1 < 0 or t1 > magB:
        pA = add(a0, scale(A, clamp(dot(A, sub(pB, a0)), f(0), magA)))
    return True, pA, pB


def contribution(beam, o, p, R):
    """One beam's RGB increment to a segment (photonbeam.cpp:499-506) or None."""
    start, end, radius, power = beam
    ok, ac, bc = closest_points(o, p, start, end)
    if not ok:
        return None
    maxd = f(R) + f(radius)
    dist = length(sub(ac, bc))
    if not dist < maxd:
        return None
    r = dist / maxd
    w = np.sqrt(f(1) - r * r, dtype=np.float32)
    k = f(1e-5)
    return tuple((f(power[i]) * k) * w for i in range(3))
