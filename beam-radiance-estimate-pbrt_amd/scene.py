"""ctypes mirror of include/bre_scene.h and the benchmark scene of SURVEY.md §8d (C1/C2).

Pure data: the same struct the C ABI takes (``bre_trace_photons``) and the oracle restatement
reads (``ora_trace_photons``).  ``cornell_scene`` must stay identical to libbre's
``bre_scene_cornell`` (checked byte for byte by tests/test_photon_oracle.py).
"""
from __future__ import annotations

import ctypes

MAX_TRIANGLES = 128               # inline in Scene.triangles
MAX_SCENE_TRIANGLES = 1 << 24     # through Scene.triangles_ext
MAX_DEPTH = 16
MEDIUM_NONE, MEDIUM_HOMOGENEOUS, MEDIUM_GRID = 0, 1, 2

F3 = ctypes.c_float * 3


class Triangle(ctypes.Structure):
    """bre_triangle: one pbrt Triangle (world-space vertices in mesh index order)."""
    _fields_ = [("p", F3 * 3), ("kd", F3), ("Le", F3), ("emit", ctypes.c_int32), ("flip", ctypes.c_int32)]


class Scene(ctypes.Structure):
    _fields_ = [("n_triangles", ctypes.c_int32),
                ("has_medium", ctypes.c_int32), ("sigma_a", F3), ("sigma_s", F3), ("g", ctypes.c_float),
                ("cam_pos", F3), ("cam_look", F3), ("cam_up", F3), ("cam_fov_deg", ctypes.c_float),
                ("triangles", Triangle * MAX_TRIANGLES),
                ("grid_n", ctypes.c_int32 * 3), ("world_to_medium", ctypes.c_float * 16),
                ("grid_density", ctypes.c_void_p), ("triangles_ext", ctypes.c_void_p)]

    def to_bytes(self) -> bytes:
        return ctypes.string_at(ctypes.addressof(self), ctypes.sizeof(self))


class RenderParams(ctypes.Structure):
    """bre_render_params: CreatePhotonBeamIntegrator's parameters (photonbeam.cpp:589-611)."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("iterations", ctypes.c_int32),
                ("start_iteration", ctypes.c_int32), ("end_iteration", ctypes.c_int32),
                ("photons_per_iteration", ctypes.c_int64), ("max_depth", ctypes.c_int32),
                ("render_surfaces", ctypes.c_int32), ("render_media", ctypes.c_int32),
                ("initial_radius", ctypes.c_float), ("alpha", ctypes.c_float)]


def render_params(width, height, iterations=64, photons=-1, max_depth=5, radius=1.0, alpha=0.5,
                  render_surfaces=True, render_media=True, start_iteration=0, end_iteration=None) -> RenderParams:
    """Defaults as the reference's (iterations 64, maxdepth 5, initialbeamradius 1, alpha 0.5)."""
    return RenderParams(int(width), int(height), int(iterations), int(start_iteration),
                        int(iterations if end_iteration is None else end_iteration), int(photons), int(max_depth),
                        int(render_surfaces), int(render_media), float(radius), float(alpha))


def _f3(v):
    return F3(*[float(x) for x in v])


def make_scene(meshes, sigma_a=None, sigma_s=None, g=0.0,
               cam_pos=(0.5, 0.5, 0.02), cam_look=(0.5, 0.5, 1.0), cam_up=(0.0, 1.0, 0.0), fov=60.0) -> Scene:
    """meshes: list of (P, indices, kd, Le) -- a pbrt "trianglemesh" with world-space points P
    (list of xyz), index triples, Lambertian kd, and Le (None = not emitting); medium present iff
    sigma_a is given (RGB or scalar).  More than MAX_TRIANGLES triangles go to an external array
    (Scene.triangles_ext, kept alive on the scene object)."""
    s = Scene()
    ctypes.memset(ctypes.addressof(s), 0, ctypes.sizeof(s))
    total = sum(len(idx) // 3 for _, idx, _, _ in meshes)
    assert total <= MAX_SCENE_TRIANGLES
    ext = (Triangle * total)() if total > MAX_TRIANGLES else None
    dst = ext if ext is not None else s.triangles
    n = 0
    for P, idx, kd, Le in meshes:
        assert len(idx) % 3 == 0
        for t in range(len(idx) // 3):
            T = dst[n]
            for v in range(3):
                T.p[v] = _f3(P[idx[3 * t + v]])
            T.kd = _f3(kd)
            if Le is not None:
                T.emit = 1
                T.Le = _f3(Le)
            n += 1
    s.n_triangles = n
    if ext is not None:
        s.triangles_ext = ctypes.addressof(ext)
        s._triangles_ref = ext
    if sigma_a is not None:
        rgb = (lambda v: (v, v, v) if isinstance(v, (int, float)) else tuple(v))
        s.has_medium = 1
        s.sigma_a = _f3(rgb(sigma_a))
        s.sigma_s = _f3(rgb(sigma_s))
        s.g = float(g)
    s.cam_pos, s.cam_look, s.cam_up = _f3(cam_pos), _f3(cam_look), _f3(cam_up)
    s.cam_fov_deg = float(fov)
    return s


WHITE = (0.73, 0.73, 0.73)
RED = (0.63, 0.065, 0.05)
GREEN = (0.14, 0.45, 0.091)
QUAD = (0, 1, 2, 0, 2, 3)  # scenes/cornell_world.pbrt: "integer indices" [0 1 2 0 2 3]


def cornell_meshes(light_L=(17.0, 12.0, 4.0)):
    """scenes/cornell_world.pbrt: unit-cube Cornell box, one two-triangle mesh per wall (normals
    inward), the area light last (facing down)."""
    return [
        ([(0, 0, 0), (0, 0, 1), (1, 0, 1), (1, 0, 0)], QUAD, WHITE, None),     # floor
        ([(0, 1, 0), (1, 1, 0), (1, 1, 1), (0, 1, 1)], QUAD, WHITE, None),     # ceiling
        ([(0, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 1)], QUAD, WHITE, None),     # back wall
        ([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0)], QUAD, WHITE, None),     # front wall (behind the camera)
        ([(0, 0, 0), (0, 1, 0), (0, 1, 1), (0, 0, 1)], QUAD, RED, None),       # left wall
        ([(1, 0, 0), (1, 0, 1), (1, 1, 1), (1, 1, 0)], QUAD, GREEN, None),     # right wall
        ([(0.35, 0.999, 0.35), (0.65, 0.999, 0.35), (0.65, 0.999, 0.65), (0.35, 0.999, 0.65)], QUAD, (0, 0, 0),
         light_L),                                                            # area light
    ]


def cornell_scene(sigma_a: float = 0.05, sigma_s: float = 0.5, g: float = 0.0) -> Scene:
    """Cornell box in homogeneous fog (sigma_a 0.05, sigma_s 0.5, g 0)."""
    return make_scene(cornell_meshes(), sigma_a, sigma_s, g)


def uv_sphere(center=(0.5, 0.35, 0.55), radius=0.2, n_theta=64, n_phi=96):
    """A triangulated sphere as one pbrt "trianglemesh": (points, indices) with n_theta rings and
    n_phi segments, outward-facing (counter-clockwise seen from outside), poles shared:
    2 * n_phi * (n_theta - 1) triangles (12,096 at the defaults)."""
    import numpy as np

    cx, cy, cz = (float(v) for v in center)
    pts = [(cx, cy + radius, cz)]
    for t in range(1, n_theta):
        th = np.pi * t / n_theta
        for k in range(n_phi):
            ph = 2 * np.pi * k / n_phi
            pts.append((cx + radius * np.sin(th) * np.cos(ph), cy + radius * np.cos(th), cz + radius * np.sin(th) * np.sin(ph)))
    pts.append((cx, cy - radius, cz))
    ring = lambda t, k: 1 + (t - 1) * n_phi + (k % n_phi)  # noqa: E731
    idx = []
    for k in range(n_phi):
        idx += [0, ring(1, k + 1), ring(1, k)]
    for t in range(1, n_theta - 1):
        for k in range(n_phi):
            a, b, c, d = ring(t, k), ring(t, k + 1), ring(t + 1, k), ring(t + 1, k + 1)
            idx += [a, b, d, a, d, c]
    south = len(pts) - 1
    for k in range(n_phi):
        idx += [south, ring(n_theta - 1, k), ring(n_theta - 1, k + 1)]
    return [tuple(np.float32(c) for c in p) for p in pts], idx


def cornell_sphere_scene(sigma_a: float = 0.05, sigma_s: float = 0.5, g: float = 0.0, n_theta=64, n_phi=96) -> Scene:
    """The C1/C2 Cornell box in fog with a white tessellated sphere (uv_sphere, 12,096 triangles at
    the defaults) on the floor side: a scene far past the 128 inline triangles, through
    Scene.triangles_ext and the scene BVH (bvh.cpp BVHAccel)."""
    P, idx = uv_sphere(n_theta=n_theta, n_phi=n_phi)
    meshes = cornell_meshes()
    return make_scene(meshes[:-1] + [(P, idx, (0.6, 0.6, 0.6), None)] + meshes[-1:], sigma_a, sigma_s, g)


def smoke_density(n: int = 64, seed: int = 7):
    """bre_smoke_density: seeded value-noise smoke (n^3 float32, x fastest), from libbre's host code."""
    import numpy as np

    from . import load_library

    lib = load_library()
    out = np.zeros(n * n * n, np.float32)
    lib.bre_smoke_density(ctypes.c_int32(n), ctypes.c_uint64(seed), out.ctypes.data_as(ctypes.c_void_p))
    return out


def grid_medium(scene: Scene, density, n, world_to_medium=None) -> Scene:
    """Turn `scene`'s medium into a GridDensityMedium over `density` (n = (nx, ny, nz) or int).
    The array is kept alive on the scene object (the struct only holds its address)."""
    import numpy as np

    nx, ny, nz = (n, n, n) if isinstance(n, int) else tuple(n)
    dens = np.ascontiguousarray(density, np.float32).reshape(-1)
    assert dens.shape[0] == nx * ny * nz
    scene.has_medium = MEDIUM_GRID
    scene.grid_n = (ctypes.c_int32 * 3)(nx, ny, nz)
    m = np.eye(4, dtype=np.float32) if world_to_medium is None else np.asarray(world_to_medium, np.float32)
    scene.world_to_medium = (ctypes.c_float * 16)(*[float(v) for v in m.reshape(-1)])
    scene.grid_density = dens.ctypes.data
    scene._density_ref = dens
    return scene


def cornell_smoke_scene(sigma_a: float = 0.5, sigma_s: float = 4.5, g: float = 0.7, n: int = 64, seed: int = 7,
                        density=None) -> Scene:
    """the Cornell box filled (on its unit cube) with a GridDensityMedium of
    seeded value-noise smoke (bre_smoke_density(n, seed)), spectrally uniform sigma_t, HG g."""
    s = cornell_scene(sigma_a, sigma_s, g)
    return grid_medium(s, smoke_density(n, seed) if density is None else density, n)
