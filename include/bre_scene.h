/*
 * bre_scene.h — scene description for the on-device photon pass and camera pass.
 *
 * The gather (bre.h) consumes beams and camera segments; this header describes the scene that
 * produces them, so the photon pass (TracePhotonBeamRecursive + emission,
 * src/integrators/photonbeam.cpp:258-325, 383-421) and the camera pass
 * (photonbeam.cpp:456-555) can run on the GPU next to the gather.
 *
 * The scene model is the subset of pbrt-v3 the benchmark scenes of SURVEY.md §8d need, kept at
 * pbrt's own granularity so every random decision and every float matches the reference:
 *   - bre_triangle      one pbrt Triangle of a "trianglemesh" (src/shapes/triangle.cpp): its three
 *                       world-space vertices in the mesh's index order, hit by the watertight
 *                       Triangle::Intersect (:177-300), with the triangle's own geometric normal
 *                       normalize(cross(p0 - p2, p1 - p2)) and shading frame ss = normalize(p1 - p0)
 *                       (dpdu for pbrt's default (0,0), (1,0), (1,1) uvs, :276-294), and a
 *                       Lambertian reflectance (MatteMaterial with sigma 0, src/materials/matte.cpp;
 *                       black kd = no BxDF, so a photon hitting it is absorbed,
 *                       reflection.cpp:708-713).  `flip` = ReverseOrientation ^
 *                       TransformSwapsHandedness (the normal is negated, :296-297).
 *   - diffuse area lights: every triangle with `emit` set is its own one-sided DiffuseAreaLight
 *                       (src/lights/diffuse.cpp:89-123; pbrtShape makes one light per shape of an
 *                       emitting mesh, api.cpp), in triangle order = scene.lights order.  The photon
 *                       pass picks one by power (ComputeLightPowerDistribution,
 *                       integrator.cpp:217-225); the camera pass uniformly (UniformSampleOneLight).
 *   - an optional medium filling all of space (every ray -- camera, photon, spawned -- travels
 *                       in it) with a Henyey-Greenstein phase function (src/core/medium.cpp:194-213):
 *                       BRE_MEDIUM_HOMOGENEOUS = HomogeneousMedium (src/media/homogeneous.cpp:44-77),
 *                       BRE_MEDIUM_GRID = GridDensityMedium (src/media/grid.{h:50-100,cpp:46-120}):
 *                       trilinear density over an nx*ny*nz grid on the medium-space unit cube, delta
 *                       tracking (Sample) and ratio tracking with Russian roulette (Tr); both draw
 *                       from the path's sampler.  sigma_a + sigma_s must be spectrally uniform.
 *   - a perspective pinhole camera (src/cameras/perspective.cpp, lensradius 0).
 * The GPU passes and the oracle evaluate it with IEEE float, no FMA contraction (DESIGN.md
 * "Photon pass").
 */
#ifndef BRE_SCENE_H
#define BRE_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BRE_MAX_TRIANGLES 128               /* triangles held inline in bre_scene.triangles */
#define BRE_MAX_SCENE_TRIANGLES (1 << 24)  /* triangles through bre_scene.triangles_ext */
#define BRE_MAX_DEPTH 16 /* maxdepth accepted by the photon / camera passes */

#define BRE_MEDIUM_NONE 0
#define BRE_MEDIUM_HOMOGENEOUS 1
#define BRE_MEDIUM_GRID 2
#define BRE_MAX_GRID_CELLS (1 << 26) /* nx*ny*nz accepted for a GridDensityMedium */

typedef struct bre_triangle {
    float p[3][3]; /* world-space vertices mesh->p[v[0..2]] (ObjectToWorld applied) */
    float kd[3];   /* Lambertian reflectance; all-zero = absorbing (no BxDF) */
    float Le[3];   /* DiffuseAreaLight "L" (Lemit) when emit != 0 */
    int32_t emit;  /* 1: a one-sided diffuse area light */
    int32_t flip;  /* 1: ReverseOrientation ^ TransformSwapsHandedness (normal negated) */
} bre_triangle;

typedef struct bre_scene {
    int32_t n_triangles;   /* 1 .. BRE_MAX_TRIANGLES inline, or 1 .. BRE_MAX_SCENE_TRIANGLES through
                              triangles_ext; at least one with emit != 0 */
    int32_t has_medium;    /* BRE_MEDIUM_NONE (vacuum) / _HOMOGENEOUS / _GRID, filling all space */
    float sigma_a[3];      /* medium sigma_a (already multiplied by "scale") */
    float sigma_s[3];      /* medium sigma_s */
    float g;               /* Henyey-Greenstein asymmetry */
    float cam_pos[3];      /* LookAt eye */
    float cam_look[3];     /* LookAt target */
    float cam_up[3];       /* LookAt up */
    float cam_fov_deg;     /* perspective "fov" (degrees, spans the shorter image axis) */
    bre_triangle triangles[BRE_MAX_TRIANGLES];
    /* GridDensityMedium only (has_medium == BRE_MEDIUM_GRID; MakeMedium "heterogeneous",
       api.cpp:547-593): */
    int32_t grid_n[3];          /* nx, ny, nz (each >= 1, product <= BRE_MAX_GRID_CELLS) */
    float world_to_medium[16];  /* WorldToMedium = Inverse(mediumToWorld * Translate(p0) *
                                   Scale(p1 - p0)), row-major 4x4 (grid.h:58) */
    const float *grid_density;  /* nx*ny*nz densities, index (z*ny + y)*nx + x (grid.h:84-88);
                                   caller-owned host memory, read during the call */
    /* Any number of triangles (BRE_MAX_SCENE_TRIANGLES): when non-NULL, the scene's triangles are
       triangles_ext[0 .. n_triangles) (caller-owned host memory, read during the call) and the
       inline array is unused.  Either way the passes intersect the scene through pbrt's BVHAccel
       (src/accelerators/bvh.cpp: SAH, 12 buckets, maxnodeprims 4 -- the "bvh" accelerator's
       defaults, CreateBVHAccelerator), built on the host over the triangles in scene order, so
       equal-distance hits resolve in the reference's order. */
    const bre_triangle *triangles_ext;
} bre_scene;

/* PhotonBeamIntegrator parameters (CreatePhotonBeamIntegrator, photonbeam.cpp:589-611). */
typedef struct bre_render_params {
    int32_t width, height;          /* film resolution (pixelBounds = [0,W) x [0,H)) */
    int32_t iterations;             /* "iterations" (default 64) */
    int32_t start_iteration;        /* "startiteration" (default 0) */
    int32_t end_iteration;          /* "enditeration" (default = iterations) */
    int64_t photons_per_iteration;  /* "photonsperiteration"; <= 0: width * height (photonbeam.h:37-39) */
    int32_t max_depth;              /* "maxdepth" (default 5) */
    int32_t render_surfaces;        /* "rendersurfaces" (default 1) */
    int32_t render_media;           /* "rendermedia" (default 1) */
    float initial_radius;           /* "initialbeamradius" (default 1) */
    float alpha;                    /* "alpha" (default 0.5) */
} bre_render_params;

/* The benchmark scene of SURVEY.md §8d (C1/C2), scenes/cornell_world.pbrt: unit-cube Cornell box
   (white floor, ceiling and back wall, red left wall, green right wall, white front wall behind
   the camera), a 0.3 x 0.3 area light just below the ceiling facing down, each wall one
   "trianglemesh" of two triangles (v0 v1 v2)(v0 v2 v3), homogeneous fog sigma_a, sigma_s (grey),
   HG g, camera at (0.5, 0.5, 0.02) looking at (0.5, 0.5, 1) with a 60 degree field of view. */
void bre_scene_cornell(bre_scene *scene, float sigma_a, float sigma_s, float g);

/* SURVEY.md §8d C3/C5 smoke: the same Cornell box with a GridDensityMedium of sigma_a, sigma_s
   (grey) and HG g over the box's unit cube (world_to_medium = identity); `density` (n^3 floats,
   caller-owned, must outlive the scene's use) is filled with bre_smoke_density's seeded value
   noise. */
void bre_scene_cornell_smoke(bre_scene *scene, float sigma_a, float sigma_s, float g, int32_t n,
                             const float *density);
/* Seeded value-noise smoke density (n^3 floats, x fastest): 3 octaves of trilinear lattice noise
   from PCG32(seed), shaped by a soft sphere of radius 0.45 around the box centre, >= 0. */
void bre_smoke_density(int32_t n, uint64_t seed, float *density);

#ifdef __cplusplus
}
#endif

#endif /* BRE_SCENE_H */
