/*
 * bre_scene.h — scene description for the on-device photon pass and camera pass.
 *
 * The gather (bre.h) consumes beams and camera segments; this header describes the scene that
 * produces them, so the photon pass (TracePhotonBeamRecursive + emission,
 * src/integrators/photonbeam.cpp:258-325, 383-421) and the camera pass
 * (photonbeam.cpp:456-555) can run on the GPU next to the gather.
 *
 * The scene model is deliberately the subset the benchmark scene of SURVEY.md §8d (C1/C2: a
 * Cornell box of matte quads, one diffuse area light, a homogeneous fog filling the box, a
 * pinhole camera inside the fog) needs:
 *   - bre_quad          parallelograms p0 + u*e1 + v*e2, u,v in [0,1], with a Lambertian
 *                       reflectance (MatteMaterial with sigma 0, src/materials/matte.cpp;
 *                       black kd = no BxDF, so a photon hitting it is absorbed,
 *                       reflection.cpp:708-713).  Geometric = shading normal =
 *                       normalize(e1 x e2); the shading tangent ss = normalize(e1).
 *   - one diffuse area light (DiffuseAreaLight, one-sided, src/lights/diffuse.cpp:89-123) on
 *                       quad `light_quad`, emitting light_L towards +normal.
 *   - an optional medium filling all of space (every ray -- camera, photon, spawned -- travels
 *                       in it) with a Henyey-Greenstein phase function (src/core/medium.cpp:194-213):
 *                       BRE_MEDIUM_HOMOGENEOUS = HomogeneousMedium (src/media/homogeneous.cpp:44-77),
 *                       BRE_MEDIUM_GRID = GridDensityMedium (src/media/grid.{h:50-100,cpp:46-120}):
 *                       trilinear density over an nx*ny*nz grid on the medium-space unit cube, delta
 *                       tracking (Sample) and ratio tracking with Russian roulette (Tr); both draw
 *                       from the path's sampler.  sigma_a + sigma_s must be spectrally uniform.
 *   - a perspective pinhole camera (src/cameras/perspective.cpp, lensradius 0).
 * Geometry contract shared by the GPU pass and the oracle (both evaluate it with IEEE float,
 * no FMA contraction): see DESIGN.md "Photon pass".
 */
#ifndef BRE_SCENE_H
#define BRE_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BRE_MAX_QUADS 64
#define BRE_MAX_DEPTH 16 /* maxdepth accepted by the photon / camera passes */

#define BRE_MEDIUM_NONE 0
#define BRE_MEDIUM_HOMOGENEOUS 1
#define BRE_MEDIUM_GRID 2
#define BRE_MAX_GRID_CELLS (1 << 26) /* nx*ny*nz accepted for a GridDensityMedium */

typedef struct bre_quad {
    float p0[3]; /* corner */
    float e1[3]; /* edge u (shading tangent direction) */
    float e2[3]; /* edge v; normal = normalize(e1 x e2) */
    float kd[3]; /* Lambertian reflectance; all-zero = absorbing (no BxDF) */
} bre_quad;

typedef struct bre_scene {
    int32_t n_quads;       /* 1 .. BRE_MAX_QUADS */
    int32_t light_quad;    /* index of the emitting quad */
    float light_L[3];      /* DiffuseAreaLight "L" (Lemit) */
    int32_t has_medium;    /* BRE_MEDIUM_NONE (vacuum) / _HOMOGENEOUS / _GRID, filling all space */
    float sigma_a[3];      /* medium sigma_a (already multiplied by "scale") */
    float sigma_s[3];      /* medium sigma_s */
    float g;               /* Henyey-Greenstein asymmetry */
    float cam_pos[3];      /* LookAt eye */
    float cam_look[3];     /* LookAt target */
    float cam_up[3];       /* LookAt up */
    float cam_fov_deg;     /* perspective "fov" (degrees, spans the shorter image axis) */
    bre_quad quads[BRE_MAX_QUADS];
    /* GridDensityMedium only (has_medium == BRE_MEDIUM_GRID; MakeMedium "heterogeneous",
       api.cpp:547-593): */
    int32_t grid_n[3];          /* nx, ny, nz (each >= 1, product <= BRE_MAX_GRID_CELLS) */
    float world_to_medium[16];  /* WorldToMedium = Inverse(mediumToWorld * Translate(p0) *
                                   Scale(p1 - p0)), row-major 4x4 (grid.h:58) */
    const float *grid_density;  /* nx*ny*nz densities, index (z*ny + y)*nx + x (grid.h:84-88);
                                   caller-owned host memory, read during the call */
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

/* The benchmark scene of SURVEY.md §8d (C1/C2): unit-cube Cornell box (white floor, ceiling and
   back wall, red left wall, green right wall, white front wall behind the camera), a 0.3 x 0.3
   area light just below the ceiling facing down, homogeneous fog sigma_a, sigma_s (grey), HG g,
   camera at (0.5, 0.5, 0.02) looking at (0.5, 0.5, 1) with a 60 degree field of view. */
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
