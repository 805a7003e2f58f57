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
 *   - an optional HomogeneousMedium (src/media/homogeneous.cpp:44-77) with a Henyey-Greenstein
 *                       phase function (src/core/medium.cpp:194-213) filling all of space: every
 *                       ray (camera, photon, spawned) travels in it.
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
    int32_t has_medium;    /* 0 = vacuum, 1 = homogeneous medium everywhere */
    float sigma_a[3];      /* HomogeneousMedium sigma_a (already multiplied by "scale") */
    float sigma_s[3];      /* HomogeneousMedium sigma_s */
    float g;               /* Henyey-Greenstein asymmetry */
    float cam_pos[3];      /* LookAt eye */
    float cam_look[3];     /* LookAt target */
    float cam_up[3];       /* LookAt up */
    float cam_fov_deg;     /* perspective "fov" (degrees, spans the shorter image axis) */
    bre_quad quads[BRE_MAX_QUADS];
} bre_scene;

/* PhotonBeamIntegrator parameters (CreatePhotonBeamIntegrator, photonbeam.cpp:589-611). */
typedef struct bre_render_params {
    int32_t width, height;          /* film resolution (pixelBounds = [0,W) x [0,H)) */
    int32_t iterations;             /* "iterations" (default 64) */
    int32_t start_iteration;        /* "startiteration" (default 0) */
    int32_t end_iteration;          /* "enditeration" (default = iterations) */
    int64_t photons_per_iteration;  /* "photonsperiteration" */
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

#ifdef __cplusplus
}
#endif

#endif /* BRE_SCENE_H */
