/*
 * bre_pbrt.h — C ABI of libbre_host.so: the .pbrt scene-format front end and the film output of
 * the photon-beam integrator, over the GPU integrator of bre.h.
 *
 *   reference (pbrt-v3 fork)                                  this ABI
 *   --------------------------------------------------------  --------------------------------
 *   pbrtParseFile / pbrtParseString (src/core/parser.h,       bre_pbrt_parse_file /
 *     pbrtparse.y, api.cpp:765-1361)                            bre_pbrt_parse_string
 *   RenderOptions::MakeIntegrator "photonbeam"                bre_pbrt_get_render_params
 *     (api.cpp:1463-1471) -> CreatePhotonBeamIntegrator
 *     (photonbeam.cpp:589-611)
 *   pbrtWorldEnd -> integrator->Render(*scene)                bre_pbrt_render
 *     (api.cpp:1361-1380, photonbeam.cpp:329-586)
 *   Film::SetImage + Film::WriteImage (film.cpp:132-210)      bre_film_finalize
 *   WriteImagePFM / ReadImagePFM (imageio.cpp:437-482)        bre_write_pfm / bre_read_pfm
 *
 * The accepted subset of the scene format is documented in host/pbrt_scene.h.  Problems in a
 * statement are reported pbrt-style (text in bre_pbrt_messages) and the statement is skipped;
 * a scene the GPU model cannot render fails the parse with BRE_ERR_INVALID_ARG.
 */
#ifndef BRE_PBRT_H
#define BRE_PBRT_H

#include <stdint.h>

#include "bre.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bre_pbrt bre_pbrt;

/* Parse a scene.  *out is always set (free it with bre_pbrt_free) so that the messages of a
   failed parse can be read; BRE_OK iff the scene is renderable. */
bre_status bre_pbrt_parse_file(const char *path, bre_pbrt **out);
bre_status bre_pbrt_parse_string(const char *text, bre_pbrt **out);
void bre_pbrt_free(bre_pbrt *p);
/* Error()/Warning() text, one message per line; counts may be NULL. */
const char *bre_pbrt_messages(const bre_pbrt *p, int32_t *n_errors, int32_t *n_warnings);
/* The scene for bre_trace_photons / bre_camera_pass / bre_render; grid_density and (for more than
   BRE_MAX_TRIANGLES triangles) triangles_ext point into the parsed scene and stay valid until
   bre_pbrt_free. */
bre_status bre_pbrt_get_scene(const bre_pbrt *p, bre_scene *out);
/* CreatePhotonBeamIntegrator's parameters for the film of the scene (quick != 0 is pbrt's
   --quick); *write_frequency (may be NULL) receives "imagewritefrequency" as given (default 1 << 31 =
   INT32_MIN, never periodic; bre_render_progressive applies the reference's (iter + 1) % k test). */
bre_status bre_pbrt_get_render_params(const bre_pbrt *p, int32_t quick, bre_render_params *out,
                                      int32_t *write_frequency);
/* Film "image" resolution, scale and output file name (NUL-terminated, truncated to cap). */
bre_status bre_pbrt_get_film(const bre_pbrt *p, int32_t *xres, int32_t *yres, float *scale, char *filename,
                             int32_t cap);
/* The whole render on GPU `device`: BRE_ERR_INVALID_ARG unless the scene's Integrator is
   "photonbeam".  Writes the film (PFM, to outfile when non-NULL, else the film's filename with a
   .pfm extension) at every write of the reference's schedule unless write_files is 0; the last
   film image (after Film::WriteImage's conversion, top row first) goes to image_rgb
   (float[3*xres*yres], may be NULL). */
bre_status bre_pbrt_render(const bre_pbrt *p, int32_t device, int32_t quick, const char *outfile,
                           int32_t write_files, float *image_rgb);
/* Film::SetImage(L) + Film::WriteImage's per-pixel conversion with the film's scale. */
bre_status bre_film_finalize(int64_t npix, const float *L_rgb, float scale, float *out_rgb);
/* PFM file IO (rows top-first in memory, bottom-first on disk, little endian). bre_read_pfm
   writes at most capacity floats; width/height are always returned when the header parses. */
bre_status bre_write_pfm(const char *path, const float *rgb, int32_t width, int32_t height);
bre_status bre_read_pfm(const char *path, float *rgb, int64_t capacity, int32_t *width, int32_t *height);

#ifdef __cplusplus
}
#endif
#endif /* BRE_PBRT_H */
