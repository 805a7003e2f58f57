// bre_pbrt_capi.cpp — the C ABI of include/bre_pbrt.h over pbrt_scene.h / photonbeam_gpu.h.
#include <cstring>
#include <string>

#include "../../include/bre_pbrt.h"
#include "photonbeam_gpu.h"

using namespace bre_host;

struct bre_pbrt {
    PbrtScene scene;
    bool ok = false;
};

static bre_status finish_parse(bre_pbrt *p, bool ok) {
    p->ok = ok;
    if (ok) p->scene.Bind();
    return ok ? BRE_OK : BRE_ERR_INVALID_ARG;
}

extern "C" {

bre_status bre_pbrt_parse_file(const char *path, bre_pbrt **out) {
    if (!out) return BRE_ERR_INVALID_ARG;
    *out = new bre_pbrt();
    if (!path) return BRE_ERR_INVALID_ARG;
    return finish_parse(*out, ParsePbrtFile(path, &(*out)->scene));
}

bre_status bre_pbrt_parse_string(const char *text, bre_pbrt **out) {
    if (!out) return BRE_ERR_INVALID_ARG;
    *out = new bre_pbrt();
    if (!text) return BRE_ERR_INVALID_ARG;
    return finish_parse(*out, ParsePbrtString(text, &(*out)->scene));
}

void bre_pbrt_free(bre_pbrt *p) { delete p; }

const char *bre_pbrt_messages(const bre_pbrt *p, int32_t *n_errors, int32_t *n_warnings) {
    if (!p) return "";
    if (n_errors) *n_errors = p->scene.errors;
    if (n_warnings) *n_warnings = p->scene.warnings;
    return p->scene.messages.c_str();
}

bre_status bre_pbrt_get_scene(const bre_pbrt *p, bre_scene *out) {
    if (!p || !out || !p->ok) return BRE_ERR_INVALID_ARG;
    *out = p->scene.scene;
    return BRE_OK;
}

static PhotonBeamParams params_of(const bre_pbrt *p, int32_t quick) {
    PhotonBeamParams::Lookup lk;
    const ParamSet &ps = p->scene.integratorParams;
    lk.findInt = [&](const char *n, int d) { return ps.FindOneInt(n, d); };
    lk.findFloat = [&](const char *n, float d) { return ps.FindOneFloat(n, d); };
    lk.findBool = [&](const char *n, bool d) { return ps.FindOneBool(n, d); };
    return PhotonBeamParams::FromLookup(lk, quick != 0, p->scene.film.xres * p->scene.film.yres);
}

bre_status bre_pbrt_get_render_params(const bre_pbrt *p, int32_t quick, bre_render_params *out,
                                      int32_t *write_frequency) {
    if (!p || !out || !p->ok) return BRE_ERR_INVALID_ARG;
    const PhotonBeamParams pp = params_of(p, quick);
    memset(out, 0, sizeof(*out));
    out->width = p->scene.film.xres;
    out->height = p->scene.film.yres;
    out->iterations = pp.nIterations;
    out->start_iteration = pp.startIteration;
    out->end_iteration = pp.endIteration;
    out->photons_per_iteration = pp.photonsPerIteration;
    out->max_depth = pp.maxDepth;
    out->render_surfaces = pp.renderSurfaces;
    out->render_media = pp.renderMedia;
    out->initial_radius = pp.initialBeamRadius;
    out->alpha = pp.alpha;
    if (write_frequency) *write_frequency = pp.writeFrequency;  // bre_render_progressive applies the reference's modulo
    return BRE_OK;
}

bre_status bre_pbrt_get_film(const bre_pbrt *p, int32_t *xres, int32_t *yres, float *scale, char *filename,
                             int32_t cap) {
    if (!p || !p->ok) return BRE_ERR_INVALID_ARG;
    if (xres) *xres = p->scene.film.xres;
    if (yres) *yres = p->scene.film.yres;
    if (scale) *scale = p->scene.film.scale;
    if (filename && cap > 0) {
        strncpy(filename, p->scene.film.filename.c_str(), (size_t)cap - 1);
        filename[cap - 1] = '\0';
    }
    return BRE_OK;
}

bre_status bre_pbrt_render(const bre_pbrt *p, int32_t device, int32_t quick, const char *outfile,
                           int32_t write_files, float *image_rgb) {
    if (!p || !p->ok) return BRE_ERR_INVALID_ARG;
    if (p->scene.integratorName != "photonbeam") return BRE_ERR_INVALID_ARG;
    FilmDesc film = p->scene.film;
    if (outfile) film.filename = outfile;
    PhotonBeamIntegrator integ(params_of(p, quick), film, device);
    if (!integ.Context()) return BRE_ERR_NO_DEVICE;
    integ.writeFiles = write_files != 0;
    if (!integ.Render(p->scene.scene)) return BRE_ERR_STATE;
    if (image_rgb && !integ.Image().empty())
        memcpy(image_rgb, integ.Image().data(), integ.Image().size() * sizeof(float));
    return BRE_OK;
}

bre_status bre_film_finalize(int64_t npix, const float *L, float scale, float *out) {
    if (npix < 0 || (npix > 0 && (!L || !out))) return BRE_ERR_INVALID_ARG;
    FilmFinalize(L, npix, scale, out);
    return BRE_OK;
}

bre_status bre_write_pfm(const char *path, const float *rgb, int32_t w, int32_t h) {
    if (!path || !rgb || w <= 0 || h <= 0) return BRE_ERR_INVALID_ARG;
    return WritePFM(path, rgb, w, h, nullptr) ? BRE_OK : BRE_ERR_STATE;
}

bre_status bre_read_pfm(const char *path, float *rgb, int64_t capacity, int32_t *w, int32_t *h) {
    if (!path) return BRE_ERR_INVALID_ARG;
    std::vector<float> img;
    int W = 0, H = 0;
    if (!ReadPFM(path, &img, &W, &H, nullptr)) return BRE_ERR_STATE;
    if (w) *w = W;
    if (h) *h = H;
    if (rgb && capacity > 0)
        memcpy(rgb, img.data(), (size_t)std::min<int64_t>(capacity, (int64_t)img.size()) * sizeof(float));
    return BRE_OK;
}

}  // extern "C"
