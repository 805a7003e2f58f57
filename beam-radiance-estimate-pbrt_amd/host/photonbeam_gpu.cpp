// photonbeam_gpu.cpp — see photonbeam_gpu.h.
#include "photonbeam_gpu.h"

#include <climits>
#include <cstdlib>
#include <cstring>

namespace bre_host {

void SegmentRecorder::Clear() {
    o_.clear();
    p_.clear();
    d_.clear();
    tmax_.clear();
    pixel_.clear();
}

void SegmentRecorder::Record(const CameraSegment &s) {
    o_.insert(o_.end(), {s.o.x, s.o.y, s.o.z});
    p_.insert(p_.end(), {s.p.x, s.p.y, s.p.z});
    d_.insert(d_.end(), {s.d.x, s.d.y, s.d.z});
    tmax_.push_back(s.tMax);
    pixel_.push_back(s.pixel);
}

void SegmentRecorder::Append(const SegmentRecorder &other) {
    o_.insert(o_.end(), other.o_.begin(), other.o_.end());
    p_.insert(p_.end(), other.p_.begin(), other.p_.end());
    d_.insert(d_.end(), other.d_.begin(), other.d_.end());
    tmax_.insert(tmax_.end(), other.tmax_.begin(), other.tmax_.end());
    pixel_.insert(pixel_.end(), other.pixel_.begin(), other.pixel_.end());
}

std::vector<int> DevicesFromEnv() {
    std::vector<int> out;
    const char *e = std::getenv("BRE_DEVICES");
    for (const char *q = e ? e : ""; *q;) {
        char *end = nullptr;
        const long v = std::strtol(q, &end, 10);
        if (end == q) break;
        out.push_back((int)v);
        q = *end == ',' ? end + 1 : end;
    }
    if (out.empty()) out.push_back(0);
    return out;
}

PhotonBeamGpuBVH::PhotonBeamGpuBVH(int device) : PhotonBeamGpuBVH(std::vector<int>{device}) {}

PhotonBeamGpuBVH::PhotonBeamGpuBVH(const std::vector<int> &devices) {
    if (devices.empty()) err_ = "no device given";
    for (int dev : devices) {
        bre_ctx *c = nullptr;
        const bre_status st = bre_create(dev, &c);
        if (st != BRE_OK) {
            err_ = "bre_create(" + std::to_string(dev) + ") failed with status " + std::to_string((int)st);
            break;
        }
        ctx_.push_back(c);
    }
    ready_ = !devices.empty() && ctx_.size() == devices.size();
}

PhotonBeamGpuBVH::~PhotonBeamGpuBVH() {
    for (bre_ctx *c : ctx_) bre_destroy(c);
}

bool PhotonBeamGpuBVH::Check(bre_status st) {
    if (st == BRE_OK) return true;
    err_ = ctx_.empty() ? "no context" : bre_last_error(ctx_[0]);
    return false;
}

bool PhotonBeamGpuBVH::SetOption(bre_option opt, int64_t value) {
    if (!Ok()) return false;
    for (bre_ctx *c : ctx_)
        if (!Check(bre_set_option(c, opt, value))) return false;
    return true;
}

bool PhotonBeamGpuBVH::Stats(bre_stats *out) const { return Ok() && bre_get_stats(ctx_[0], out) == BRE_OK; }

bool PhotonBeamGpuBVH::Build(const std::vector<PhotonBeam> &beams) {
    if (!Ok()) return false;
    const size_t n = beams.size();
    std::vector<float> s(3 * n), e(3 * n), r(n), pw(3 * n);
    for (size_t i = 0; i < n; ++i) {
        const PhotonBeam &b = beams[i];
        s[3 * i] = b.start.x; s[3 * i + 1] = b.start.y; s[3 * i + 2] = b.start.z;
        e[3 * i] = b.end.x; e[3 * i + 1] = b.end.y; e[3 * i + 2] = b.end.z;
        r[i] = b.radius;
        pw[3 * i] = b.powerEnd.x; pw[3 * i + 1] = b.powerEnd.y; pw[3 * i + 2] = b.powerEnd.z;
    }
    if (ctx_.size() == 1) return Check(bre_set_beams(ctx_[0], (int64_t)n, s.data(), e.data(), r.data(), pw.data()));
    return Check(bre_set_beams_sharded(ctx_.data(), (int)ctx_.size(), (int64_t)n, s.data(), e.data(), r.data(),
                                       pw.data()));
}

bool PhotonBeamGpuBVH::Gather(const SegmentRecorder &segs, float currentBeamRadius, std::vector<float> &pixelLd) {
    if (!Ok()) return false;
    const int64_t npix = (int64_t)(pixelLd.size() / 3);
    if (ctx_.size() == 1)
        return Check(bre_gather(ctx_[0], segs.Size(), segs.O(), segs.P(), segs.D(), segs.TMax(), segs.Pixel(),
                                currentBeamRadius, npix, pixelLd.data(), nullptr, nullptr));
    return Check(bre_gather_sharded(ctx_.data(), (int)ctx_.size(), segs.Size(), segs.O(), segs.P(), segs.D(),
                                    segs.TMax(), segs.Pixel(), currentBeamRadius, npix, pixelLd.data(), nullptr,
                                    nullptr));
}

bool PhotonBeamGpuBVH::Gather(const std::vector<SegmentRecorder> &recorders, float currentBeamRadius,
                              std::vector<float> &pixelLd) {
    merged_.Clear();
    for (const SegmentRecorder &r : recorders) merged_.Append(r);
    if (merged_.Size() == 0) return Ok();
    return Gather(merged_, currentBeamRadius, pixelLd);
}

PhotonBeamParams PhotonBeamParams::FromLookup(const Lookup &ps, bool quickRender, int pixelCount) {
    PhotonBeamParams p;
    p.nIterations = ps.findInt("iterations", ps.findInt("numiterations", 64));
    p.startIteration = ps.findInt("startiteration", 0);
    p.endIteration = ps.findInt("enditeration", p.nIterations);
    p.maxDepth = ps.findInt("maxdepth", 5);
    p.photonsPerIteration = ps.findInt("photonsperiteration", -1);
    p.writeFrequency = ps.findInt("imagewritefrequency", 1 << 31);
    p.initialBeamRadius = ps.findFloat("initialbeamradius", 1.f);
    p.alpha = ps.findFloat("alpha", 0.5f);
    // like the reference, --quick shrinks nIterations after endIteration was already defaulted
    if (quickRender) p.nIterations = p.nIterations / 16 > 1 ? p.nIterations / 16 : 1;
    p.renderSurfaces = ps.findBool("rendersurfaces", true);
    p.renderMedia = ps.findBool("rendermedia", true);
    if (p.photonsPerIteration <= 0) p.photonsPerIteration = pixelCount;
    return p;
}

float BeamRadiusAt(const PhotonBeamParams &p, int iteration) {
    return bre_beam_radius_at(p.initialBeamRadius, p.alpha, iteration);
}

void ResolveImage(const std::vector<float> &pixelLd, int iteration, std::vector<float> &rgb) {
    rgb.resize(pixelLd.size());
    bre_resolve_image((int64_t)(pixelLd.size() / 3), pixelLd.data(), iteration, rgb.data());
}

PhotonBeamIntegrator::PhotonBeamIntegrator(const PhotonBeamParams &params, const FilmDesc &film, int device)
    : params_(params), film_(film) {
    const bre_status st = bre_create(device, &ctx_);
    if (st != BRE_OK) {
        ctx_ = nullptr;
        err_ = "bre_create failed with status " + std::to_string((int)st);
    }
}

PhotonBeamIntegrator::~PhotonBeamIntegrator() { bre_destroy(ctx_); }

std::string PfmFilename(const std::string &filename) {
    const size_t dot = filename.find_last_of('.');
    const size_t slash = filename.find_last_of('/');
    if (dot != std::string::npos && (slash == std::string::npos || dot > slash)) {
        std::string ext = filename.substr(dot);
        for (auto &c : ext) c = (char)tolower((unsigned char)c);
        if (ext == ".pfm") return filename;
        return filename.substr(0, dot) + ".pfm";
    }
    return filename + ".pfm";
}

int PhotonBeamIntegrator::OnImage(int32_t, const float *L, void *user) {
    PhotonBeamIntegrator *self = static_cast<PhotonBeamIntegrator *>(user);
    const int64_t npix = (int64_t)self->film_.xres * self->film_.yres;
    self->image_.resize((size_t)npix * 3);
    FilmFinalize(L, npix, self->film_.scale, self->image_.data());  // Film::SetImage + WriteImage
    ++self->written_;
    if (!self->writeFiles) return 0;
    std::string err;
    if (!WritePFM(PfmFilename(self->film_.filename), self->image_.data(), self->film_.xres, self->film_.yres, &err)) {
        self->err_ = err;
        return 1;
    }
    return 0;
}

bool PhotonBeamIntegrator::Render(const bre_scene &scene) {
    if (!ctx_) return false;
    bre_render_params rp;
    memset(&rp, 0, sizeof(rp));
    rp.width = film_.xres;
    rp.height = film_.yres;
    rp.iterations = params_.nIterations;
    rp.start_iteration = params_.startIteration;
    rp.end_iteration = params_.endIteration;
    rp.photons_per_iteration = params_.photonsPerIteration;
    rp.max_depth = params_.maxDepth;
    rp.render_surfaces = params_.renderSurfaces;
    rp.render_media = params_.renderMedia;
    rp.initial_radius = params_.initialBeamRadius;
    rp.alpha = params_.alpha;
    written_ = 0;
    // the reference's default 1 << 31 is INT_MIN, which never divides iter + 1: "at the end only"
    const int32_t wf = params_.writeFrequency;  // the reference's (iter + 1) % writeFrequency, negatives included
    const bre_status st = bre_render_progressive(ctx_, &scene, &rp, wf, &PhotonBeamIntegrator::OnImage, this);
    if (st != BRE_OK) {
        if (err_.empty()) err_ = bre_last_error(ctx_);
        return false;
    }
    return true;
}

std::unique_ptr<PhotonBeamIntegrator> CreatePhotonBeamIntegrator(const ParamSet &params, const FilmDesc &film,
                                                                 bool quickRender, int device) {
    PhotonBeamParams::Lookup lk;
    lk.findInt = [&](const char *n, int d) { return params.FindOneInt(n, d); };
    lk.findFloat = [&](const char *n, float d) { return params.FindOneFloat(n, d); };
    lk.findBool = [&](const char *n, bool d) { return params.FindOneBool(n, d); };
    const PhotonBeamParams p = PhotonBeamParams::FromLookup(lk, quickRender, film.xres * film.yres);
    return std::unique_ptr<PhotonBeamIntegrator>(new PhotonBeamIntegrator(p, film, device));
}

}  // namespace bre_host
