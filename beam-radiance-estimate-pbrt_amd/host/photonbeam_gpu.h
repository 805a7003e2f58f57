// photonbeam_gpu.h — host-side C++ mirror of the reference's photon-beam integrator surface,
// driving libbre.so through the C ABI (include/bre.h).
//
// Reference interface mirrored (bwiberg/beam-radiance-estimate-pbrt):
//   struct PhotonBeam                          src/core/photonbeambvh.h:48-73
//   PhotonBeamBVH(vector<shared_ptr<..>>&&)    src/core/photonbeambvh.h:91-99  -> PhotonBeamGpuBVH
//   Intersect(ray) + gather loop body           src/integrators/photonbeam.cpp:494-508
//                                              -> SegmentRecorder::Record + PhotonBeamGpuBVH::Gather
//   CreatePhotonBeamIntegrator ParamSet lookups src/integrators/photonbeam.cpp:589-611
//                                              -> PhotonBeamParams::FromLookup
//   radius schedule / image resolve            photonbeam.cpp:354-356, 562, 578
//
// Errors: pbrt reports with Error() and continues; here every failing call throws nothing and
// returns false with the libbre message in LastError(), so a caller can map it to Error().
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/bre.h"
#include "pbrt_scene.h"

namespace bre_host {

struct Float3 {
    float x = 0, y = 0, z = 0;
};

// Mirror of pbrt::PhotonBeam (powerStart kept for layout fidelity; the reference always sets it
// to black and the gather never reads it).
struct PhotonBeam {
    Float3 start, end;
    float radius = 0;
    Float3 powerStart, powerEnd;
};

// One camera-ray segment of the camera pass: ray.o, ray.d, ray.tMax after Scene::Intersect, the
// hit point isect.p, and the pixel it belongs to (photonbeam.cpp:474-477, 481, 495-499).
struct CameraSegment {
    Float3 o, p, d;
    float tMax = 0;
    int32_t pixel = 0;
};

// Records the segments of one iteration's camera pass in SoA form, ready for one bre_gather call.
// The gather result never feeds back into the camera path (photonbeam.cpp:494-510), so deferring
// every segment of the iteration to one batched call is semantically identical.
class SegmentRecorder {
  public:
    void Clear();
    void Record(const CameraSegment &s);
    // Append another recorder's segments (the per-thread recorders of one pass into one batch).
    void Append(const SegmentRecorder &other);
    int64_t Size() const { return (int64_t)tmax_.size(); }
    const float *O() const { return o_.data(); }
    const float *P() const { return p_.data(); }
    const float *D() const { return d_.data(); }
    const float *TMax() const { return tmax_.data(); }
    const int32_t *Pixel() const { return pixel_.data(); }

  private:
    std::vector<float> o_, p_, d_, tmax_;
    std::vector<int32_t> pixel_;
};

// GPU replacement of PhotonBeamBVH for one iteration's beam set, on one or several GPUs.
class PhotonBeamGpuBVH {
  public:
    explicit PhotonBeamGpuBVH(int device = 0);
    // One libbre context per entry of `devices` (one per GPU; a repeated ordinal puts several
    // contexts on one device): Build replicates the beam set on every device, Gather deals the
    // coherence-sorted segment packets round-robin over them and sums their films on the host
    // (bre_set_beams_sharded / bre_gather_sharded).  This is how a single pbrt process uses all
    // GPUs of a node without Python or RCCL.
    explicit PhotonBeamGpuBVH(const std::vector<int> &devices);
    ~PhotonBeamGpuBVH();
    PhotonBeamGpuBVH(const PhotonBeamGpuBVH &) = delete;
    PhotonBeamGpuBVH &operator=(const PhotonBeamGpuBVH &) = delete;

    bool Ok() const { return ready_; }
    int Devices() const { return (int)ctx_.size(); }
    // Replaces `PhotonBeamBVH photonBeamBVH(std::move(photonBeams))` (photonbeam.cpp:438).
    bool Build(const std::vector<PhotonBeam> &beams);
    // Replaces the per-segment Intersect + contribution loop (photonbeam.cpp:494-508) for all
    // recorded segments; adds into pixelLd (3 floats per pixel), like PhotonBeamPixel::Ld.
    bool Gather(const SegmentRecorder &segs, float currentBeamRadius, std::vector<float> &pixelLd);
    // The same for every recorder of an iteration (the camera pass's per-thread recorders) in ONE
    // batched call, so the whole iteration is sorted into coherent packets and the film crosses
    // PCIe once per iteration.
    bool Gather(const std::vector<SegmentRecorder> &recorders, float currentBeamRadius, std::vector<float> &pixelLd);
    bool SetOption(bre_option opt, int64_t value);
    bool Stats(bre_stats *out) const;
    const std::string &LastError() const { return err_; }

  private:
    bool Check(bre_status st);
    std::vector<bre_ctx *> ctx_;
    bool ready_ = false;      // every context was created
    SegmentRecorder merged_;  // concatenation buffer of Gather(recorders)
    std::string err_;
};

// The GPU ordinals of the BRE_DEVICES environment variable ("0,1,2,3"; default "0"): the
// adapter patch's one-process multi-GPU switch.
std::vector<int> DevicesFromEnv();

// Integrator parameters with the reference's names and defaults (photonbeam.cpp:591-604).
struct PhotonBeamParams {
    int nIterations = 64;
    int startIteration = 0;
    int endIteration = 64;
    int maxDepth = 5;
    int photonsPerIteration = -1;  // -1 -> pixel count (photonbeam.h:37-39)
    int writeFrequency = 1 << 31;  // as written in the reference (INT_MIN after overflow)
    float initialBeamRadius = 1.f;
    float alpha = 0.5f;
    bool renderSurfaces = true;
    bool renderMedia = true;

    // Lookup callbacks stand in for pbrt's ParamSet::FindOneInt/Float/Bool.
    struct Lookup {
        std::function<int(const char *, int)> findInt;
        std::function<float(const char *, float)> findFloat;
        std::function<bool(const char *, bool)> findBool;
    };
    static PhotonBeamParams FromLookup(const Lookup &ps, bool quickRender, int pixelCount);
};

// currentBeamRadius at the start of `iteration` (photonbeam.cpp:354-356, 562).
float BeamRadiusAt(const PhotonBeamParams &p, int iteration);
// L = Ld / (iter + 1) per pixel (photonbeam.cpp:578).
void ResolveImage(const std::vector<float> &pixelLd, int iteration, std::vector<float> &rgb);

// Mirror of pbrt::PhotonBeamIntegrator (photonbeam.h:18-60) with Render (photonbeam.cpp:329-586)
// running on the GPU through bre_render_progressive: per iteration the photon pass, BVH build,
// camera pass and gather stay in HBM; at the reference's write schedule (:564-584) the image
// L = Ld / (iter + 1) goes through Film::SetImage + Film::WriteImage (FilmFinalize) and is
// written to the film's file as PFM.
class PhotonBeamIntegrator {
  public:
    PhotonBeamIntegrator(const PhotonBeamParams &params, const FilmDesc &film, int device = 0);
    ~PhotonBeamIntegrator();
    PhotonBeamIntegrator(const PhotonBeamIntegrator &) = delete;
    PhotonBeamIntegrator &operator=(const PhotonBeamIntegrator &) = delete;

    // Integrator::Render(const Scene &): false (with LastError) on any failure.
    bool Render(const bre_scene &scene);
    // The last image handed to the film, after WriteImage's conversion (top row first, 3 floats
    // per pixel), and how many times the film was written.
    const std::vector<float> &Image() const { return image_; }
    int ImagesWritten() const { return written_; }
    const PhotonBeamParams &Params() const { return params_; }
    const FilmDesc &Film() const { return film_; }
    bool writeFiles = true;  // false: keep the images in memory only (tests)
    bre_ctx *Context() { return ctx_; }
    const std::string &LastError() const { return err_; }

  private:
    static int OnImage(int32_t iteration, const float *L, void *self);
    PhotonBeamParams params_;
    FilmDesc film_;
    bre_ctx *ctx_ = nullptr;
    std::vector<float> image_;
    int written_ = 0;
    std::string err_;
};

// CreatePhotonBeamIntegrator(const ParamSet &, shared_ptr<const Camera>) (photonbeam.cpp:589-611):
// the camera's film supplies the pixel count for photonsperiteration's default.
std::unique_ptr<PhotonBeamIntegrator> CreatePhotonBeamIntegrator(const ParamSet &params, const FilmDesc &film,
                                                                 bool quickRender = false, int device = 0);

// The PFM name the film is written to: the film's filename with a .pfm extension (this build
// writes PFM only; pbrt picks the writer by extension, imageio.cpp WriteImage).
std::string PfmFilename(const std::string &filename);

}  // namespace bre_host
