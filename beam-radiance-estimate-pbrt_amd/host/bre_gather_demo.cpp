// bre_gather_demo.cpp — C++ host program using the integrator mirror (photonbeam_gpu.h) the way
// adapters/pbrt/photonbeam.patch does: build the iteration's beams (PhotonBeamGpuBVH::Build,
// photonbeam.cpp:438), record camera segments in per-thread SegmentRecorders (:494-508), one
// batched Gather of all recorders into the pixel Ld buffer, ResolveImage (:578).
//
//   bre_gather_demo [W]                      built-in lattice scene, prints the image sum
//   bre_gather_demo --beams B --segments S --out O [--split K] [--iteration I] [--devices D]
//       B: int64 n, then n x {start xyz, end xyz, radius, powerEnd rgb} float32
//       S: int64 n, int64 nPixels, float32 R, then n x {o xyz, p xyz, d xyz, tMax} float32 + int32 pixel
//       O: nPixels x rgb float32, the resolved image L = Ld / (I + 1)
//       K: number of recorders the segments are dealt to round-robin (the patch's per-thread
//          recorders), all gathered in one call
//       D: GPU ordinals separated by commas, one libbre context each (e.g. 0,1,2,3; 0,0,0 puts three
//          contexts on GPU 0): the beams are replicated and the segment packets split over them
// Exit code 0 on success, 1 on a libbre or IO error, 2 without a GPU.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "photonbeam_gpu.h"

using namespace bre_host;

namespace {

template <typename T>
bool ReadAll(FILE *f, T *dst, size_t n) {
    return std::fread(dst, sizeof(T), n, f) == n;
}

int FileMode(const char *beamsPath, const char *segPath, const char *outPath, int split, int iteration,
             const std::vector<int> &devices) {
    FILE *fb = std::fopen(beamsPath, "rb");
    FILE *fs = std::fopen(segPath, "rb");
    if (!fb || !fs) {
        std::fprintf(stderr, "bre_gather_demo: cannot open %s\n", !fb ? beamsPath : segPath);
        return 1;
    }
    int64_t nb = 0, ns = 0, npix = 0;
    float R = 0;
    if (!ReadAll(fb, &nb, 1) || nb < 0 || !ReadAll(fs, &ns, 1) || !ReadAll(fs, &npix, 1) || !ReadAll(fs, &R, 1) ||
        ns < 0 || npix <= 0) {
        std::fprintf(stderr, "bre_gather_demo: bad header\n");
        return 1;
    }
    std::vector<PhotonBeam> beams((size_t)nb);
    for (auto &b : beams) {
        float v[10];
        if (!ReadAll(fb, v, 10)) {
            std::fprintf(stderr, "bre_gather_demo: short beam file\n");
            return 1;
        }
        b.start = {v[0], v[1], v[2]};
        b.end = {v[3], v[4], v[5]};
        b.radius = v[6];
        b.powerEnd = {v[7], v[8], v[9]};
    }
    std::vector<SegmentRecorder> recorders((size_t)(split > 0 ? split : 1));
    for (int64_t i = 0; i < ns; ++i) {
        float v[10];
        int32_t pixel;
        if (!ReadAll(fs, v, 10) || !ReadAll(fs, &pixel, 1)) {
            std::fprintf(stderr, "bre_gather_demo: short segment file\n");
            return 1;
        }
        CameraSegment s;
        s.o = {v[0], v[1], v[2]};
        s.p = {v[3], v[4], v[5]};
        s.d = {v[6], v[7], v[8]};
        s.tMax = v[9];
        s.pixel = pixel;
        recorders[(size_t)(i % (int64_t)recorders.size())].Record(s);
    }
    std::fclose(fb);
    std::fclose(fs);

    PhotonBeamGpuBVH bvh(devices);
    if (!bvh.Ok()) {
        std::fprintf(stderr, "no GPU: %s\n", bvh.LastError().c_str());
        return 2;
    }
    if (!bvh.Build(beams)) {
        std::fprintf(stderr, "build: %s\n", bvh.LastError().c_str());
        return 1;
    }
    std::vector<float> ld(3 * (size_t)npix, 0.f);
    if (!bvh.Gather(recorders, R, ld)) {
        std::fprintf(stderr, "gather: %s\n", bvh.LastError().c_str());
        return 1;
    }
    std::vector<float> rgb;
    ResolveImage(ld, iteration, rgb);
    FILE *fo = std::fopen(outPath, "wb");
    if (!fo || std::fwrite(rgb.data(), sizeof(float), rgb.size(), fo) != rgb.size()) {
        std::fprintf(stderr, "bre_gather_demo: cannot write %s\n", outPath);
        return 1;
    }
    std::fclose(fo);
    bre_stats st;
    if (bvh.Stats(&st))
        std::printf("bre_gather_demo: %lld beams, %lld segments from %zu recorders in one gather on %d contexts, "
                    "%lld nodes\n", (long long)nb, (long long)ns, recorders.size(), bvh.Devices(),
                    (long long)st.n_nodes);
    return 0;
}

int LatticeMode(int W) {
    const int H = W;
    PhotonBeamParams params;
    params.initialBeamRadius = 0.02f;
    std::vector<PhotonBeam> beams;
    // a lattice of diagonal beams through the unit cube
    for (int i = 0; i < 24; ++i)
        for (int j = 0; j < 24; ++j) {
            PhotonBeam b;
            b.start = {i / 24.f, j / 24.f, 0.05f};
            b.end = {i / 24.f + 0.1f, j / 24.f + 0.05f, 0.9f};
            b.radius = BeamRadiusAt(params, 0);
            b.powerEnd = {1.f, 0.5f, 0.25f};
            beams.push_back(b);
        }
    PhotonBeamGpuBVH bvh(0);
    if (!bvh.Ok()) {
        std::fprintf(stderr, "no GPU: %s\n", bvh.LastError().c_str());
        return 2;
    }
    if (!bvh.Build(beams)) {
        std::fprintf(stderr, "build: %s\n", bvh.LastError().c_str());
        return 1;
    }
    SegmentRecorder rec;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            CameraSegment s;
            s.o = {0.5f, 0.5f, -1.f};
            float qx = (x + 0.5f) / W, qy = (y + 0.5f) / H;
            float dx = qx - 0.5f, dy = qy - 0.5f, dz = 1.f;
            float l = std::sqrt(dx * dx + dy * dy + dz * dz);
            s.d = {dx / l, dy / l, dz / l};
            s.tMax = 2.f / s.d.z;
            s.p = {s.o.x + s.d.x * s.tMax, s.o.y + s.d.y * s.tMax, s.o.z + s.d.z * s.tMax};
            s.pixel = y * W + x;
            rec.Record(s);
        }
    std::vector<float> ld(3 * (size_t)W * H, 0.f);
    if (!bvh.Gather(rec, BeamRadiusAt(params, 0), ld)) {
        std::fprintf(stderr, "gather: %s\n", bvh.LastError().c_str());
        return 1;
    }
    std::vector<float> rgb;
    ResolveImage(ld, 0, rgb);
    double sum = 0;
    for (float v : rgb) sum += v;
    std::printf("bre_gather_demo: %zu beams, %lld segments, image sum %.9g\n", beams.size(), (long long)rec.Size(), sum);
    return sum > 0 ? 0 : 1;
}

}  // namespace

int main(int argc, char **argv) {
    const char *beams = nullptr, *segs = nullptr, *out = nullptr;
    int split = 1, iteration = 0;
    std::vector<int> devices{0};
    for (int i = 1; i < argc; ++i) {
        const bool more = i + 1 < argc;
        if (!std::strcmp(argv[i], "--beams") && more) beams = argv[++i];
        else if (!std::strcmp(argv[i], "--segments") && more) segs = argv[++i];
        else if (!std::strcmp(argv[i], "--out") && more) out = argv[++i];
        else if (!std::strcmp(argv[i], "--split") && more) split = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--iteration") && more) iteration = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--devices") && more) {
            devices.clear();
            for (const char *q = argv[++i]; *q;) {
                char *e = nullptr;
                devices.push_back((int)std::strtol(q, &e, 10));
                if (e == q) break;
                q = *e == ',' ? e + 1 : e;
            }
        }
        else if (argv[i][0] != '-' && !beams) return LatticeMode(std::atoi(argv[i]));
        else {
            std::fprintf(stderr, "usage: bre_gather_demo [W] | --beams B --segments S --out O [--split K] "
                                 "[--iteration I] [--devices D0,D1,..]\n");
            return 1;
        }
    }
    if (beams || segs || out) {
        if (!beams || !segs || !out) {
            std::fprintf(stderr, "bre_gather_demo: --beams, --segments and --out go together\n");
            return 1;
        }
        return FileMode(beams, segs, out, split, iteration, devices);
    }
    return LatticeMode(64);
}
