// bre_gather_demo.cpp — C++ host program using the integrator mirror (photonbeam_gpu.h):
// one iteration of "build beams -> record camera segments -> batched gather -> resolve image"
// on a small deterministic scene, printing the image sum.  Exit code 0 on success.
#include <cmath>
#include <cstdio>
#include <vector>

#include "photonbeam_gpu.h"

using namespace bre_host;

int main(int argc, char **argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 64, H = W;
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
