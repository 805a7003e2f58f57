// bre_oracle_photon.cpp — CPU restatement of the reference photon pass (TEST INFRASTRUCTURE).
//
// THIS FILE IS PART OF THE PARITY ORACLE, NOT THE PRODUCT.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load liboracle_bre.so.  The product photon pass is the HIP
// kernel in beam-radiance-estimate-pbrt_amd/csrc/bre_photon.hip, written independently as an
// explicit-stack state machine; this file keeps the reference's recursive structure so the two
// can be compared beam for beam.
//
// What it restates (reference = bwiberg/beam-radiance-estimate-pbrt, read as text only):
//   * photon emission loop              src/integrators/photonbeam.cpp:383-421
//   * AwesomeHaltonSampler              src/integrators/photonbeam.cpp:226-256  (the 1000 burned
//                                       Halton dimensions never touch the PCG32 stream)
//   * TracePhotonBeamRecursive          src/integrators/photonbeam.cpp:258-325
//   * RNG (PCG32) SetSequence / UniformUInt32 / UniformFloat   src/core/rng.h:78-85, 129-144
//   * DiffuseAreaLight::Sample_Le / L   src/lights/diffuse.cpp:89-123, diffuse.h:56-58
//   * CosineSampleHemisphere / ConcentricSampleDisk            src/core/sampling.h:159-165,
//                                                               src/core/sampling.cpp:113-133
//   * CoordinateSystem / SphericalDirection                    src/core/geometry.h:1020-1027, 1465-1470
//   * OffsetRayOrigin / NextFloatUp/Down                       src/core/geometry.h:1438-1458,
//                                                               src/core/pbrt.h (NextFloatUp/Down)
//   * HomogeneousMedium::Tr / Sample    src/media/homogeneous.cpp:44-77
//   * GridDensityMedium::Density / Sample / Tr           src/media/grid.cpp:46-118, grid.h:58-88
//     (WorldToMedium through Transform::operator()(Ray), transform.h:236-299; Bounds3::IntersectP
//     with t0/t1, geometry.h:1386-1408)
//   * HenyeyGreenstein::Sample_p / p, PhaseHG                  src/core/medium.cpp:194-218, medium.h:69-72
//   * BSDF::Sample_f (one Lambertian BxDF), BxDF::Sample_f     src/core/reflection.cpp:378-389, 703-768
//   * Spectrum (RGB) y(), Exp, operator/ (true division)       src/core/spectrum.h:181-194, 222-227, 462-465
//
// Interpretation notes:
//   * Point2f(Get1D(), Get1D()) (AwesomeHaltonSampler::Get2D, photonbeam.cpp:239-241) has
//     unspecified argument order.  The reference's build (its Dockerfile: g++ 4.8) evaluates
//     constructor arguments right to left on x86-64 (checked with this image's g++ on a
//     stand-alone snippet), so x = second draw, y = first draw.
//   * Transcendentals (log, exp, sin, cos) come from include/bre_fmath.h on both sides, so the
//     GPU pass and this restatement agree bit for bit.  Since round 6 they return the host glibc
//     libm's expf / logf / sinf / cosf bits for every float input (glibc >= 2.28's algorithms,
//     x86-64 FMA variants; tests/test_fmath_libm.py): the reference built on this image computes
//     the same.  (The libm of an older build differs: the Dockerfile pbrt-v3 ships names Ubuntu
//     12.04, glibc 2.15, whose float routines are other algorithms.)  With ora_set_libm(1) the
//     oracle calls the host libm itself (tests/test_faithful.py: nothing changes).
//   * Scene geometry: pbrt Triangles (include/bre_scene.h) -- Triangle::Intersect (watertight,
//     src/shapes/triangle.cpp:177-300), Triangle::Sample / Area (:535-568), one DiffuseAreaLight per
//     emitting triangle chosen by power (ComputeLightPowerDistribution, integrator.cpp:217-225;
//     Distribution1D::SampleDiscrete, sampling.h:55-100).  Scene::Intersect visits the triangles
//     in order (the reference's BVH order only matters for exact ties).
//
// Parity status: the photon pass has no reference test, golden vector or fixture
// and the reference cannot be built here: UNPINNED except for the primitives
// the reference's own tests cover — Henyey-Greenstein (src/tests/hg.cpp:10-81, restated in
// tests/test_photon_oracle.py) — and the published PCG32 test vector.

#include "ora_pbrt.h"

namespace orp {

struct Beam {
    V3 start, end;
    Float radius;
    Spectrum power;
};

// TracePhotonBeamRecursive (photonbeam.cpp:258-325)
static void TraceRecursive(Ray photonRay, int depth, Spectrum beta, Sampler &sampler, const Scene &sc,
                           int MaxDepth, Float BeamRadius, std::vector<Beam> &out) {
    Isect isect;
    for (; depth < MaxDepth; ++depth) {
        photonRay.tMax = Infinity;  // each loop ray is freshly spawned with tMax = Infinity
        if (!Intersect(sc, photonRay, &isect)) break;
        Spectrum betaMedium(1.0f);
        bool miValid = false;
        Float tScatter = 0;
        if (sc.medium) miValid = MediumSample(sc, photonRay, sampler, &tScatter);
        if (beta.IsBlack()) break;
        if (miValid) {
            V3 wo = -photonRay.d, wi;
            Float u0, u1;
            sampler.Get2D(&u0, &u1);
            HG_Sample_p(sc.g, wo, &wi, u0, u1);
            Ray scattered;
            scattered.o = photonRay(tScatter);  // MediumInteraction::SpawnRay: no offset
            scattered.d = wi;
            scattered.tMax = Infinity;
            Spectrum scatteredBeta = beta * MediumTr(sc, photonRay, sampler);
            TraceRecursive(scattered, depth + 1, scatteredBeta, sampler, sc, MaxDepth, BeamRadius, out);
        }
        if (sc.medium) betaMedium = MediumTr(sc, photonRay, sampler);
        Beam b;
        b.start = photonRay.o;
        b.end = isect.p;
        b.radius = BeamRadius;
        b.power = betaMedium * beta;
        out.push_back(b);

        // BSDF (MatteMaterial -> one LambertianReflection, or none when kd is black)
        const Tri &q = sc.tris[isect.tri];
        Float u0, u1;
        sampler.Get2D(&u0, &u1);  // evaluated before Sample_f runs
        if (q.kd.IsBlack()) break;  // matchingComps == 0: f = 0, pdf = 0
        V3 wo = -photonRay.d;
        V3 woL(Dot(wo, q.ss), Dot(wo, q.ts), Dot(wo, q.n));
        if (woL.z == 0) break;
        V3 wiL = CosineSampleHemisphere(u0, u1);
        if (woL.z < 0) wiL.z *= -1;
        Float pdf = (woL.z * wiL.z > 0) ? std::fabs(wiL.z) * InvPi : 0;
        if (pdf == 0) break;
        Spectrum fr = q.kd * InvPi;
        if (fr.IsBlack()) break;
        V3 wi(q.ss.x * wiL.x + q.ts.x * wiL.y + q.n.x * wiL.z, q.ss.y * wiL.x + q.ts.y * wiL.y + q.n.y * wiL.z,
              q.ss.z * wiL.x + q.ts.z * wiL.y + q.n.z * wiL.z);
        Spectrum betaNew = betaMedium * beta * fr * AbsDot(wi, q.n) / pdf;
        photonRay.o = OffsetRayOrigin(isect.p, isect.pError, isect.n, wi);
        photonRay.d = wi;
        Float qrr = std::max((Float)0, 1 - betaNew.y() / beta.y());
        if (sampler.Get1D() < qrr) break;
        beta = betaNew / (1 - qrr);
    }
}

// Emission (photonbeam.cpp:383-421): the light by power (lightDistr->SampleDiscrete), then
// DiffuseAreaLight::Sample_Le (diffuse.cpp:89-123) on its triangle (Triangle::Sample)
static void TracePhoton(const Scene &sc, uint64_t seq, int MaxDepth, Float BeamRadius, std::vector<Beam> &out) {
    if (sc.lights.empty()) return;  // no light to shoot from (libbre rejects such scenes)
    Sampler sampler(seq);
    Float lightPdf;
    const int lightNum = SampleDiscrete(sc, sampler.Get1D(), &lightPdf);
    const Tri &L = sc.tris[sc.lights[lightNum]];
    Float u0x, u0y, u1x, u1y;
    sampler.Get2D(&u0x, &u0y);
    sampler.Get2D(&u1x, &u1y);
    sampler.Get1D();  // uLightTime (shutter is [0,0])
    const ShapeSample ps = SampleTri(L, u0x, u0y);
    const Float pdfPos = ps.pdf;
    const V3 nLight = ps.n;
    V3 w = CosineSampleHemisphere(u1x, u1y);
    Float pdfDir = w.z * InvPi;
    V3 v1, v2;
    CoordinateSystem(nLight, &v1, &v2);
    w = w.x * v1 + w.y * v2 + w.z * nLight;
    Ray ray;
    ray.o = OffsetRayOrigin(ps.p, ps.pError, nLight, w);
    ray.d = w;
    ray.tMax = Infinity;
    Spectrum Le = Dot(nLight, w) > 0 ? L.Le : Spectrum(0.f);  // DiffuseAreaLight::L, one-sided
    if (pdfPos == 0 || pdfDir == 0 || Le.IsBlack()) return;
    Spectrum beta = (AbsDot(nLight, ray.d) * Le) / (lightPdf * pdfPos * pdfDir);
    if (beta.IsBlack()) return;
    TraceRecursive(ray, 0, beta, sampler, sc, MaxDepth, BeamRadius, out);
}

int g_ora_libm = 0;

}  // namespace orp

extern "C" {

// 1: transcendentals from the host libm (as the reference) instead of include/bre_fmath.h
void ora_set_libm(int on) { orp::g_ora_libm = on != 0; }

}  // extern "C"

extern "C" {

// Photons [0, n_photons) of `iteration`: photon i draws from PCG32 sequence
// iteration*n_photons + i + 1.  Beams are written photon-major, in the reference's push order,
// up to `capacity`; the return value is the total count (so a caller can size and call again).
// counts (optional, int32[n_photons]) receives the beams of each photon.
int64_t ora_trace_photons(const bre_scene *scene, int64_t n_photons, int32_t iteration, int32_t max_depth,
                          float beam_radius, int64_t capacity, float *start, float *end, float *radius,
                          float *power, int32_t *counts) {
    orp::Scene sc = orp::make_scene(scene);
    std::vector<orp::Beam> beams;
    int64_t total = 0;
    for (int64_t i = 0; i < n_photons; ++i) {
        beams.clear();
        uint64_t seq = (uint64_t)iteration * (uint64_t)n_photons + (uint64_t)i + 1;
        orp::TracePhoton(sc, seq, max_depth, beam_radius, beams);
        if (counts) counts[i] = (int32_t)beams.size();
        for (const orp::Beam &b : beams) {
            if (total < capacity) {
                for (int k = 0; k < 3; ++k) {
                    start[3 * total + k] = b.start[k];
                    end[3 * total + k] = b.end[k];
                    power[3 * total + k] = b.power.c[k];
                }
                radius[total] = b.radius;
            }
            ++total;
        }
    }
    return total;
}

// PCG32 as pbrt seeds it (RNG(seq)): n outputs of UniformUInt32, or UniformFloat if as_float.
void ora_pcg32(uint64_t seq, int64_t n, int32_t as_float, uint32_t *out) {
    orp::RNG r(seq);
    for (int64_t i = 0; i < n; ++i) {
        if (as_float) {
            float f = r.UniformFloat();
            memcpy(&out[i], &f, 4);
        } else {
            out[i] = r.UniformUInt32();
        }
    }
}

// PCG32 as pbrt's default-constructed RNG() (rng.h:129: PCG32_DEFAULT_STATE / _STREAM): n outputs of
// UniformUInt32 (the stream fp_tests.cpp's NextUpDownFloat test draws its floats from)
void ora_pcg32_default(int64_t n, uint32_t *out) {
    orp::RNG r;
    for (int64_t i = 0; i < n; ++i) out[i] = r.UniformUInt32();
}

// NextFloatUp (up != 0) / NextFloatDown of n floats (pbrt.h:215-239, the OffsetRayOrigin steps)
void ora_next_float(int32_t up, int64_t n, const float *x, float *y) {
    for (int64_t i = 0; i < n; ++i) y[i] = up ? orp::NextFloatUp(x[i]) : orp::NextFloatDown(x[i]);
}

// FloatToBits(BitsToFloat(u)) of n words (pbrt.h:191-202): the bit casts the float stepping uses
void ora_float_bits(int64_t n, const uint32_t *u, uint32_t *out) {
    for (int64_t i = 0; i < n; ++i) out[i] = bre_f2u(bre_u2f(u[i]));
}

// FindInterval(n, [&](int i) { return a[i] <= x; }) for m values of x (pbrt.h:377-389), the search of
// both Distribution1D samplers
void ora_find_interval(const float *a, int32_t n, int64_t m, const float *x, int32_t *out) {
    for (int64_t i = 0; i < m; ++i) {
        const float v = x[i];
        out[i] = orp::FindInterval(n, [&](int k) { return a[k] <= v; });
    }
}

// PCG32 seeded like pcg32_srandom(initstate, initseq) (pbrt fixes initstate): for the
// published test vector of the PCG reference implementation.
void ora_pcg32_srandom(uint64_t initstate, uint64_t initseq, int64_t n, uint32_t *out) {
    orp::RNG r(0);
    r.state = 0u;
    r.inc = (initseq << 1u) | 1u;
    r.UniformUInt32();
    r.state += initstate;
    r.UniformUInt32();
    for (int64_t i = 0; i < n; ++i) out[i] = r.UniformUInt32();
}

// HenyeyGreenstein::Sample_p for n (wo, u) pairs: wi[3n], returns pdf[n]
void ora_hg_sample(float g, int64_t n, const float *wo, const float *u, float *wi, float *pdf) {
    for (int64_t i = 0; i < n; ++i) {
        orp::V3 w(wo + 3 * i), o;
        pdf[i] = orp::HG_Sample_p(g, w, &o, u[2 * i], u[2 * i + 1]);
        wi[3 * i] = o.x;
        wi[3 * i + 1] = o.y;
        wi[3 * i + 2] = o.z;
    }
}
void ora_hg_p(float g, int64_t n, const float *wo, const float *wi, float *p) {
    for (int64_t i = 0; i < n; ++i) p[i] = orp::HG_p(g, orp::V3(wo + 3 * i), orp::V3(wi + 3 * i));
}

// HomogeneousMedium::Tr for n rays (d[3n], tmax[n]) -> tr[3n]
void ora_homogeneous_tr(const float *sigma_a, const float *sigma_s, int64_t n, const float *d, const float *tmax,
                        float *tr) {
    bre_scene s;
    memset(&s, 0, sizeof(s));
    s.has_medium = 1;
    memcpy(s.sigma_a, sigma_a, 12);
    memcpy(s.sigma_s, sigma_s, 12);
    orp::Scene sc = orp::make_scene(&s);
    for (int64_t i = 0; i < n; ++i) {
        orp::Ray r;
        r.d = orp::V3(d + 3 * i);
        r.tMax = tmax[i];
        orp::Spectrum t = orp::HomogeneousTr(sc, r);
        for (int k = 0; k < 3; ++k) tr[3 * i + k] = t.c[k];
    }
}

// CosineSampleHemisphere for n sample pairs -> w[3n]
void ora_cosine_hemisphere(int64_t n, const float *u, float *w) {
    for (int64_t i = 0; i < n; ++i) {
        orp::V3 v = orp::CosineSampleHemisphere(u[2 * i], u[2 * i + 1]);
        w[3 * i] = v.x;
        w[3 * i + 1] = v.y;
        w[3 * i + 2] = v.z;
    }
}

// include/bre_fmath.h on the host: kind 0 = log, 1 = exp, 2 = sin, 3 = cos
void ora_fmath(int32_t kind, int64_t n, const float *x, float *y) {
    for (int64_t i = 0; i < n; ++i) {
        float s, c;
        switch (kind) {
            case 0: y[i] = bre_logf(x[i]); break;
            case 1: y[i] = bre_expf(x[i]); break;
            case 2: bre_sincosf(x[i], &s, &c); y[i] = s; break;
            default: bre_sincosf(x[i], &s, &c); y[i] = c; break;
        }
    }
}

}  // extern "C"

extern "C" {

// GridDensityMedium::Density at n medium-space points p[3n] (grid.cpp:46-60)
void ora_grid_density(const bre_scene *scene, int64_t n, const float *p, float *out) {
    orp::Scene sc = orp::make_scene(scene);
    for (int64_t i = 0; i < n; ++i) out[i] = orp::GridDensity(sc, orp::V3(p + 3 * i));
}

// GridDensityMedium::Tr (kind 0) or ::Sample (kind 1; out = medium-space t or -1 when no
// interaction) for n world rays, ray i drawing from PCG32 sequence seq0 + i; draws[i] = number of
// sampler draws it used
void ora_grid_eval(const bre_scene *scene, int32_t kind, int64_t n, const float *o, const float *d,
                   const float *tmax, uint64_t seq0, float *out, int32_t *draws) {
    orp::Scene sc = orp::make_scene(scene);
    struct Counting {
        orp::Sampler s;
        int32_t n = 0;
        explicit Counting(uint64_t q) : s(q) {}
        orp::Float Get1D() {
            ++n;
            return s.Get1D();
        }
    };
    for (int64_t i = 0; i < n; ++i) {
        orp::Ray r;
        r.o = orp::V3(o + 3 * i);
        r.d = orp::V3(d + 3 * i);
        r.tMax = tmax[i];
        Counting cs(seq0 + (uint64_t)i);
        if (kind == 0) {
            out[i] = orp::GridTr(sc, r, cs).c[0];
        } else {
            orp::Float t = 0;
            out[i] = orp::GridSample(sc, r, cs, &t) ? t : -1.f;
        }
        if (draws) draws[i] = cs.n;
    }
}

}  // extern "C"

extern "C" {

// Test support: the reference's own shape and sampling tests (src/tests/shapes.cpp,
// src/tests/sampling.cpp) restated on the oracle's pbrt primitives (tests/test_ref_tests.py).

// For n rays (o, d, tMax = +inf): how many of the scene's triangles Triangle::Intersect hits
// (Triangle.Watertight, shapes.cpp:28-152, requires >= 1 from inside a closed mesh)
void ora_tri_hits(const bre_scene *scene, int64_t n, const float *o, const float *d, int32_t *hits) {
    orp::Scene sc = orp::make_scene(scene);
    for (int64_t i = 0; i < n; ++i) {
        int32_t k = 0;
        for (const orp::Tri &T : sc.tris) {
            orp::Ray r;
            r.o = orp::V3(o + 3 * i);
            r.d = orp::V3(d + 3 * i);
            r.tMax = orp::Infinity;
            orp::Float t;
            orp::Isect is;
            k += orp::IntersectTri(T, r, &t, &is) ? 1 : 0;
        }
        hits[i] = k;
    }
}

// Scene::Intersect for n rays (o, d, tMax = +inf): through the scene's BVHAccel (use_bvh != 0, what
// the passes use) or over the triangles in scene order (the round-2 restatement); the hit distance
// (the final ray.tMax, +inf for a miss) and triangle (-1 for a miss).  *depth: the BVH's depth.
void ora_scene_intersect(const bre_scene *scene, int64_t n, const float *o, const float *d, int32_t use_bvh,
                         float *t_out, int32_t *tri_out, int32_t *depth) {
    orp::Scene sc = orp::make_scene(scene);
    for (int64_t i = 0; i < n; ++i) {
        orp::Ray r;
        r.o = orp::V3(o + 3 * i);
        r.d = orp::V3(d + 3 * i);
        r.tMax = orp::Infinity;
        orp::Isect is;
        const bool hit = use_bvh ? orp::Intersect(sc, r, &is) : orp::IntersectLinear(sc, r, &is);
        t_out[i] = r.tMax;
        tri_out[i] = hit ? is.tri : -1;
    }
    if (depth) {
        // depth of the flattened tree: walk it with an explicit stack of (node, level)
        int best = 0;
        std::vector<std::pair<int, int>> st;
        if (!sc.nodes.empty()) st.push_back({0, 1});
        while (!st.empty()) {
            const auto [k, lv] = st.back();
            st.pop_back();
            best = std::max(best, lv);
            const orp::LinearBVHNode &nd = sc.nodes[(size_t)k];
            if (nd.nPrimitives == 0) {
                st.push_back({k + 1, lv + 1});
                st.push_back({nd.offset, lv + 1});
            }
        }
        *depth = best;
    }
}

// Triangle::Sample(u) (triangle.cpp:543-568, area measure) of triangle `tri` for n sample pairs
void ora_tri_sample(const bre_scene *scene, int32_t tri, int64_t n, const float *u, float *p, float *nrm,
                    float *pdf) {
    orp::Scene sc = orp::make_scene(scene);
    const orp::Tri &T = sc.tris[tri];
    for (int64_t i = 0; i < n; ++i) {
        const orp::ShapeSample s = orp::SampleTri(T, u[2 * i], u[2 * i + 1]);
        for (int k = 0; k < 3; ++k) {
            p[3 * i + k] = s.p[k];
            nrm[3 * i + k] = s.n[k];
        }
        pdf[i] = s.pdf;
    }
}

// Distribution1D(func, nf) (sampling.h:55-100): SampleDiscrete for m values of u (index, pdf,
// uRemapped) and DiscretePDF of every entry (Distribution1D.Discrete, sampling.cpp:231-280)
void ora_distribution1d(const float *func, int32_t nf, int64_t m, const float *u, int32_t *idx, float *pdf,
                        float *urem, float *dpdf) {
    const orp::Distribution1D dist(func, nf);
    for (int64_t i = 0; i < m; ++i) idx[i] = dist.SampleDiscrete(u[i], &pdf[i], &urem[i]);
    for (int i = 0; i < nf; ++i) dpdf[i] = dist.DiscretePDF(i);
}

// Distribution1D::SampleContinuous for m values of u: x, pdf, offset (Distribution1D.Continuous,
// sampling.cpp:282-303)
void ora_distribution1d_continuous(const float *func, int32_t nf, int64_t m, const float *u, float *x, float *pdf,
                                   int32_t *off) {
    const orp::Distribution1D dist(func, nf);
    for (int64_t i = 0; i < m; ++i) {
        int o = 0;
        x[i] = dist.SampleContinuous(u[i], &pdf[i], &o);
        off[i] = o;
    }
}

// Triangle.Reintersect (src/tests/shapes.cpp:154-208) on the oracle's pbrt primitives, with the
// test's own random streams: triangle i's vertices, sample point and ray origin come from RNG(i)
// through pExp (shapes.cpp:18-21: 10^Lerp(u, -8, 8), std::pow in double); a ray from the origin to
// Triangle::Sample's point is intersected (Triangle::Intersect, with its pError), and
// rays_per_tri rays leaving the hit -- SpawnRay along UniformSampleSphere directions and SpawnRayTo
// random pExp points (interaction.h:64-72, OffsetRayOrigin geometry.h:1438-1458, ShadowEpsilon
// pbrt.h:178) -- must not hit the triangle again.  Returns the re-intersections (the reference
// expects none); *tested: spawned rays checked, *used: triangles whose first ray hit.
int64_t ora_tri_reintersect(int32_t n_tris, int32_t rays_per_tri, int64_t *tested, int32_t *used) {
    using namespace orp;
    int64_t bad = 0, nt = 0;
    int32_t nu = 0;
    for (int i = 0; i < n_tris; ++i) {
        RNG rng((uint64_t)i);
        const auto pExp = [&]() {
            const Float logu = Lerp(rng.UniformFloat(), -8.f, 8.f);
            return (Float)std::pow(10, logu);
        };
        V3 v[3];
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) v[j][k] = pExp();
        if (Cross(v[1] - v[0], v[2] - v[0]).LengthSquared() < 1e-20f) continue;  // GetRandomTriangle
        bre_scene bs;
        std::memset(&bs, 0, sizeof(bs));
        bs.n_triangles = 1;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) bs.triangles[0].p[j][k] = v[j][k];
        const Scene sc = make_scene(&bs);
        const Tri &T = sc.tris[0];
        Float u0 = rng.UniformFloat();
        Float u1 = rng.UniformFloat();
        const ShapeSample pTri = SampleTri(T, u0, u1);
        V3 o;
        for (int j = 0; j < 3; ++j) o[j] = pExp();
        Ray r{o, pTri.p - o, Infinity};
        Float tHit;
        Isect isect;
        if (!IntersectTri(T, r, &tHit, &isect)) continue;
        ++nu;
        for (int j = 0; j < rays_per_tri; ++j) {
            u0 = rng.UniformFloat();
            u1 = rng.UniformFloat();
            // UniformSampleSphere (sampling.cpp:98-103)
            const Float z = 1 - 2 * u0;
            const Float rr = std::sqrt(std::max((Float)0, (Float)1 - z * z));
            const Float phi = 2 * Pi * u1;
            const V3 w(rr * std::cos(phi), rr * std::sin(phi), z);
            Ray out{OffsetRayOrigin(isect.p, isect.pError, isect.n, w), w, Infinity};  // SpawnRay(w)
            Isect tmp;
            bad += IntersectTri(T, out, &tHit, &tmp) ? 1 : 0;
            V3 p2;
            for (int k = 0; k < 3; ++k) p2[k] = pExp();
            // SpawnRayTo(p2): origin offset toward p2, d = p2 - p, tMax = 1 - ShadowEpsilon
            Ray to{OffsetRayOrigin(isect.p, isect.pError, isect.n, p2 - isect.p), p2 - isect.p, 1 - 0.0001f};
            bad += IntersectTri(T, to, &tHit, &tmp) ? 1 : 0;
            nt += 2;
        }
    }
    if (tested) *tested = nt;
    if (used) *used = nu;
    return bad;
}

}  // extern "C"
