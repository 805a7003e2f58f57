// bre_oracle_camera.cpp — CPU restatement of the reference camera pass (TEST INFRASTRUCTURE).
//
// THIS FILE IS PART OF THE PARITY ORACLE, NOT THE PRODUCT (see bre_oracle_photon.cpp).  The
// product camera pass is beam-radiance-estimate-pbrt_amd/csrc/bre_camera.hip.
//
// What it restates (reference = bwiberg/beam-radiance-estimate-pbrt, read as text only):
//   * camera loop of PhotonBeamIntegrator::Render      src/integrators/photonbeam.cpp:444-555
//     (segment = [ray.o, isect.p] of every surface-hit camera ray, :494-508; rendersurfaces /
//     rendermedia switches; RR on luminance < 0.25, :547-552)
//   * AwesomeSampler over the HaltonSampler            photonbeam.cpp:188-224, 456-462
//   * HaltonSampler                                    src/samplers/halton.cpp:63-127
//   * GlobalSampler::SetSampleNumber / Get1D / Get2D   src/core/sampler.cpp:165-195
//   * RadicalInverse / ScrambledRadicalInverse / ReverseBits / InverseRadicalInverse
//                                                      src/core/lowdiscrepancy.{h:67-91, cpp:385-445, 2500-2520}
//   * ComputeRadicalInversePermutations, Shuffle       lowdiscrepancy.cpp:2500-2514, sampling.h:151-157
//   * Sampler::GetCameraSample                         src/core/sampler.cpp:46-52
//   * UniformSampleOneLight / EstimateDirect           src/core/integrator.cpp:85-214
//   * DiffuseAreaLight::Sample_Li / Pdf_Li / L         src/lights/diffuse.cpp:68-87, diffuse.h:56-58
//   * Shape::Sample(ref) / Shape::Pdf(ref, wi)         src/core/shape.cpp:56-87
//   * VisibilityTester::Tr, Scene::IntersectTr         src/core/light.cpp:63-81, scene.cpp:62-75
//   * BSDF::f / BSDF::Pdf / BSDF::Sample_f             src/core/reflection.cpp:650-768
//   * Interaction::SpawnRayTo, Interaction(wo normalised)  src/core/interaction.h:50-78
//   * PowerHeuristic                                   src/core/sampling.h:171-174
//   * Transform::operator()(Ray) origin offset         src/core/transform.h:251-264
//
// Interpretation notes:
//   * Camera rays: a pinhole (lensradius 0) with pbrt's screen window (the "fov" spans the
//     shorter image axis) and LookAt frame, evaluated directly rather than through pbrt's 4x4
//     RasterToCamera / CameraToWorld matrix chain: the same ray up to float rounding of the
//     matrix products, with the origin offset of Transform::operator()(Ray).  The same
//     arithmetic is the product's contract (DESIGN.md "Camera pass").
//   * Halton permutation tables cover all 1000 prime dimensions.  Past its 1000th draw the
//     AwesomeSampler switches to PCG32 sequence GoodPixelIndex = iterNumPixels++ (photonbeam.cpp:
//     457-458), a counter the reference's camera-pass threads bump without synchronisation; this
//     restatement takes the single-threaded ParallelFor2D order (tiles row-major, pixels x-fastest).
//     Only GridDensityMedium paths (ratio tracking draws) get anywhere near 1000 draws.
//   * The reference adds gather and surface terms to one pixel.Ld in path order; this
//     restatement returns them separately (segments for the gather, surface radiance per pixel).
//
// Parity status: unpinned for the camera pass as a whole (no reference fixture, no runnable
// reference).  Pinned primitives: RadicalInverse and ScrambledRadicalInverse by
// restating src/tests/sampling.cpp:14-66 (tests/test_camera_oracle.py).

#include "ora_pbrt.h"

namespace orp {

static const int kHaltonDims = 1000;  // PrimeTableSize (lowdiscrepancy.h:38) = AwesomeSampler's limit
static const Float ShadowEpsilon = 0.0001f;

// ---- low-discrepancy primitives ----
static inline uint32_t ReverseBits32(uint32_t n) {
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ff) << 8) | ((n & 0xff00ff00) >> 8);
    n = ((n & 0x0f0f0f0f) << 4) | ((n & 0xf0f0f0f0) >> 4);
    n = ((n & 0x33333333) << 2) | ((n & 0xcccccccc) >> 2);
    n = ((n & 0x55555555) << 1) | ((n & 0xaaaaaaaa) >> 1);
    return n;
}
static inline uint64_t ReverseBits64(uint64_t n) {
    uint64_t n0 = ReverseBits32((uint32_t)n);
    uint64_t n1 = ReverseBits32((uint32_t)(n >> 32));
    return (n0 << 32) | n1;
}
static inline uint64_t InverseRadicalInverse(uint64_t base, uint64_t inverse, int nDigits) {
    uint64_t index = 0;
    for (int i = 0; i < nDigits; ++i) {
        uint64_t digit = inverse % base;
        inverse /= base;
        index = index * base + digit;
    }
    return index;
}
static inline Float RadicalInverseSpecialized(uint64_t base, uint64_t a) {
    const Float invBase = (Float)1 / (Float)base;
    uint64_t reversedDigits = 0;
    Float invBaseN = 1;
    while (a) {
        uint64_t next = a / base;
        uint64_t digit = a - next * base;
        reversedDigits = reversedDigits * base + digit;
        invBaseN *= invBase;
        a = next;
    }
    return std::min(reversedDigits * invBaseN, OneMinusEpsilon);
}
static inline Float ScrambledRadicalInverseSpecialized(uint64_t base, const uint16_t *perm, uint64_t a) {
    const Float invBase = (Float)1 / (Float)base;
    uint64_t reversedDigits = 0;
    Float invBaseN = 1;
    while (a) {
        uint64_t next = a / base;
        uint64_t digit = a - next * base;
        reversedDigits = reversedDigits * base + perm[digit];
        invBaseN *= invBase;
        a = next;
    }
    return std::min(invBaseN * (reversedDigits + invBase * perm[0] / (1 - invBase)), OneMinusEpsilon);
}

static std::vector<int> first_primes(int n) {
    std::vector<int> p;
    for (int c = 2; (int)p.size() < n; ++c) {
        bool prime = true;
        for (int q : p) {
            if (q * q > c) break;
            if (c % q == 0) {
                prime = false;
                break;
            }
        }
        if (prime) p.push_back(c);
    }
    return p;
}

template <typename T>
static void Shuffle(T *samp, int count, int nDimensions, RNG &rng) {
    for (int i = 0; i < count; ++i) {
        int other = i + rng.UniformUInt32(count - i);
        for (int j = 0; j < nDimensions; ++j) std::swap(samp[nDimensions * i + j], samp[nDimensions * other + j]);
    }
}

static inline int64_t ModI(int64_t a, int64_t b) {
    int64_t r = a - (a / b) * b;
    return (r < 0) ? r + b : r;
}
static void extendedGCD(uint64_t a, uint64_t b, int64_t *x, int64_t *y) {
    if (b == 0) {
        *x = 1;
        *y = 0;
        return;
    }
    int64_t d = a / b, xp, yp;
    extendedGCD(b, a % b, &xp, &yp);
    *x = yp;
    *y = xp - (d * yp);
}
static uint64_t multiplicativeInverse(int64_t a, int64_t n) {
    int64_t x, y;
    extendedGCD(a, n, &x, &y);
    return ModI(x, n);
}

struct Halton {
    std::vector<int> primes, primeSums;
    std::vector<uint16_t> perms;
    int baseScales[2], baseExponents[2];
    int sampleStride;
    int multInverse[2];

    Halton(int width, int height) {
        primes = first_primes(kHaltonDims);
        int sum = 0;
        for (int p : primes) {
            primeSums.push_back(sum);
            sum += p;
        }
        perms.resize(sum);
        RNG rng;  // default-seeded, as HaltonSampler's ctor (halton.cpp:70-73)
        uint16_t *p = perms.data();
        for (int i = 0; i < kHaltonDims; ++i) {
            for (int j = 0; j < primes[i]; ++j) p[j] = (uint16_t)j;
            Shuffle(p, primes[i], 1, rng);
            p += primes[i];
        }
        const int res[2] = {width, height};
        for (int i = 0; i < 2; ++i) {
            int base = (i == 0) ? 2 : 3;
            int scale = 1, exp = 0;
            while (scale < std::min(res[i], 128)) {
                scale *= base;
                ++exp;
            }
            baseScales[i] = scale;
            baseExponents[i] = exp;
        }
        sampleStride = baseScales[0] * baseScales[1];
        multInverse[0] = (int)multiplicativeInverse(baseScales[1], baseScales[0]);
        multInverse[1] = (int)multiplicativeInverse(baseScales[0], baseScales[1]);
    }
    int64_t IndexForSample(int px, int py, int64_t sampleNum) const {
        int64_t offset = 0;
        if (sampleStride > 1) {
            const int pm[2] = {(int)ModI(px, 128), (int)ModI(py, 128)};
            for (int i = 0; i < 2; ++i) {
                uint64_t dimOffset = InverseRadicalInverse(i == 0 ? 2 : 3, (uint64_t)pm[i], baseExponents[i]);
                offset += dimOffset * (sampleStride / baseScales[i]) * multInverse[i];
            }
            offset %= sampleStride;
        }
        return offset + sampleNum * sampleStride;
    }
    Float SampleDimension(int64_t index, int dim) const {
        if (dim == 0) return (Float)((double)ReverseBits64((uint64_t)(index >> baseExponents[0])) * 0x1p-64);
        if (dim == 1) return RadicalInverseSpecialized(3, (uint64_t)(index / baseScales[1]));
        return ScrambledRadicalInverseSpecialized((uint64_t)primes[dim], &perms[primeSums[dim]], (uint64_t)index);
    }
};

// AwesomeSampler(0, haltonTileSampler, 1000, GoodPixelIndex) after StartPixel + SetSampleNumber(iter)
// (photonbeam.cpp:188-224, 456-462; GlobalSampler::Get1D/Get2D, sampler.cpp:178-195)
struct CameraSampler {
    const Halton *h;
    int64_t index;
    int dimension = 0;
    size_t sampleCount = 0;
    RNG rng;
    Float Get1D() {
        sampleCount++;
        if (sampleCount <= (size_t)kHaltonDims) return h->SampleDimension(index, dimension++);
        return rng.UniformFloat();
    }
    void Get2D(Float *x, Float *y) {
        sampleCount += 2;
        if (sampleCount <= (size_t)kHaltonDims) {
            *x = h->SampleDimension(index, dimension);
            *y = h->SampleDimension(index, dimension + 1);
            dimension += 2;
            return;
        }
        Float first = rng.UniformFloat();  // Point2f(rng.UniformFloat(), rng.UniformFloat()), right to left
        Float second = rng.UniformFloat();
        *x = second;
        *y = first;
    }
};

struct Camera {
    V3 pos, dir, right, nup;
    Float sx0, sx1, sy0, sy1, tanAng, W, H;
};
static Camera make_camera(const bre_scene *s, int width, int height) {
    Camera c;
    c.pos = V3(s->cam_pos);
    V3 look(s->cam_look), up(s->cam_up);
    c.dir = Normalize(look - c.pos);
    c.right = Normalize(Cross(Normalize(up), c.dir));
    c.nup = Cross(c.dir, c.right);
    const Float aspect = (Float)width / (Float)height;
    if (aspect > 1.f) {
        c.sx0 = -aspect;
        c.sx1 = aspect;
        c.sy0 = -1.f;
        c.sy1 = 1.f;
    } else {
        c.sx0 = -1.f;
        c.sx1 = 1.f;
        c.sy0 = -1.f / aspect;
        c.sy1 = 1.f / aspect;
    }
    c.tanAng = std::tan(((Pi / 180) * s->cam_fov_deg) / 2);
    c.W = (Float)width;
    c.H = (Float)height;
    return c;
}
static Ray GenerateRay(const Camera &c, Float fx, Float fy) {
    const Float sx = c.sx0 + (fx / c.W) * (c.sx1 - c.sx0);
    const Float sy = c.sy1 - (fy / c.H) * (c.sy1 - c.sy0);
    const V3 dc = Normalize(V3(sx * c.tanAng, sy * c.tanAng, 1));
    Ray r;
    r.d = c.right * dc.x + c.nup * dc.y + c.dir * dc.z;
    const V3 oError = Abs(c.pos) * gamma(3);
    r.o = c.pos;
    const Float l2 = r.d.LengthSquared();
    if (l2 > 0) {
        const Float dt = Dot(Abs(r.d), oError) / l2;
        r.o = r.o + r.d * dt;
    }
    r.tMax = Infinity;
    return r;
}

// ---- BSDF of a matte triangle (reflection.cpp:650-768) ----
static inline V3 WorldToLocal(const Tri &q, const V3 &v) { return V3(Dot(v, q.ss), Dot(v, q.ts), Dot(v, q.n)); }
static inline V3 LocalToWorld(const Tri &q, const V3 &v) {
    return V3(q.ss.x * v.x + q.ts.x * v.y + q.n.x * v.z, q.ss.y * v.x + q.ts.y * v.y + q.n.y * v.z,
              q.ss.z * v.x + q.ts.z * v.y + q.n.z * v.z);
}
static Spectrum BSDF_f(const Tri &q, const V3 &woW, const V3 &wiW) {
    if (q.kd.IsBlack()) return Spectrum(0.f);  // no BxDF
    V3 wo = WorldToLocal(q, woW);
    if (wo.z == 0) return Spectrum(0.f);
    bool reflect = Dot(wiW, q.n) * Dot(woW, q.n) > 0;
    Spectrum f(0.f);
    if (reflect) f = f + q.kd * InvPi;
    return f;
}
static Float BSDF_Pdf(const Tri &q, const V3 &woW, const V3 &wiW) {
    if (q.kd.IsBlack()) return 0.f;
    V3 wo = WorldToLocal(q, woW), wi = WorldToLocal(q, wiW);
    if (wo.z == 0) return 0.;
    Float pdf = 0.f;
    pdf += (wo.z * wi.z > 0) ? std::abs(wi.z) * InvPi : 0;
    return pdf / 1;
}
// returns f; *pdf untouched when wo.z == 0 (as the reference)
static Spectrum BSDF_Sample_f(const Tri &q, const V3 &woW, V3 *wiW, Float ux, Float uy, Float *pdf) {
    if (q.kd.IsBlack()) {
        *pdf = 0;
        return Spectrum(0.f);
    }
    V3 wo = WorldToLocal(q, woW);
    if (wo.z == 0) return Spectrum(0.);
    *pdf = 0;
    V3 wi = CosineSampleHemisphere(ux, uy);
    if (wo.z < 0) wi.z *= -1;
    *pdf = (wo.z * wi.z > 0) ? std::abs(wi.z) * InvPi : 0;
    Spectrum f = q.kd * InvPi;
    if (*pdf == 0) return Spectrum(0.f);
    *wiW = LocalToWorld(q, wi);
    return f;
}

static inline Float PowerHeuristic(int nf, Float fPdf, int ng, Float gPdf) {
    Float f = nf * fPdf, g = ng * gPdf;
    return (f * f) / (f * f + g * g);
}

struct Interaction {
    V3 p, pError, n, wo;
    int tri;
};

static Spectrum VisibilityTr(const Scene &sc, const Interaction &p0, const Interaction &p1, CameraSampler &cs) {
    Ray ray;
    ray.o = OffsetRayOrigin(p0.p, p0.pError, p0.n, p1.p - p0.p);
    V3 target = OffsetRayOrigin(p1.p, p1.pError, p1.n, ray.o - p1.p);
    ray.d = target - ray.o;
    ray.tMax = 1 - ShadowEpsilon;
    Spectrum Tr(1.f);
    Isect isect;
    bool hit = Intersect(sc, ray, &isect);
    if (hit) return Spectrum(0.0f);  // every triangle has a material
    if (sc.medium) Tr = Tr * MediumTr(sc, ray, cs);
    return Tr;
}

// EstimateDirect (integrator.cpp:99-199) for the area light on triangle `li` (handleMedia = true)
static Spectrum EstimateDirect(const Scene &sc, const Interaction &it, int li, Float usx, Float usy, Float ulx,
                               Float uly, CameraSampler &cs) {
    const Tri &L = sc.tris[li];
    const Tri &q = sc.tris[it.tri];
    Spectrum Ld(0.f);
    V3 wi;
    Float lightPdf = 0, scatteringPdf = 0;
    // DiffuseAreaLight::Sample_Li (diffuse.cpp:68-81) -> Shape::Sample(ref, u) (shape.cpp:56-70)
    const ShapeSample ss = SampleTri(L, ulx, uly);
    Interaction pS;
    pS.p = ss.p;
    pS.pError = ss.pError;
    pS.n = ss.n;
    lightPdf = ss.pdf;
    V3 w = pS.p - it.p;
    if (w.LengthSquared() == 0) {
        lightPdf = 0;
    } else {
        w = Normalize(w);
        lightPdf *= (it.p - pS.p).LengthSquared() / AbsDot(pS.n, -w);
        if (std::isinf(lightPdf)) lightPdf = 0.f;
    }
    Spectrum Li(0.f);
    if (lightPdf == 0 || (pS.p - it.p).LengthSquared() == 0) {
        lightPdf = 0;
    } else {
        wi = Normalize(pS.p - it.p);
        Li = Dot(pS.n, -wi) > 0 ? L.Le : Spectrum(0.f);
    }
    if (lightPdf > 0 && !Li.IsBlack()) {
        Spectrum f = BSDF_f(q, it.wo, wi) * AbsDot(wi, q.n);
        scatteringPdf = BSDF_Pdf(q, it.wo, wi);
        if (!f.IsBlack()) {
            Li = Li * VisibilityTr(sc, it, pS, cs);
            if (!Li.IsBlack()) {
                Float weight = PowerHeuristic(1, lightPdf, 1, scatteringPdf);
                Ld = Ld + f * Li * weight / lightPdf;
            }
        }
    }
    // BSDF sampling (an area light is not a delta light)
    {
        Spectrum f = BSDF_Sample_f(q, it.wo, &wi, usx, usy, &scatteringPdf);
        f = f * AbsDot(wi, q.n);
        if (!f.IsBlack() && scatteringPdf > 0) {
            // DiffuseAreaLight::Pdf_Li -> Shape::Pdf(ref, wi) (shape.cpp:72-87): this triangle alone
            Ray ray;
            ray.o = OffsetRayOrigin(it.p, it.pError, it.n, wi);
            ray.d = wi;
            ray.tMax = Infinity;
            Float tHit;
            Isect isL;
            if (!IntersectTri(L, ray, &tHit, &isL)) return Ld;
            lightPdf = (it.p - isL.p).LengthSquared() / (AbsDot(isL.n, -wi) * L.area);
            if (std::isinf(lightPdf)) lightPdf = 0.f;
            if (lightPdf == 0) return Ld;
            Float weight = PowerHeuristic(1, scatteringPdf, 1, lightPdf);
            // Scene::IntersectTr
            Ray r2;
            r2.o = OffsetRayOrigin(it.p, it.pError, it.n, wi);
            r2.d = wi;
            r2.tMax = Infinity;
            Spectrum Tr(1.f);
            Isect lh;
            bool found = Intersect(sc, r2, &lh);
            if (sc.medium) Tr = Tr * MediumTr(sc, r2, cs);
            Spectrum Lr(0.f);
            // lightIsect.primitive->GetAreaLight() == &light: the same triangle
            if (found && lh.tri == li) Lr = Dot(lh.n, -wi) > 0 ? L.Le : Spectrum(0.f);
            if (!Lr.IsBlack()) Ld = Ld + f * Lr * Tr * weight / scatteringPdf;
        }
    }
    return Ld;
}

struct Segment {
    V3 o, p, d;
    Float tmax;
    int pixel, depth;
};

// One camera path (photonbeam.cpp:456-553).  Returns false if the path needed more Halton
// dimensions than the table holds.
static bool CameraPath(const Scene &sc, const Camera &cam, const Halton &h, int px, int py, int width, int iter,
                       int maxDepth, bool renderSurfaces, bool renderMedia, uint64_t goodPixelIndex,
                       std::vector<Segment> &segs, Spectrum *Ld) {
    CameraSampler cs;
    cs.h = &h;
    cs.index = h.IndexForSample(px, py, iter);
    cs.rng = RNG(goodPixelIndex);
    Float fx, fy, lx, ly;
    cs.Get2D(&fx, &fy);
    fx = (Float)px + fx;
    fy = (Float)py + fy;
    cs.Get1D();           // time
    cs.Get2D(&lx, &ly);   // lens (pinhole)
    Ray ray = GenerateRay(cam, fx, fy);
    Spectrum beta(1.f);
    bool specularBounce = false;
    const int pixel = py * width + px;
    const int nLights = (int)sc.lights.size();
    for (int depth = 0; depth < maxDepth; ++depth) {
        Isect isect;
        ray.tMax = Infinity;
        if (!Intersect(sc, ray, &isect)) break;  // area lights have no Le(ray)
        Spectrum mediumBeta(1.0f);
        if (sc.medium) mediumBeta = MediumTr(sc, ray, cs);
        if (renderMedia) segs.push_back(Segment{ray.o, isect.p, ray.d, ray.tMax, pixel, depth});
        beta = beta * mediumBeta;
        if (!renderSurfaces) break;  // every triangle has a BSDF
        const Tri &q = sc.tris[isect.tri];
        V3 wo = -ray.d;
        // isect.Le(wo): the triangle's own area light, one-sided (diffuse.h:56-58)
        if (depth == 0 || specularBounce)
            if (q.emit) *Ld = *Ld + beta * (Dot(isect.n, wo) > 0 ? q.Le : Spectrum(0.f));
        // UniformSampleOneLight (integrator.cpp:54-82), no light distribution: uniform choice
        const Float ul = cs.Get1D();
        const int lightNum = std::min((int)(ul * nLights), nLights - 1);
        const Float lightPdf = Float(1) / nLights;
        Float ulx, uly, usx, usy;
        cs.Get2D(&ulx, &uly);
        cs.Get2D(&usx, &usy);
        Interaction it;
        it.p = isect.p;
        it.pError = isect.pError;
        it.n = isect.n;
        it.wo = Normalize(wo);
        it.tri = isect.tri;
        *Ld = *Ld + beta * (EstimateDirect(sc, it, sc.lights[lightNum], usx, usy, ulx, uly, cs) / lightPdf);
        if (depth < maxDepth - 1) {
            Float ux, uy, pdf = 0;
            cs.Get2D(&ux, &uy);
            V3 wi;
            Spectrum f = BSDF_Sample_f(q, wo, &wi, ux, uy, &pdf);
            if (pdf == 0. || f.IsBlack()) break;
            specularBounce = false;
            beta = beta * (f * AbsDot(wi, q.n) / pdf);
            ray.o = OffsetRayOrigin(isect.p, isect.pError, isect.n, wi);
            ray.d = wi;
        }
        if (beta.y() < 0.25) {
            Float continueProb = std::min((Float)1, beta.y());
            if (cs.Get1D() > continueProb) break;
            beta = beta / continueProb;
        }
    }
    return true;
}

}  // namespace orp

extern "C" {

// Camera pass of one iteration over a width x height film: segments of every pixel in
// row-major pixel order, depth order within a pixel (up to `capacity` written; returns the
// total, or -1 if a path ran out of Halton dimensions).  ld_rgb (optional, float[3*W*H]) gets the
// surface radiance (rendersurfaces) added.
int64_t ora_camera_pass(const bre_scene *scene, int32_t width, int32_t height, int32_t iteration, int32_t max_depth,
                        int32_t render_surfaces, int32_t render_media, int64_t capacity, float *o, float *p, float *d,
                        float *tmax, int32_t *pixel, int32_t *depth, float *ld_rgb) {
    orp::Scene sc = orp::make_scene(scene);
    orp::Camera cam = orp::make_camera(scene, width, height);
    orp::Halton h(width, height);
    // GoodPixelIndex of each pixel: ParallelFor2D's serial order over 16x16 tiles, then the tile's
    // Bounds2i iteration (photonbeam.cpp:444-458)
    std::vector<uint64_t> good((size_t)width * height);
    {
        const int tileSize = 16, ntx = (width + tileSize - 1) / tileSize, nty = (height + tileSize - 1) / tileSize;
        uint64_t counter = 0;
        for (int ty = 0; ty < nty; ++ty)
            for (int tx = 0; tx < ntx; ++tx) {
                int x0 = tx * tileSize, x1 = std::min(x0 + tileSize, width);
                int y0 = ty * tileSize, y1 = std::min(y0 + tileSize, height);
                for (int y = y0; y < y1; ++y)
                    for (int x = x0; x < x1; ++x) good[(size_t)y * width + x] = counter++;
            }
    }
    std::vector<orp::Segment> segs;
    int64_t total = 0;
    for (int py = 0; py < height; ++py) {
        for (int px = 0; px < width; ++px) {
            segs.clear();
            orp::Spectrum Ld(0.f);
            if (!orp::CameraPath(sc, cam, h, px, py, width, iteration, max_depth, render_surfaces != 0,
                                 render_media != 0, good[(size_t)py * width + px], segs, &Ld))
                return -1;
            if (ld_rgb)
                for (int c = 0; c < 3; ++c) ld_rgb[3 * (py * width + px) + c] += Ld.c[c];
            for (const orp::Segment &s : segs) {
                if (total < capacity) {
                    for (int k = 0; k < 3; ++k) {
                        o[3 * total + k] = s.o[k];
                        p[3 * total + k] = s.p[k];
                        d[3 * total + k] = s.d[k];
                    }
                    tmax[total] = s.tmax;
                    pixel[total] = s.pixel;
                    depth[total] = s.depth;
                }
                ++total;
            }
        }
    }
    return total;
}

// HaltonSampler sample values for tests: out[i] = SampleDimension(IndexForSample(px, py, num), dim)
void ora_halton(int32_t width, int32_t height, int64_t n, const int32_t *px, const int32_t *py, const int64_t *num,
                const int32_t *dim, float *out) {
    orp::Halton h(width, height);
    for (int64_t i = 0; i < n; ++i) out[i] = h.SampleDimension(h.IndexForSample(px[i], py[i], num[i]), dim[i]);
}

// RadicalInverse(baseIndex, a) for baseIndex 0 (base 2) or any prime index (unscrambled)
float ora_radical_inverse(int32_t base_index, uint64_t a) {
    if (base_index == 0) return (float)((double)orp::ReverseBits64(a) * 0x1p-64);
    static std::vector<int> primes = orp::first_primes(orp::kHaltonDims);
    return orp::RadicalInverseSpecialized((uint64_t)primes[base_index], a);
}

float ora_scrambled_radical_inverse(int32_t base_index, uint64_t a, const uint16_t *perm) {
    static std::vector<int> primes = orp::first_primes(orp::kHaltonDims);
    return orp::ScrambledRadicalInverseSpecialized((uint64_t)primes[base_index], perm, a);
}

// Shuffle(perm, n, 1, RNG(seq)) (sampling.h:151-157) in place
void ora_shuffle(uint64_t seq, int32_t n, uint16_t *perm) {
    orp::RNG rng(seq);
    orp::Shuffle(perm, n, 1, rng);
}

}  // extern "C"
