// bre_camera.hip — the camera pass on the GPU: one thread per pixel walks the camera path of
// PhotonBeamIntegrator::Render (src/integrators/photonbeam.cpp:456-553) and emits the segment
// [ray.o, isect.p] of every surface-hit camera ray (the gather's input, :494-508), plus the
// surface radiance of rendersurfaces (emission + UniformSampleOneLight, :522-528).
//
// Samples: the reference's AwesomeSampler over a HaltonSampler (:456-462) — below its
// 1000-dimension switch every draw is HaltonSampler::SampleDimension(index, dim) with
// index = GetIndexForSample(iteration) of the pixel (src/samplers/halton.cpp:97-127), a pure
// function, so each thread evaluates its own dimensions; the permutation tables come from the
// host (ComputeRadicalInversePermutations with a default-seeded PCG32, lowdiscrepancy.cpp:2500).
//
// Output order: slot (depth, pixel) with pixels in 8x8-tile order, then compacted by a scan, so
// segments are depth-major and each 64-segment gather packet is one 8x8 pixel tile at one depth
// (coherent rays for the packet-proxy kernel).  Surface radiance goes straight to the pixel (one
// thread per pixel: no atomics).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "bre_device.h"
#include "bre_trace.h"

namespace bre {

// ---------------- host: Halton tables and camera constants ----------------
namespace {

uint32_t host_pcg(uint64_t &state, uint64_t inc) {
    const uint64_t old = state;
    state = old * 0x5851f42d4c957f2dULL + inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}

// RNG::UniformUInt32(b), rng.h:96-102
uint32_t host_pcg_bounded(uint64_t &state, uint64_t inc, uint32_t b) {
    const uint32_t threshold = (~b + 1u) % b;
    while (true) {
        const uint32_t r = host_pcg(state, inc);
        if (r >= threshold) return r % b;
    }
}

int64_t mod_i64(int64_t a, int64_t b) {
    const int64_t r = a - (a / b) * b;
    return r < 0 ? r + b : r;
}

void ext_gcd(uint64_t a, uint64_t b, int64_t *x, int64_t *y) {
    if (b == 0) {
        *x = 1;
        *y = 0;
        return;
    }
    const int64_t d = a / b;
    int64_t xp, yp;
    ext_gcd(b, a % b, &xp, &yp);
    *x = yp;
    *y = xp - d * yp;
}

}  // namespace

void prepare_camera(const bre_scene *s, int width, int height, DevCamera *c, std::vector<uint16_t> *perms) {
    DevCamera k{};
    k.width = width;
    k.height = height;
    // LookAt frame and screen window (perspective.cpp, CreatePerspectiveCamera)
    k.pos = mk(s->cam_pos[0], s->cam_pos[1], s->cam_pos[2]);
    const f3 look = mk(s->cam_look[0], s->cam_look[1], s->cam_look[2]);
    const f3 up = mk(s->cam_up[0], s->cam_up[1], s->cam_up[2]);
    k.dir = normalize3(sub3(look, k.pos));
    k.right = normalize3(cross3d(normalize3(up), k.dir));
    k.nup = cross3d(k.dir, k.right);
    const float aspect = (float)width / (float)height;
    if (aspect > 1.f) {
        k.sx0 = -aspect;
        k.sx1 = aspect;
        k.sy0 = -1.f;
        k.sy1 = 1.f;
    } else {
        k.sx0 = -1.f;
        k.sx1 = 1.f;
        k.sy0 = -1.f / aspect;
        k.sy1 = 1.f / aspect;
    }
    k.tan_ang = std::tan(((kPi / 180) * s->cam_fov_deg) / 2);
    k.fw = (float)width;
    k.fh = (float)height;
    // HaltonSampler ctor (halton.cpp:63-95)
    const int res[2] = {width, height};
    for (int i = 0; i < 2; ++i) {
        const int base = i == 0 ? 2 : 3;
        int scale = 1, e = 0;
        while (scale < std::min(res[i], 128)) {
            scale *= base;
            ++e;
        }
        k.base_scale[i] = scale;
        k.base_exp[i] = e;
    }
    k.stride = k.base_scale[0] * k.base_scale[1];
    for (int i = 0; i < 2; ++i) {
        int64_t x, y;
        const int64_t a = k.base_scale[1 - i], n = k.base_scale[i];
        ext_gcd((uint64_t)a, (uint64_t)n, &x, &y);
        k.mult_inv[i] = (int)mod_i64(x, n);
    }
    // first kHaltonDims primes and their permutations, drawn from RNG() in prime order
    int found = 0;
    for (int cnd = 2; found < kHaltonDims; ++cnd) {
        bool prime = true;
        for (int j = 0; j < found && k.primes[j] * k.primes[j] <= cnd; ++j)
            if (cnd % k.primes[j] == 0) {
                prime = false;
                break;
            }
        if (prime) k.primes[found++] = cnd;
    }
    int sum = 0;
    for (int i = 0; i < kHaltonDims; ++i) {
        k.prime_sums[i] = sum;
        sum += k.primes[i];
    }
    perms->assign((size_t)sum, 0);
    uint64_t st = 0x853c49e6748fea9bULL;
    const uint64_t inc = 0xda3e39cb94b95bdbULL;
    uint16_t *p = perms->data();
    for (int i = 0; i < kHaltonDims; ++i) {
        const int n = k.primes[i];
        for (int j = 0; j < n; ++j) p[j] = (uint16_t)j;
        for (int j = 0; j < n; ++j) {  // Shuffle(p, n, 1, rng)
            const int other = j + (int)host_pcg_bounded(st, inc, (uint32_t)(n - j));
            std::swap(p[j], p[other]);
        }
        p += n;
    }
    *c = k;
}

// ---------------- device ----------------
namespace {

constexpr int kCamBlock = 64;  // one 8x8 pixel tile per block

// uint64 digit loops with a 32-bit fast path (the Halton index stays below 2^32 for
// iteration < 138000 at 512x512); integer results are identical either way
__device__ __forceinline__ float radical_inverse_3(uint64_t a) {
    const float inv_base = (float)1 / (float)3;
    uint64_t rev = 0;
    float inv_n = 1;
    while (a) {
        const uint64_t next = a / 3;
        rev = rev * 3 + (a - next * 3);
        inv_n *= inv_base;
        a = next;
    }
    return smin(kOneMinusEps, (float)rev * inv_n);  // std::min(reversedDigits * invBaseN, 1-eps)
}

__device__ __forceinline__ float scrambled_radical_inverse(uint32_t base, const uint16_t *__restrict__ perm,
                                                          uint64_t a) {
    const float inv_base = (float)1 / (float)base;
    uint64_t rev = 0;
    float inv_n = 1;
    if (a < (1ull << 32)) {
        uint32_t a32 = (uint32_t)a;
        while (a32) {
            const uint32_t next = a32 / base;
            rev = rev * base + perm[a32 - next * base];
            inv_n *= inv_base;
            a32 = next;
        }
    } else {
        while (a) {
            const uint64_t next = a / base;
            rev = rev * base + perm[a - next * base];
            inv_n *= inv_base;
            a = next;
        }
    }
    return smin(kOneMinusEps, inv_n * ((float)rev + inv_base * (float)perm[0] / (1 - inv_base)));
}

__device__ __forceinline__ uint32_t rev_bits32(uint32_t n) { return __builtin_bitreverse32(n); }

// AwesomeSampler(0, tileSampler, 1000, GoodPixelIndex) (photonbeam.cpp:188-224, 459): draws
// 1..1000 are HaltonSampler dimensions 0..999 of the pixel's sample index (the two advance in
// lockstep until the switch; a Get2D that would cross it is drawn from the RNG whole), later draws
// come from PCG32 sequence GoodPixelIndex, two-draw points built right to left as in g++.
struct HaltonDev {
    const DevCamera *C;
    const uint16_t *perms;
    int64_t index;
    int count;  // AwesomeSampler::sampleCount
    Pcg rng;
    __device__ __forceinline__ float sample(int d) const {
        if (d == 0) {
            const uint64_t a = (uint64_t)(index >> C->base_exp[0]);
            const uint64_t r = ((uint64_t)rev_bits32((uint32_t)a) << 32) | rev_bits32((uint32_t)(a >> 32));
            return (float)((double)r * 0x1p-64);
        }
        if (d == 1) return radical_inverse_3((uint64_t)(index / C->base_scale[1]));
        return scrambled_radical_inverse((uint32_t)C->primes[d], perms + C->prime_sums[d], (uint64_t)index);
    }
    __device__ __forceinline__ float get1d() {
        ++count;
        if (count <= kHaltonDims) return sample(count - 1);
        return pcg_float(rng);
    }
    __device__ __forceinline__ void get2d(float &x, float &y) {
        count += 2;
        if (count <= kHaltonDims) {
            x = sample(count - 2);
            y = sample(count - 1);
        } else {
            pcg_2d(rng, x, y);
        }
    }
};
__device__ __forceinline__ float smp_1d(HaltonDev &h) { return h.get1d(); }

// GoodPixelIndex = globalNumPixels (always 0) + iterNumPixels++ (photonbeam.cpp:351, 457-458).  The
// reference increments that counter from every camera-pass thread without synchronisation, so its
// value is scheduling-dependent; we use the single-threaded order (tiles row-major, ParallelFor2D's
// serial loop, then Bounds2i iteration order x-fastest inside the 16x16 tile).  It only seeds the
// PCG32 draws past the 1000th of a path.
__device__ __forceinline__ uint64_t good_pixel_index(int W, int H, int px, int py) {
    const int tx = px >> 4, ty = py >> 4;
    const int th = min(16, H - ty * 16), tw = min(16, W - tx * 16);
    return (uint64_t)ty * 16 * (uint64_t)W + (uint64_t)tx * 16 * (uint64_t)th + (uint64_t)((py & 15) * tw + (px & 15));
}

__device__ __forceinline__ uint64_t inv_radical_inverse(uint64_t base, uint64_t inverse, int ndig) {
    uint64_t idx = 0;
    for (int i = 0; i < ndig; ++i) {
        const uint64_t digit = inverse % base;
        inverse /= base;
        idx = idx * base + digit;
    }
    return idx;
}

// GetIndexForSample (halton.cpp:97-115)
__device__ __forceinline__ int64_t halton_index(const DevCamera &C, int px, int py, int64_t sample_num) {
    int64_t off = 0;
    if (C.stride > 1) {
        const int pm[2] = {px & 127, py & 127};  // Mod(p, kMaxResolution) for p >= 0
        for (int i = 0; i < 2; ++i) {
            const uint64_t dim_off = inv_radical_inverse(i == 0 ? 2 : 3, (uint64_t)pm[i], C.base_exp[i]);
            off += dim_off * (uint64_t)(C.stride / C.base_scale[i]) * (uint64_t)C.mult_inv[i];
        }
        off %= C.stride;
    }
    return off + sample_num * C.stride;
}

// ---- matte triangle BSDF (reflection.cpp:650-768) ----
__device__ __forceinline__ f3 to_local(const PTri &q, f3 v) { return mk(dot3(v, q.ss), dot3(v, q.ts), dot3(v, q.n)); }
__device__ __forceinline__ f3 to_world(const PTri &q, f3 v) {
    return mk(q.ss.x * v.x + q.ts.x * v.y + q.n.x * v.z, q.ss.y * v.x + q.ts.y * v.y + q.n.y * v.z,
              q.ss.z * v.x + q.ts.z * v.y + q.n.z * v.z);
}
__device__ __forceinline__ void bsdf_f(const PTri &q, f3 wo_w, f3 wi_w, float f[3]) {
    f[0] = f[1] = f[2] = 0.f;
    if (q.absorb) return;
    if (to_local(q, wo_w).z == 0) return;
    const bool reflect = dot3(wi_w, q.n) * dot3(wo_w, q.n) > 0;
    if (reflect)
        for (int c = 0; c < 3; ++c) f[c] = 0.f + q.kd[c] * kInvPi;
}
__device__ __forceinline__ float bsdf_pdf(const PTri &q, f3 wo_w, f3 wi_w) {
    if (q.absorb) return 0.f;
    const f3 wo = to_local(q, wo_w), wi = to_local(q, wi_w);
    if (wo.z == 0) return 0.f;
    float pdf = 0.f;
    pdf += (wo.z * wi.z > 0) ? fabsf(wi.z) * kInvPi : 0.f;
    return pdf / 1;
}
// BSDF::Sample_f; *pdf untouched when wo.z == 0 (as the reference); returns false for f = 0
__device__ __forceinline__ bool bsdf_sample(const PTri &q, f3 wo_w, float ux, float uy, f3 &wi_w, float &pdf,
                                            float f[3]) {
    f[0] = f[1] = f[2] = 0.f;
    if (q.absorb) {
        pdf = 0.f;
        return false;
    }
    const f3 wo = to_local(q, wo_w);
    if (wo.z == 0) return false;
    f3 wi = cosine_hemisphere(ux, uy);
    if (wo.z < 0) wi.z *= -1;
    pdf = (wo.z * wi.z > 0) ? fabsf(wi.z) * kInvPi : 0.f;
    if (pdf == 0) return false;
    wi_w = to_world(q, wi);
    for (int c = 0; c < 3; ++c) f[c] = q.kd[c] * kInvPi;
    return true;
}

__device__ __forceinline__ float power_heuristic(float fpdf, float gpdf) {
    const float f = 1 * fpdf, g = 1 * gpdf;
    return (f * f) / (f * f + g * g);
}

// EstimateDirect (integrator.cpp:108-214) for the area light on triangle `li`, handleMedia = true
__device__ void estimate_direct(const DevScene &S, HaltonDev &hs, f3 p, f3 perr, const PTri &q, f3 wo, int li,
                                float usx, float usy, float ulx, float uly, float Ld[3]) {
    const PTri &L = S.t[li];
    Ld[0] = Ld[1] = Ld[2] = 0.f;
    float scat_pdf = 0.f;
    // DiffuseAreaLight::Sample_Li (diffuse.cpp:68-81) -> Shape::Sample(ref, u) (shape.cpp:56-70)
    const ShapeSample ps = sample_tri(L, ulx, uly);
    const f3 sp = ps.p;
    float light_pdf = ps.pdf;
    f3 w = sub3(sp, p);
    if (lensq3(w) == 0) {
        light_pdf = 0;
    } else {
        w = normalize3(w);
        light_pdf *= lensq3(sub3(p, sp)) / fabsf(dot3(ps.n, neg3(w)));
        if (isinf(light_pdf)) light_pdf = 0.f;
    }
    f3 wi = mk(0, 0, 0);
    float Li[3] = {0.f, 0.f, 0.f};
    if (light_pdf == 0 || lensq3(sub3(sp, p)) == 0) {
        light_pdf = 0;
    } else {
        wi = normalize3(sub3(sp, p));
        if (dot3(ps.n, neg3(wi)) > 0)
            for (int c = 0; c < 3; ++c) Li[c] = L.Le[c];
    }
    if (light_pdf > 0 && !black3(Li)) {
        float f[3];
        bsdf_f(q, wo, wi, f);
        const float ad = fabsf(dot3(wi, q.n));
        for (int c = 0; c < 3; ++c) f[c] = f[c] * ad;
        scat_pdf = bsdf_pdf(q, wo, wi);
        if (!black3(f)) {
            // VisibilityTester::Tr over Interaction::SpawnRayTo(pShape)
            const f3 ro = offset_origin(p, perr, q.n, sub3(sp, p));
            const f3 target = offset_origin(sp, ps.perr, ps.n, sub3(ro, sp));
            const f3 rd = sub3(target, ro);
            float tmax = 1 - 0.0001f;
            Hit h;
            if (intersect_scene(S, ro, rd, tmax, h)) {
                Li[0] = Li[1] = Li[2] = 0.f;  // every triangle has a material
            } else if (S.medium) {
                float tr[3];
                medium_tr_any(S, hs, ro, rd, tmax, tr);
                for (int c = 0; c < 3; ++c) Li[c] = Li[c] * (1.f * tr[c]);
            }
            if (!black3(Li)) {
                const float wgt = power_heuristic(light_pdf, scat_pdf);
                for (int c = 0; c < 3; ++c) Ld[c] = Ld[c] + f[c] * Li[c] * wgt / light_pdf;
            }
        }
    }
    // BSDF sampling
    {
        float f[3];
        bsdf_sample(q, wo, usx, usy, wi, scat_pdf, f);
        const float ad = fabsf(dot3(wi, q.n));
        for (int c = 0; c < 3; ++c) f[c] = f[c] * ad;
        if (!black3(f) && scat_pdf > 0) {
            // DiffuseAreaLight::Pdf_Li -> Shape::Pdf(ref, wi) (shape.cpp:72-87): this triangle alone
            const f3 ro = offset_origin(p, perr, q.n, wi);
            float tl;
            Hit hl;
            if (!intersect_tri(L, ro, wi, __builtin_huge_valf(), tl, hl)) return;
            light_pdf = lensq3(sub3(p, hl.p)) / (fabsf(dot3(L.n, neg3(wi))) * L.area);
            if (isinf(light_pdf)) light_pdf = 0.f;
            if (light_pdf == 0) return;
            const float wgt = power_heuristic(scat_pdf, light_pdf);
            float tmax = __builtin_huge_valf();
            Hit h;
            const bool found = intersect_scene(S, ro, wi, tmax, h);
            float tr[3] = {1.f, 1.f, 1.f};
            if (S.medium) {
                float t2[3];
                medium_tr_any(S, hs, ro, wi, tmax, t2);
                for (int c = 0; c < 3; ++c) tr[c] = tr[c] * t2[c];
            }
            // lightIsect.primitive->GetAreaLight() == &light: the same triangle, one-sided
            if (found && h.tri == li && dot3(L.n, neg3(wi)) > 0 && !black3(L.Le))
                for (int c = 0; c < 3; ++c) Ld[c] = Ld[c] + f[c] * L.Le[c] * tr[c] * wgt / scat_pdf;
        }
    }
}

__global__ __launch_bounds__(kCamBlock, 6) void k_camera(const DevScene *__restrict__ Sp, const DevCamera *__restrict__ Cp,
                                                     const uint16_t *__restrict__ perms, int iteration, int max_depth,
                                                     int render_surfaces, int render_media, int64_t nslots,
                                                     float *__restrict__ so, float *__restrict__ sp_,
                                                     float *__restrict__ sd, float *__restrict__ st,
                                                     int32_t *__restrict__ spix, int32_t *__restrict__ valid,
                                                     float *__restrict__ surface, unsigned int *__restrict__ flags,
                                                     int shard_rank, int shard_count, int shard_block, int classes) {
    const DevScene &S = *Sp;
    const DevCamera &C = *Cp;
    const int64_t slot = (int64_t)blockIdx.x * kCamBlock + threadIdx.x;
    const int tiles_x = (C.width + 7) / 8;
    const int px = (int)(blockIdx.x % tiles_x) * 8 + (int)(threadIdx.x & 7);
    const int py = (int)(blockIdx.x / tiles_x) * 8 + (int)(threadIdx.x >> 3);
    for (int dd = 0; dd < max_depth; ++dd) valid[dd * nslots + slot] = 0;
    if (px >= C.width || py >= C.height) return;
    // image-tile sharding: this context walks only the reference's 16x16 camera-pass tiles
    // (photonbeam.cpp:345-347, 444-452) of the blocks of shard_block x shard_block tiles whose
    // row-major block index = rank (mod count).  shard_block 0 is the PACKET sharding: every tile is
    // walked (the gather takes the rank's range of sorted packets) and the surface radiance of pixel p
    // is added by rank p mod count only, so the ranks' films sum to the whole film.
    const bool packet_shard = shard_block == 0;
    if (shard_count > 1 && !packet_shard) {
        const int nbx = (((C.width + 15) >> 4) + shard_block - 1) / shard_block;
        if ((((py >> 4) / shard_block) * nbx + (px >> 4) / shard_block) % shard_count != shard_rank) return;
    }
    const int pixel = py * C.width + px;

    HaltonDev hs{Cp, perms, halton_index(C, px, py, iteration), 0, Pcg{}};
    pcg_seed(hs.rng, good_pixel_index(C.width, C.height, px, py));
    float fx, fy, lx, ly;
    hs.get2d(fx, fy);
    fx = (float)px + fx;
    fy = (float)py + fy;
    (void)hs.get1d();  // time
    hs.get2d(lx, ly);  // lens (pinhole)
    // pinhole camera ray (DESIGN.md "Camera pass": pbrt's screen window, LookAt frame and
    // Transform::operator()(Ray) origin offset)
    const float sx = C.sx0 + (fx / C.fw) * (C.sx1 - C.sx0);
    const float sy = C.sy1 - (fy / C.fh) * (C.sy1 - C.sy0);
    const f3 dc = normalize3(mk(sx * C.tan_ang, sy * C.tan_ang, 1));
    f3 d = add3(add3(scale3(C.right, dc.x), scale3(C.nup, dc.y)), scale3(C.dir, dc.z));
    f3 o = C.pos;
    {
        const f3 oerr = scale3(abs3(C.pos), gamma_n(3));
        const float l2 = lensq3(d);
        if (l2 > 0) {
            const float dt = dot3(abs3(d), oerr) / l2;
            o = add3(o, scale3(d, dt));
        }
    }
    float beta[3] = {1.f, 1.f, 1.f};
    float Ld[3] = {0.f, 0.f, 0.f};
    for (int depth = 0; depth < max_depth; ++depth) {
        float tmax = __builtin_huge_valf();
        Hit hit;
        if (!intersect_scene(S, o, d, tmax, hit)) break;  // area lights: Le(ray) = 0
        float mb[3] = {1.f, 1.f, 1.f};
        if (S.medium) medium_tr_any(S, hs, o, d, tmax, mb);
        if (render_media) {
            const int64_t k = depth * nslots + slot;
            so[3 * k + 0] = o.x;
            so[3 * k + 1] = o.y;
            so[3 * k + 2] = o.z;
            sp_[3 * k + 0] = hit.p.x;
            sp_[3 * k + 1] = hit.p.y;
            sp_[3 * k + 2] = hit.p.z;
            sd[3 * k + 0] = d.x;
            sd[3 * k + 1] = d.y;
            sd[3 * k + 2] = d.z;
            st[k] = tmax;
            spix[k] = pixel;
            valid[k] = 1;
        }
        for (int c = 0; c < 3; ++c) beta[c] = beta[c] * mb[c];
        if (!render_surfaces) break;
        const PTri &q = S.t[hit.tri];
        const f3 wo = neg3(d);
        // isect.Le(wo): the triangle's own area light, one-sided (diffuse.h:56-58)
        if (depth == 0 && q.emit && dot3(q.n, wo) > 0)
            for (int c = 0; c < 3; ++c) Ld[c] = Ld[c] + beta[c] * q.Le[c];
        // UniformSampleOneLight (integrator.cpp:54-82): light uniformly, uLight, uScattering
        const int ln = min((int)(hs.get1d() * S.n_lights), S.n_lights - 1);
        const float light_pdf = 1.f / (float)S.n_lights;  // Float(1) / nLights
        float ulx, uly, usx, usy;
        hs.get2d(ulx, uly);
        hs.get2d(usx, usy);
        float ed[3];
        estimate_direct(S, hs, hit.p, hit.perr, q, normalize3(wo), S.light_tri[ln], usx, usy, ulx, uly, ed);
        for (int c = 0; c < 3; ++c) Ld[c] = Ld[c] + beta[c] * (ed[c] / light_pdf);
        if (depth < max_depth - 1) {
            float ux, uy, pdf = 0.f, f[3];
            hs.get2d(ux, uy);
            f3 wi;
            if (!bsdf_sample(q, wo, ux, uy, wi, pdf, f) || pdf == 0 || black3(f)) break;
            const float ad = fabsf(dot3(wi, q.n));
            for (int c = 0; c < 3; ++c) beta[c] = beta[c] * (f[c] * ad / pdf);
            o = offset_origin(hit.p, hit.perr, q.n, wi);
            d = wi;
        }
        const float y = lum3(beta);
        if (y < 0.25f) {
            const float cp = smin(1.f, y);  // std::min((Float)1, beta.y())
            if (hs.get1d() > cp) break;
            for (int c = 0; c < 3; ++c) beta[c] = beta[c] / cp;
        }
    }
    // film classes (BRE_OPT_FILM_CLASSES): pixel p's surface radiance goes to plane p % classes
    if (surface && render_surfaces && (!packet_shard || pixel % shard_count == shard_rank)) {
        float *sf = surface + 3 * ((int64_t)(pixel % classes) * C.width * C.height + pixel);
        for (int c = 0; c < 3; ++c) sf[c] += Ld[c];
    }
}

__global__ void k_compact(int64_t nslots_total, const int32_t *__restrict__ valid, const int64_t *__restrict__ offs,
                          const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
                          const float *__restrict__ st, const int32_t *__restrict__ spix, float *__restrict__ o,
                          float *__restrict__ p, float *__restrict__ d, float *__restrict__ t, int32_t *__restrict__ pix,
                          int32_t *__restrict__ depth, int64_t nslots) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nslots_total || !valid[k]) return;
    const int64_t w = offs[k];
    for (int c = 0; c < 3; ++c) {
        o[3 * w + c] = so[3 * k + c];
        p[3 * w + c] = sp_[3 * k + c];
        d[3 * w + c] = sd[3 * k + c];
    }
    t[w] = st[k];
    pix[w] = spix[k];
    if (depth) depth[w] = (int32_t)(k / nslots);
}

}  // namespace

int64_t camera_slots(int width, int height) {
    return (int64_t)((width + 7) / 8) * ((height + 7) / 8) * 64;
}

hipError_t launch_camera(const DevScene *scene, int stack_depth, const DevCamera *cam, const uint16_t *perms, int width,
                         int height, int iteration, int max_depth, int render_surfaces, int render_media,
                         const CamSlots &s, float *surface, unsigned int *flags, int shard_rank, int shard_count,
                         int shard_block, int classes, hipStream_t stream) {
    const int64_t nslots = camera_slots(width, height);
    if (nslots == 0) return hipSuccess;
    hipLaunchKernelGGL(k_camera, dim3((unsigned)(nslots / kCamBlock)), dim3(kCamBlock),
                       scene_stack_bytes(stack_depth, kCamBlock), stream, scene, cam, perms,
                       iteration, max_depth, render_surfaces, render_media, nslots, s.o, s.p, s.d, s.t, s.pix,
                       s.valid, surface, flags, shard_rank, shard_count, shard_block, classes < 1 ? 1 : classes);
    return hipGetLastError();
}

size_t camera_scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::exclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int64_t *)nullptr, int64_t(0),
                                  (size_t)n, rocprim::plus<int64_t>());
    return std::max(bytes, slot_scan_temp_bytes(n));
}

hipError_t launch_camera_scan(void *tmp, size_t tmp_bytes, const CamSlots &s, int64_t nslots, int max_depth,
                              int64_t *offs, hipStream_t stream, bool slot) {
    const int64_t total = nslots * max_depth;
    if (total == 0) return hipSuccess;
    if (slot) return slot_exclusive_scan(s.valid, offs, total, nullptr, tmp, stream);  // one-wave (bre_slot.hip)
    return rocprim::exclusive_scan(tmp, tmp_bytes, s.valid, offs, int64_t(0), (size_t)total, rocprim::plus<int64_t>(),
                                   stream);
}

hipError_t launch_camera_compact(const CamSlots &s, int64_t nslots, int max_depth, const int64_t *offs, float *o,
                                 float *p, float *d, float *t, int32_t *pix, int32_t *depth, hipStream_t stream) {
    const int64_t total = nslots * max_depth;
    if (total == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((total + 63) / 64);  // one-wave workgroups (bre_slot.hip)
    hipLaunchKernelGGL(k_compact, dim3(blocks), dim3(64), 0, stream, total, s.valid, offs, s.o, s.p, s.d, s.t,
                       s.pix, o, p, d, t, pix, depth, nslots);
    return hipGetLastError();
}

}  // namespace bre
