// bre_photon.hip — the photon pass on the GPU: emission + TracePhotonBeamRecursive
// (src/integrators/photonbeam.cpp:258-325, 383-421) for every photon of an iteration, one thread
// per photon, producing the beam set the gather consumes.
//
// The reference recurses on every medium scattering event (the scattered photon is traced to
// completion, then the parent path continues, :274-288).  Here the recursion is an explicit
// per-thread stack of suspended parent frames (at most maxdepth of them, since each level adds
// one to depth), and the random numbers are drawn in exactly the reference's order from the
// photon's own PCG32 sequence iter*N + i + 1 (:386-389), so each photon's beams, their order and
// their bits are those of the reference's single-threaded loop.
//
// Output is deterministic and photon-major: pass 1 counts each photon's beams, an inclusive scan
// gives offsets, pass 2 re-traces and writes beam k of photon i at offsets[i] + k.  Tracing twice
// costs less than the atomics + sort a single pass would need to restore the order, and keeps
// memory at exactly the beam count (the per-photon bound 2^maxdepth - 1 would be 31x at depth 5).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>

#include "bre_device.h"
#include "bre_trace.h"

namespace bre {

float grid_max_density(const bre_scene *s) {
    float mx = 0;
    const int64_t n = (int64_t)s->grid_n[0] * s->grid_n[1] * s->grid_n[2];
    for (int64_t i = 0; i < n; ++i) mx = std::max(mx, s->grid_density[i]);
    return mx;
}

void prepare_scene(const bre_scene *s, DevScene *out, const float *d_density) {
    DevScene d{};
    d.n_quads = s->n_quads;
    d.light = s->light_quad;
    d.medium = s->has_medium == BRE_MEDIUM_GRID ? BRE_MEDIUM_GRID : (s->has_medium ? BRE_MEDIUM_HOMOGENEOUS : 0);
    if (d.medium == BRE_MEDIUM_GRID) {
        // GridDensityMedium ctor (grid.h:58-77): sigma_t = (sigma_a + sigma_s)[0]; invMaxDensity
        for (int k = 0; k < 3; ++k) d.gn[k] = s->grid_n[k];
        d.grid_sigma_t = s->sigma_a[0] + s->sigma_s[0];
        d.grid_inv_max = 1 / grid_max_density(s);
        for (int k = 0; k < 16; ++k) d.w2m[k] = s->world_to_medium[k];
        d.density = d_density;
    }
    for (int c = 0; c < 3; ++c) {
        d.Le[c] = s->light_L[c];
        d.sigma_t[c] = s->sigma_a[c] + s->sigma_s[c];  // HomogeneousMedium ctor: sigma_a + sigma_s
    }
    d.g = s->g;
    for (int i = 0; i < s->n_quads; ++i) {
        const bre_quad &q = s->quads[i];
        PQuad &Q = d.q[i];
        Q.p0 = mk(q.p0[0], q.p0[1], q.p0[2]);
        Q.e1 = mk(q.e1[0], q.e1[1], q.e1[2]);
        Q.e2 = mk(q.e2[0], q.e2[1], q.e2[2]);
        const f3 c = cross3d(Q.e1, Q.e2);
        Q.area = len3(c);
        Q.n = normalize3(c);
        Q.ss = normalize3(Q.e1);
        Q.ts = cross3d(Q.n, Q.ss);
        Q.inv_e1sq = 1 / dot3(Q.e1, Q.e1);
        Q.inv_e2sq = 1 / dot3(Q.e2, Q.e2);
        for (int k = 0; k < 3; ++k) Q.kd[k] = q.kd[k];
        Q.absorb = (q.kd[0] == 0 && q.kd[1] == 0 && q.kd[2] == 0) ? 1 : 0;
    }
    *out = d;
}

namespace {

constexpr int kPhotonBlock = 128;

// A path suspended at a medium scattering event while its scattered child is traced.
struct Frame {
    f3 o, d;     // photonRay
    float tmax;  // its surface hit distance
    f3 p, perr;  // isect.p and its error bound
    int quad;
    int depth;
    float beta[3];
};

template <bool EMIT>
__global__ __launch_bounds__(kPhotonBlock) void k_photons(const DevScene *__restrict__ Sp, int64_t n, uint64_t seq0,
                                                          int max_depth, float radius, int32_t *__restrict__ counts,
                                                          const int64_t *__restrict__ offsets, float *__restrict__ bs,
                                                          float *__restrict__ be, float *__restrict__ br,
                                                          float *__restrict__ bp) {
    const int64_t i = (int64_t)blockIdx.x * kPhotonBlock + threadIdx.x;
    if (i >= n) return;
    const DevScene &S = *Sp;
    Pcg rng;
    pcg_seed(rng, seq0 + (uint64_t)i);
    int64_t w = EMIT ? offsets[i] : 0;
    int cnt = 0;

    // ---- emission, photonbeam.cpp:393-418 (one light: lightPdf = 1) ----
    (void)pcg_float(rng);  // lightSample
    float u0x, u0y, u1x, u1y;
    pcg_2d(rng, u0x, u0y);
    pcg_2d(rng, u1x, u1y);
    (void)pcg_float(rng);  // uLightTime
    const PQuad &L = S.q[S.light];
    const f3 ue1 = scale3(L.e1, u0x), ve2 = scale3(L.e2, u0y);
    const f3 lp = add3(add3(L.p0, ue1), ve2);
    const f3 lperr = scale3(add3(add3(abs3(L.p0), abs3(ue1)), abs3(ve2)), gamma_n(6));
    const float pdf_pos = 1 / L.area;
    const f3 wl = cosine_hemisphere(u1x, u1y);
    const float pdf_dir = wl.z * kInvPi;
    f3 v1, v2;
    coord_system(L.n, v1, v2);
    f3 d = add3(add3(scale3(v1, wl.x), scale3(v2, wl.y)), scale3(L.n, wl.z));
    f3 o = offset_origin(lp, lperr, L.n, d);
    const bool front = dot3(L.n, d) > 0;  // DiffuseAreaLight::L, one-sided
    float beta[3];
    bool alive = !(pdf_pos == 0 || pdf_dir == 0 || !front || black3(S.Le));
    if (alive) {
        const float ad = fabsf(dot3(L.n, d));
        const float den = 1.0f * pdf_pos * pdf_dir;
        for (int c = 0; c < 3; ++c) beta[c] = (ad * S.Le[c]) / den;
        alive = !black3(beta);
    }

    // ---- TracePhotonBeamRecursive as a state machine ----
    Frame stk[BRE_MAX_DEPTH];
    int sp = 0;
    int depth = 0;
    float tmax = 0;
    Hit hit;
    bool resume = false;
    while (alive) {
        bool stop = false;
        if (!resume) {
            tmax = __builtin_huge_valf();
            if (depth >= max_depth || !intersect_scene(S, o, d, tmax, hit)) {
                stop = true;
            } else {
                bool scattered = false;
                float ts = 0;
                if (S.medium) scattered = medium_sample_any(S, rng, o, d, tmax, ts);
                if (black3(beta)) {
                    stop = true;
                } else if (scattered) {
                    // HG direction from the scattering point; the child path starts there with
                    // beta * Tr(whole segment) (photonbeam.cpp:276-285)
                    float hx, hy;
                    pcg_2d(rng, hx, hy);
                    const f3 wi = hg_sample(S.g, neg3(d), hx, hy);
                    float tr[3];
                    medium_tr_any(S, rng, o, d, tmax, tr);
                    Frame &f = stk[sp++];
                    f.o = o;
                    f.d = d;
                    f.tmax = tmax;
                    f.p = hit.p;
                    f.perr = hit.perr;
                    f.quad = hit.quad;
                    f.depth = depth;
                    for (int c = 0; c < 3; ++c) {
                        f.beta[c] = beta[c];
                        beta[c] = beta[c] * tr[c];
                    }
                    o = ray_at(o, d, ts);  // MediumInteraction::SpawnRay: no offset
                    d = wi;
                    depth += 1;
                    continue;
                }
            }
        }
        if (!stop) {
            resume = false;
            // beam for the whole surface-hit segment, powerEnd = Tr * beta (:289-294)
            float bm[3] = {1.f, 1.f, 1.f};
            if (S.medium) medium_tr_any(S, rng, o, d, tmax, bm);
            if (EMIT) {
                const int64_t k = w + cnt;
                bs[3 * k + 0] = o.x;
                bs[3 * k + 1] = o.y;
                bs[3 * k + 2] = o.z;
                be[3 * k + 0] = hit.p.x;
                be[3 * k + 1] = hit.p.y;
                be[3 * k + 2] = hit.p.z;
                br[k] = radius;
                for (int c = 0; c < 3; ++c) bp[3 * k + c] = bm[c] * beta[c];
            }
            ++cnt;
            // surface scattering (:296-323): Lambertian BSDF::Sample_f
            float ux, uy;
            pcg_2d(rng, ux, uy);
            const PQuad &q = S.q[hit.quad];
            if (q.absorb) {
                stop = true;
            } else {
                const f3 wo = neg3(d);
                const float woz = dot3(wo, q.n);
                if (woz == 0) {
                    stop = true;
                } else {
                    f3 wil = cosine_hemisphere(ux, uy);
                    if (woz < 0) wil.z *= -1;
                    const float pdf = (woz * wil.z > 0) ? fabsf(wil.z) * kInvPi : 0.f;
                    float fr[3];
                    for (int c = 0; c < 3; ++c) fr[c] = q.kd[c] * kInvPi;
                    if (pdf == 0 || black3(fr)) {
                        stop = true;
                    } else {
                        const f3 wi = mk(q.ss.x * wil.x + q.ts.x * wil.y + q.n.x * wil.z,
                                         q.ss.y * wil.x + q.ts.y * wil.y + q.n.y * wil.z,
                                         q.ss.z * wil.x + q.ts.z * wil.y + q.n.z * wil.z);
                        const float ad = fabsf(dot3(wi, q.n));
                        float bn[3];
                        for (int c = 0; c < 3; ++c) bn[c] = bm[c] * beta[c] * fr[c] * ad / pdf;
                        o = offset_origin(hit.p, hit.perr, q.n, wi);
                        d = wi;
                        const float qrr = smax(0.f, 1 - lum3(bn) / lum3(beta));
                        if (pcg_float(rng) < qrr) {
                            stop = true;
                        } else {
                            for (int c = 0; c < 3; ++c) beta[c] = bn[c] / (1 - qrr);
                            depth += 1;
                        }
                    }
                }
            }
            if (!stop) continue;
        }
        // this path ends: resume the innermost suspended parent after its recursive call
        if (sp == 0) break;
        const Frame &f = stk[--sp];
        o = f.o;
        d = f.d;
        tmax = f.tmax;
        hit.p = f.p;
        hit.perr = f.perr;
        hit.quad = f.quad;
        depth = f.depth;
        for (int c = 0; c < 3; ++c) beta[c] = f.beta[c];
        resume = true;
    }
    if (!EMIT) counts[i] = cnt;
}

inline unsigned grid_of(int64_t n) { return (unsigned)((n + kPhotonBlock - 1) / kPhotonBlock); }

}  // namespace

hipError_t launch_photons(const DevScene *scene, int64_t n, uint64_t seq0, int max_depth, float radius,
                          int32_t *counts, const int64_t *offsets, float *start, float *end, float *rad,
                          float *power, bool emit, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (emit)
        hipLaunchKernelGGL(k_photons<true>, dim3(grid_of(n)), dim3(kPhotonBlock), 0, s, scene, n, seq0, max_depth,
                           radius, counts, offsets, start, end, rad, power);
    else
        hipLaunchKernelGGL(k_photons<false>, dim3(grid_of(n)), dim3(kPhotonBlock), 0, s, scene, n, seq0, max_depth,
                           radius, counts, offsets, start, end, rad, power);
    return hipGetLastError();
}

size_t count_scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int64_t *)nullptr, (size_t)n,
                                  rocprim::plus<int64_t>());
    return bytes;
}

// offsets[0] = 0, offsets[k + 1] = counts[0] + ... + counts[k]
hipError_t launch_count_scan(void *tmp, size_t bytes, const int32_t *counts, int64_t *offsets, int64_t n,
                             hipStream_t s) {
    hipError_t e = hipMemsetAsync(offsets, 0, sizeof(int64_t), s);
    if (e != hipSuccess || n == 0) return e;
    return rocprim::inclusive_scan(tmp, bytes, counts, offsets + 1, (size_t)n, rocprim::plus<int64_t>(), s);
}

}  // namespace bre
