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
// Output is deterministic and photon-major: beam k of photon i lands at offsets[i] + k, offsets the
// inclusive scan of the per-photon counts.  The default single-trace form (round 4) traces each photon
// once, writing its first `cap` beams to the photon's own slots of a scratch array and its count;
// after the scan a copy puts the slots at their offsets, and only the photons with more than `cap`
// beams are traced again, straight to their offsets (the same code and random sequence: the same
// bits).  cap is sized so the scratch stays within 2.5 GB (62 slots at 1M photons; C2's photons
// average 2.7 beams, but the few long paths re-traced past 16 slots cost 0.25 ms); the two-trace form
// (count, scan, re-trace every photon) is the fallback.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <vector>

#include "bre_device.h"
#include "bre_trace.h"

namespace bre {

float grid_max_density(const bre_scene *s) {
    float mx = 0;
    const int64_t n = (int64_t)s->grid_n[0] * s->grid_n[1] * s->grid_n[2];
    for (int64_t i = 0; i < n; ++i) mx = std::max(mx, s->grid_density[i]);
    return mx;
}

void prepare_medium(const bre_scene *s, DevScene *dp, const float *d_density) {
    DevScene &d = *dp;
    d.medium = s->has_medium == BRE_MEDIUM_GRID ? BRE_MEDIUM_GRID : (s->has_medium ? BRE_MEDIUM_HOMOGENEOUS : 0);
    if (d.medium == BRE_MEDIUM_GRID) {
        // GridDensityMedium ctor (grid.h:58-77): sigma_t = (sigma_a + sigma_s)[0]; invMaxDensity
        for (int k = 0; k < 3; ++k) d.gn[k] = s->grid_n[k];
        d.grid_sigma_t = s->sigma_a[0] + s->sigma_s[0];
        d.grid_inv_max = 1 / grid_max_density(s);
        for (int k = 0; k < 16; ++k) d.w2m[k] = s->world_to_medium[k];
        d.density = d_density;
    }
    for (int c = 0; c < 3; ++c)
        d.sigma_t[c] = s->sigma_a[c] + s->sigma_s[c];  // HomogeneousMedium ctor: sigma_a + sigma_s
    d.g = s->g;
}

void prepare_geometry(const bre_scene *s, HostScene *out) {
    DevScene &d = out->head;
    d.n_tris = s->n_triangles;
    const bre_triangle *tri = scene_triangles(s);
    out->tris.resize((size_t)s->n_triangles);
    out->light_tri.clear();
    out->light_func.clear();
    for (int i = 0; i < s->n_triangles; ++i) {
        const bre_triangle &t = tri[i];
        PTri &T = out->tris[(size_t)i];
        T.p0 = mk(t.p[0][0], t.p[0][1], t.p[0][2]);
        T.p1 = mk(t.p[1][0], t.p[1][1], t.p[1][2]);
        T.p2 = mk(t.p[2][0], t.p[2][1], t.p[2][2]);
        const f3 dp02 = sub3(T.p0, T.p2), dp12 = sub3(T.p1, T.p2);
        // dpdu for pbrt's default uvs (0,0), (1,0), (1,1): (duv12[1] dp02 - duv02[1] dp12) invdet
        // with duv12[1] = duv02[1] = -1, invdet = 1 (triangle.cpp:276-285)
        const f3 dpdu = scale3(sub3(scale3(dp02, -1.f), scale3(dp12, -1.f)), 1.f);
        T.n = normalize3(cross3d(dp02, dp12));
        T.ns = normalize3(cross3d(sub3(T.p1, T.p0), sub3(T.p2, T.p0)));
        if (t.flip) {
            T.n = neg3(T.n);
            T.ns = neg3(T.ns);
        }
        T.ss = normalize3(dpdu);
        T.ts = cross3d(T.n, T.ss);
        T.area = (float)(0.5 * (double)len3(cross3d(sub3(T.p1, T.p0), sub3(T.p2, T.p0))));
        for (int k = 0; k < 3; ++k) {
            T.kd[k] = t.kd[k];
            T.Le[k] = t.Le[k];
        }
        T.absorb = (t.kd[0] == 0 && t.kd[1] == 0 && t.kd[2] == 0) ? 1 : 0;
        T.emit = t.emit != 0;
        if (T.emit) {
            out->light_tri.push_back(i);
            // DiffuseAreaLight::Power() = (twoSided ? 2 : 1) * Lemit * area * Pi (diffuse.cpp:64-66), .y()
            float pw[3];
            for (int k = 0; k < 3; ++k) pw[k] = ((T.Le[k] * 1.f) * T.area) * kPi;
            out->light_func.push_back(lum3(pw));
        }
    }
    const int nl = (int)out->light_tri.size();
    d.n_lights = nl;
    // Distribution1D(func, n) (sampling.h:57-69)
    std::vector<float> &cdf = out->light_cdf;
    const std::vector<float> &func = out->light_func;
    cdf.assign((size_t)nl + 1, 0.f);
    for (int i = 1; i < nl + 1; ++i) cdf[(size_t)i] = cdf[(size_t)i - 1] + func[(size_t)i - 1] / (float)nl;
    d.light_func_int = cdf[(size_t)nl];
    if (d.light_func_int == 0) {
        for (int i = 1; i < nl + 1; ++i) cdf[(size_t)i] = (float)i / (float)nl;
    } else {
        for (int i = 1; i < nl + 1; ++i) cdf[(size_t)i] /= d.light_func_int;
    }
    out->depth = build_scene_bvh(out->tris, &out->nodes, &out->prims);
    d.n_nodes = (int)out->nodes.size();
    d.stack_depth = out->depth;
}

void prepare_scene(const bre_scene *s, HostScene *out, const float *d_density) {
    out->head = DevScene{};
    prepare_geometry(s, out);
    prepare_medium(s, &out->head, d_density);
}

namespace {

#ifndef BRE_PHOTON_BLOCK
#define BRE_PHOTON_BLOCK 64  // one wave: fits a concurrent gather's slots (bre_slot.hip; 128 until round 5)
#endif
constexpr int kPhotonBlock = BRE_PHOTON_BLOCK;

// A path suspended at a medium scattering event while its scattered child is traced.
struct Frame {
    f3 o, d;     // photonRay
    float tmax;  // its surface hit distance
    f3 p, perr;  // isect.p and its error bound
    int tri;
    int depth;
    float beta[3];
};

// MODE 0: count each photon's beams; 1: write them at offsets[i] + k (with over > 0: only the photons
// whose count exceeds `over`, the single-trace form's overflow); 2: write the first `over` beams to
// the photon's slots i * over + k and count them all.
template <int MODE>
__global__ __launch_bounds__(kPhotonBlock, 6) void k_photons(const DevScene *__restrict__ Sp, int64_t n, uint64_t seq0,
                                                          int max_depth, float radius, int32_t *__restrict__ counts,
                                                          const int64_t *__restrict__ offsets, float *__restrict__ bs,
                                                          float *__restrict__ be, float *__restrict__ br,
                                                          float *__restrict__ bp, int over) {
    const int64_t i = (int64_t)blockIdx.x * kPhotonBlock + threadIdx.x;
    if (i >= n) return;
    if (MODE == 1 && over > 0 && counts[i] <= over) return;
    const DevScene &S = *Sp;
    Pcg rng;
    pcg_seed(rng, seq0 + (uint64_t)i);
    const int64_t w = MODE == 1 ? offsets[i] : (MODE == 2 ? i * (int64_t)over : 0);
    int cnt = 0;

    // ---- emission, photonbeam.cpp:393-418: a light by power, DiffuseAreaLight::Sample_Le ----
    float light_pdf;
    const int ln = sample_light(S, pcg_float(rng), light_pdf);  // lightSample
    float u0x, u0y, u1x, u1y;
    pcg_2d(rng, u0x, u0y);
    pcg_2d(rng, u1x, u1y);
    (void)pcg_float(rng);  // uLightTime
    const PTri &L = S.t[S.light_tri[ln]];
    const ShapeSample ps = sample_tri(L, u0x, u0y);
    const float pdf_pos = ps.pdf;
    const f3 wl = cosine_hemisphere(u1x, u1y);
    const float pdf_dir = wl.z * kInvPi;
    f3 v1, v2;
    coord_system(ps.n, v1, v2);
    f3 d = add3(add3(scale3(v1, wl.x), scale3(v2, wl.y)), scale3(ps.n, wl.z));
    f3 o = offset_origin(ps.p, ps.perr, ps.n, d);
    const bool front = dot3(ps.n, d) > 0;  // DiffuseAreaLight::L, one-sided
    float beta[3];
    bool alive = !(pdf_pos == 0 || pdf_dir == 0 || !front || black3(L.Le));
    if (alive) {
        const float ad = fabsf(dot3(ps.n, d));
        const float den = light_pdf * pdf_pos * pdf_dir;
        for (int c = 0; c < 3; ++c) beta[c] = (ad * L.Le[c]) / den;
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
                    f.tri = hit.tri;
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
            if (MODE == 1 || (MODE == 2 && cnt < over)) {
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
            const PTri &q = S.t[hit.tri];
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
        hit.tri = f.tri;
        depth = f.depth;
        for (int c = 0; c < 3; ++c) beta[c] = f.beta[c];
        resume = true;
    }
    if (MODE != 1) counts[i] = cnt;
}

// The single-trace form's copy: photon i's first min(count, cap) beams from its slots to its offsets.
// Each wave copies the beams of its 64 photons as one run: lane j takes the wave's j-th beam (owner by
// a search of the wave's prefix sums in LDS), so the writes of consecutive lanes are consecutive and a
// photon's slots are read together (a thread per photon strided its reads by cap slots: 0.27 ms at C2).
constexpr int kSlotsBlock = 64;
__global__ __launch_bounds__(kSlotsBlock) void k_photon_slots(int64_t n, int cap, const int32_t *__restrict__ counts,
                                                      const int64_t *__restrict__ offsets, const float *__restrict__ ss,
                                                      const float *__restrict__ se, const float *__restrict__ sr,
                                                      const float *__restrict__ sp, float *__restrict__ bs,
                                                      float *__restrict__ be, float *__restrict__ br,
                                                      float *__restrict__ bp) {
    __shared__ int pre[kSlotsBlock / 64][65];      // per wave: exclusive prefix sums of the photons' copied beams
    __shared__ int64_t off[kSlotsBlock / 64][64];  // per wave: the photons' output offsets
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * kSlotsBlock + threadIdx.x;
    const int64_t i0 = i - lane;
    const int m = i < n ? min(counts[i], cap) : 0;
    int incl = m;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    pre[w][lane + 1] = incl;
    if (lane == 0) pre[w][0] = 0;
    off[w][lane] = i < n ? offsets[i] : 0;
    __builtin_amdgcn_wave_barrier();
    const int total = __shfl(incl, 63);
    for (int j = lane; j < total; j += 64) {
        int lo = 0, hi = 64;  // the photon p with pre[p] <= j < pre[p + 1]
#pragma unroll
        for (int it = 0; it < 6; ++it) {
            const int mid = (lo + hi) >> 1;
            if (pre[w][mid] <= j) lo = mid;
            else hi = mid;
        }
        const int k = j - pre[w][lo];
        const int64_t a = (i0 + lo) * (int64_t)cap + k, b = off[w][lo] + k;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            bs[3 * b + c] = ss[3 * a + c];
            be[3 * b + c] = se[3 * a + c];
            bp[3 * b + c] = sp[3 * a + c];
        }
        br[b] = sr[a];
    }
}

inline unsigned grid_of(int64_t n) { return (unsigned)((n + kPhotonBlock - 1) / kPhotonBlock); }

}  // namespace

hipError_t launch_photons(const DevScene *scene, int stack_depth, int64_t n, uint64_t seq0, int max_depth,
                          float radius, int32_t *counts, const int64_t *offsets, float *start, float *end,
                          float *rad, float *power, int mode, int over, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t lds = scene_stack_bytes(stack_depth, kPhotonBlock);
    if (mode == 1)
        hipLaunchKernelGGL(k_photons<1>, dim3(grid_of(n)), dim3(kPhotonBlock), lds, s, scene, n, seq0, max_depth,
                           radius, counts, offsets, start, end, rad, power, over);
    else if (mode == 2)
        hipLaunchKernelGGL(k_photons<2>, dim3(grid_of(n)), dim3(kPhotonBlock), lds, s, scene, n, seq0, max_depth,
                           radius, counts, offsets, start, end, rad, power, over);
    else
        hipLaunchKernelGGL(k_photons<0>, dim3(grid_of(n)), dim3(kPhotonBlock), lds, s, scene, n, seq0, max_depth,
                           radius, counts, offsets, start, end, rad, power, 0);
    return hipGetLastError();
}

hipError_t launch_photon_slots(int64_t n, int cap, const int32_t *counts, const int64_t *offsets, const float *ss,
                               const float *se, const float *sr, const float *sp, float *start, float *end,
                               float *rad, float *power, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_photon_slots, dim3((unsigned int)((n + kSlotsBlock - 1) / kSlotsBlock)), dim3(kSlotsBlock), 0, s, n, cap, counts, offsets,
                       ss, se, sr, sp, start, end, rad, power);
    return hipGetLastError();
}

size_t count_scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int64_t *)nullptr, (size_t)n,
                                  rocprim::plus<int64_t>());
    return std::max(bytes, slot_scan_temp_bytes(n));
}

// offsets[0] = 0, offsets[k + 1] = counts[0] + ... + counts[k].  slot: the one-wave scan (bre_slot.hip)
hipError_t launch_count_scan(void *tmp, size_t bytes, const int32_t *counts, int64_t *offsets, int64_t n,
                             hipStream_t s, bool slot) {
    if (slot) return slot_exclusive_scan(counts, offsets, n, offsets + n, tmp, s);
    hipError_t e = hipMemsetAsync(offsets, 0, sizeof(int64_t), s);
    if (e != hipSuccess || n == 0) return e;
    return rocprim::inclusive_scan(tmp, bytes, counts, offsets + 1, (size_t)n, rocprim::plus<int64_t>(), s);
}

}  // namespace bre
