// bre_trace.h — scene evaluation for the on-device photon and camera passes (host + device).
//
// Float arithmetic follows the reference's operation order (see the file:line next to each
// function) and is compiled without FMA contraction, with correctly rounded division and sqrt,
// and with the transcendentals of include/bre_fmath.h, so a photon path on the GPU takes the
// same random decisions and produces the same beam bits as the CPU restatement in oracle/.
#pragma once

#include "../../include/bre_fmath.h"
#include "../../include/bre_scene.h"
#include "bre_math.h"

#include <vector>

namespace bre {

#define BRE_TD __host__ __device__ __forceinline__

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInv4Pi = 0.07957747154594766788f;
constexpr float kPiOver2 = 1.57079632679489661923f;
constexpr float kPiOver4 = 0.78539816339744830961f;
constexpr float kOneMinusEps = 0x1.fffffep-1f;
constexpr float kMaxFloat = 3.402823466e+38f;

// gamma(n) of pbrt.h:263-265 in float
BRE_TD float gamma_n(int n) {
    const float eps = 0x1p-24f;
    return (n * eps) / (1 - n * eps);
}

// ---- PCG32 as pbrt seeds and uses it (rng.h:78-85, 129-144) ----
struct Pcg {
    uint64_t state, inc;
};
BRE_TD uint32_t pcg_next(Pcg &r) {
    const uint64_t old = r.state;
    r.state = old * 0x5851f42d4c957f2dULL + r.inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
BRE_TD void pcg_seed(Pcg &r, uint64_t seq) {
    r.state = 0u;
    r.inc = (seq << 1u) | 1u;
    (void)pcg_next(r);
    r.state += 0x853c49e6748fea9bULL;
    (void)pcg_next(r);
}
BRE_TD float pcg_float(Pcg &r) {
    return smin(kOneMinusEps, (float)pcg_next(r) * 0x1p-32f);  // std::min(OneMinusEpsilon, .)
}
// Get2D of the reference's samplers: Point2f(Get1D(), Get1D()) built by g++ right to left
// (photonbeam.cpp:207-212, 239-241), so x is the second draw.
BRE_TD void pcg_2d(Pcg &r, float &x, float &y) {
    const float first = pcg_float(r);
    const float second = pcg_float(r);
    x = second;
    y = first;
}

// ---- vector helpers (geometry.h) ----
BRE_TD f3 neg3(f3 a) { return mk(-a.x, -a.y, -a.z); }
BRE_TD f3 abs3(f3 a) { return mk(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
BRE_TD f3 normalize3(f3 v) { return div3(v, len3(v)); }
BRE_TD f3 ray_at(f3 o, f3 d, float t) { return add3(o, scale3(d, t)); }
// CoordinateSystem, geometry.h:1020-1027
BRE_TD void coord_system(f3 v1, f3 &v2, f3 &v3) {
    if (fabsf(v1.x) > fabsf(v1.y))
        v2 = div3(mk(-v1.z, 0, v1.x), sqrtf(v1.x * v1.x + v1.z * v1.z));
    else
        v2 = div3(mk(0, v1.z, -v1.y), sqrtf(v1.y * v1.y + v1.z * v1.z));
    v3 = cross3d(v1, v2);
}
BRE_TD float next_up(float v) {
    if (v == __builtin_huge_valf()) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = bre_f2u(v);
    if (v >= 0) ++ui;
    else --ui;
    return bre_u2f(ui);
}
BRE_TD float next_down(float v) {
    if (v == -__builtin_huge_valf()) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = bre_f2u(v);
    if (v > 0) --ui;
    else ++ui;
    return bre_u2f(ui);
}
// OffsetRayOrigin, geometry.h:1438-1458
BRE_TD f3 offset_origin(f3 p, f3 perr, f3 n, f3 w) {
    const float d = dot3(abs3(n), perr);
    f3 off = scale3(n, d);
    if (dot3(w, n) < 0) off = neg3(off);
    f3 po = add3(p, off);
    po.x = off.x > 0 ? next_up(po.x) : (off.x < 0 ? next_down(po.x) : po.x);
    po.y = off.y > 0 ? next_up(po.y) : (off.y < 0 ? next_down(po.y) : po.y);
    po.z = off.z > 0 ? next_up(po.z) : (off.z < 0 ? next_down(po.z) : po.z);
    return po;
}

// ---- sampling (sampling.cpp:113-133, sampling.h:159-165) ----
BRE_TD f3 cosine_hemisphere(float ux, float uy) {
    const float ox = 2.f * ux - 1, oy = 2.f * uy - 1;
    float dx = 0, dy = 0;
    if (!(ox == 0 && oy == 0)) {
        float theta, r;
        if (fabsf(ox) > fabsf(oy)) {
            r = ox;
            theta = kPiOver4 * (oy / ox);
        } else {
            r = oy;
            theta = kPiOver2 - kPiOver4 * (ox / oy);
        }
        float s, c;
        bre_sincosf(theta, &s, &c);
        dx = c * r;
        dy = s * r;
    }
    return mk(dx, dy, sqrtf(smax(0.f, 1 - dx * dx - dy * dy)));
}

// ---- Henyey-Greenstein Sample_p (medium.cpp:194-213); the returned pdf is unused here ----
BRE_TD f3 hg_sample(float g, f3 wo, float u0, float u1) {
    float cos_t;
    if ((double)fabsf(g) < 1e-3) {  // std::abs(g) < 1e-3 compares in double
        cos_t = 1 - 2 * u0;
    } else {
        const float sq = (1 - g * g) / (1 - g + 2 * g * u0);
        cos_t = (1 + g * g - sq * sq) / (2 * g);
    }
    const float sin_t = sqrtf(smax(0.f, 1 - cos_t * cos_t));
    const float phi = 2 * kPi * u1;
    f3 v1, v2;
    coord_system(wo, v1, v2);
    float sp, cp;
    bre_sincosf(phi, &sp, &cp);
    // SphericalDirection(sinT, cosT, phi, v1, v2, -wo), geometry.h:1465-1470
    return add3(add3(scale3(v1, sin_t * cp), scale3(v2, sin_t * sp)), scale3(neg3(wo), cos_t));
}

// ---- scene on the device: pbrt Triangles (include/bre_scene.h) ----
struct PTri {
    f3 p0, p1, p2;
    f3 n;        // Triangle::Intersect's normal: normalize(cross(p0 - p2, p1 - p2)), negated if flip
    f3 ss, ts;   // BSDF frame: ss = normalize(dpdu), ts = cross(ns, ss)
    f3 ns;       // Triangle::Sample's normal: normalize(cross(p1 - p0, p2 - p0)), negated if flip
    float kd[3], Le[3];
    float area;  // 0.5 * |cross(p1 - p0, p2 - p0)|
    int absorb;  // kd all zero: no BxDF
    int emit;    // a DiffuseAreaLight
};

// One node of the scene's bounding volume hierarchy: the reference's BVHAccel LinearBVHNode
// (src/accelerators/bvh.cpp, 32 B, depth-first order: an interior node's first child follows it).
struct SceneNode {
    float lo[3], hi[3];  // Bounds3f
    int32_t offset;      // leaf: primitivesOffset; interior: secondChildOffset
    uint16_t nprims;     // 0 for an interior node
    uint8_t axis;        // interior: split axis
    uint8_t pad;
};
static_assert(sizeof(SceneNode) == 32, "SceneNode is BVHAccel's 32-B LinearBVHNode");
constexpr int kSceneStack = 64;  // BVHAccel::Intersect's nodesToVisit[64]: the deepest tree accepted

struct DevScene {
    int n_tris, n_lights, medium, n_nodes;  // medium: BRE_MEDIUM_NONE / _HOMOGENEOUS / _GRID
    int stack_depth;                        // traversal stack entries per thread (the tree depth)
    float sigma_t[3];
    float g;
    // the triangles in scene order, the BVHAccel over them (nodes + primitive order) and
    // scene.lights (the emitting triangles, in order) with the Distribution1D of their Power().y()
    // (ComputeLightPowerDistribution, integrator.cpp:217-225; sampling.h:55-69): device arrays
    const PTri *t;
    const SceneNode *nodes;
    const int32_t *prims;       // BVH primitive slot -> triangle index
    const int32_t *light_tri;
    const float *light_func;
    const float *light_cdf;     // n_lights + 1
    float light_func_int;
    // GridDensityMedium (grid.h:50-80): sigma_t = (sigma_a + sigma_s)[0], invMaxDensity
    int gn[3];
    float grid_sigma_t, grid_inv_max;
    float w2m[16];            // WorldToMedium, row-major
    const float *density;     // device copy of the grid (nx*ny*nz)
};

// Host side of the scene: everything prepare_scene derives, in host memory; the context uploads
// the arrays and points the DevScene at them.
struct HostScene {
    DevScene head;  // scalars; the array pointers are filled after the upload
    std::vector<PTri> tris;
    std::vector<SceneNode> nodes;
    std::vector<int32_t> prims;
    std::vector<int32_t> light_tri;
    std::vector<float> light_func, light_cdf;
    int depth = 0;  // deepest node of the BVH (root = 1)
};

// host: derive the per-triangle constants, the light distribution and the scene BVH exactly as
// oracle/ora_pbrt.h make_scene does; `d_density` is the device copy of s->grid_density (grid media)
void prepare_scene(const bre_scene *s, HostScene *out, const float *d_density = nullptr);
// the two halves of prepare_scene: the triangles, lights and BVH (out->head's geometry fields and
// the arrays), and the medium fields of a DevScene
void prepare_geometry(const bre_scene *s, HostScene *out);
void prepare_medium(const bre_scene *s, DevScene *d, const float *d_density);
// host: the scene's BVHAccel (bvh.cpp: SAH, 12 buckets, maxPrimsInNode 4, depth-first layout) over
// the triangles' world bounds; returns the tree depth
int build_scene_bvh(const std::vector<PTri> &tris, std::vector<SceneNode> *nodes, std::vector<int32_t> *prims);
// the scene's triangle array: the inline one or triangles_ext (bre_scene.h)
inline const bre_triangle *scene_triangles(const bre_scene *s) { return s->triangles_ext ? s->triangles_ext : s->triangles; }
// host: GridDensityMedium ctor's maxDensity loop (grid.h:73-76), std::max order
float grid_max_density(const bre_scene *s);

struct Hit {
    f3 p, perr;
    int tri;
};

BRE_TD int max_dim(f3 v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
BRE_TD float comp(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
BRE_TD f3 permute3(f3 v, int x, int y, int z) { return mk(comp(v, x), comp(v, y), comp(v, z)); }
BRE_TD float max_comp(f3 v) { return smax(v.x, smax(v.y, v.z)); }

// Triangle::Intersect, triangle.cpp:177-300: the watertight test (translate to the ray origin,
// permute so |d| is largest in z, shear, edge functions with a double-precision fallback on zero,
// scaled t against tMax, conservative t > deltaT), then the barycentric hit point and its error bound
__device__ __forceinline__ bool intersect_tri(const PTri &T, f3 o, f3 dir, float tmax, float &t, Hit &h) {
    f3 p0t = sub3(T.p0, o), p1t = sub3(T.p1, o), p2t = sub3(T.p2, o);
    const int kz = max_dim(abs3(dir));
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    const f3 d = permute3(dir, kx, ky, kz);
    p0t = permute3(p0t, kx, ky, kz);
    p1t = permute3(p1t, kx, ky, kz);
    p2t = permute3(p2t, kx, ky, kz);
    const float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1.f / d.z;
    p0t.x += Sx * p0t.z;
    p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z;
    p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z;
    p2t.y += Sy * p2t.z;
    float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        e0 = (float)((double)p2t.y * (double)p1t.x - (double)p2t.x * (double)p1t.y);
        e1 = (float)((double)p0t.y * (double)p2t.x - (double)p0t.x * (double)p2t.y);
        e2 = (float)((double)p1t.y * (double)p0t.x - (double)p1t.x * (double)p0t.y);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    const float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz;
    p1t.z *= Sz;
    p2t.z *= Sz;
    const float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < tmax * det)) return false;
    if (det > 0 && (tScaled <= 0 || tScaled > tmax * det)) return false;
    const float invDet = 1 / det;
    const float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    t = tScaled * invDet;
    const float maxZt = max_comp(abs3(mk(p0t.z, p1t.z, p2t.z)));
    const float deltaZ = gamma_n(3) * maxZt;
    const float maxXt = max_comp(abs3(mk(p0t.x, p1t.x, p2t.x)));
    const float maxYt = max_comp(abs3(mk(p0t.y, p1t.y, p2t.y)));
    const float deltaX = gamma_n(5) * (maxXt + maxZt);
    const float deltaY = gamma_n(5) * (maxYt + maxZt);
    const float deltaE = 2 * (gamma_n(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    const float maxE = max_comp(abs3(mk(e0, e1, e2)));
    const float deltaT = 3 * (gamma_n(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    if (t <= deltaT) return false;
    const float xs = fabsf(b0 * T.p0.x) + fabsf(b1 * T.p1.x) + fabsf(b2 * T.p2.x);
    const float ys = fabsf(b0 * T.p0.y) + fabsf(b1 * T.p1.y) + fabsf(b2 * T.p2.y);
    const float zs = fabsf(b0 * T.p0.z) + fabsf(b1 * T.p1.z) + fabsf(b2 * T.p2.z);
    h.perr = scale3(mk(xs, ys, zs), gamma_n(7));
    h.p = add3(add3(scale3(T.p0, b0), scale3(T.p1, b1)), scale3(T.p2, b2));
    return true;
}

// Scene::Intersect = BVHAccel::Intersect (bvh.cpp): depth-first through the scene BVH, near child
// first by dirIsNeg[axis], every node tested with the reference's slab test against the CURRENT
// tMax, every leaf triangle with Triangle::Intersect, each hit shrinking tMax (primitive.cpp:97-101).
// The triangles are tested in the reference's order, so among equal-t hits the same one wins.  The
// stack lives in the kernel's dynamic LDS (entry k of thread t at [k * blockDim.x + t]), sized by
// the launch to the tree's depth (scene_stack_bytes): it holds at most one entry per level of the
// current path.  The host rejects trees deeper than kSceneStack (upload_scene).
__device__ __forceinline__ bool intersect_scene(const DevScene &S, f3 o, f3 d, float &tmax, Hit &h) {
    extern __shared__ int bre_scene_stack[];
    int *stack = bre_scene_stack + threadIdx.x;
    const int stride = blockDim.x;
    const f3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
    const int n0 = inv.x < 0, n1 = inv.y < 0, n2 = inv.z < 0;
    int sp = 0, cur = 0;
    bool hit = false;
    while (true) {
        const SceneNode &nd = S.nodes[cur];
        const Box6 b{nd.lo[0], nd.lo[1], nd.lo[2], nd.hi[0], nd.hi[1], nd.hi[2]};
        if (slab_test(b, o, inv, n0, n1, n2, tmax, nullptr)) {
            if (nd.nprims > 0) {
                for (int i = 0; i < nd.nprims; ++i) {
                    const int ti = S.prims[nd.offset + i];
                    float t;
                    Hit tmp;
                    if (!intersect_tri(S.t[ti], o, d, tmax, t, tmp)) continue;
                    tmax = t;
                    h.p = tmp.p;
                    h.perr = tmp.perr;
                    h.tri = ti;
                    hit = true;
                }
                if (sp == 0) break;
                cur = stack[--sp * stride];
            } else {
                const int neg = nd.axis == 0 ? n0 : (nd.axis == 1 ? n1 : n2);
                stack[sp++ * stride] = neg ? cur + 1 : nd.offset;
                cur = neg ? nd.offset : cur + 1;
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp * stride];
        }
    }
    return hit;
}

// Triangle::Sample(u, pdf), triangle.cpp:543-568, with UniformSampleTriangle
struct ShapeSample {
    f3 p, perr, n;
    float pdf;
};
BRE_TD ShapeSample sample_tri(const PTri &T, float u0, float u1) {
    ShapeSample r;
    const float su0 = sqrtf(u0);
    const float b0 = 1 - su0, b1 = u1 * su0;
    const float b2 = 1 - b0 - b1;
    const f3 a = scale3(T.p0, b0), b = scale3(T.p1, b1), c = scale3(T.p2, b2);
    r.p = add3(add3(a, b), c);
    r.n = T.ns;
    r.perr = scale3(add3(add3(abs3(a), abs3(b)), abs3(c)), gamma_n(6));
    r.pdf = 1 / T.area;
    return r;
}

// FindInterval, pbrt.h:377-389: bisection for the last index with pred true, then
// Clamp(first - 1, 0, size - 2) (pbrt.h:278-284: the low bound is tested first)
template <typename Pred>
BRE_TD int find_interval(int size, const Pred &pred) {
    int first = 0, len = size;
    while (len > 0) {
        const int half = len >> 1, middle = first + half;
        if (pred(middle)) {
            first = middle + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    const int v = first - 1;
    return v < 0 ? 0 : (v > size - 2 ? size - 2 : v);
}

// Distribution1D::SampleDiscrete with FindInterval (sampling.h:90-100, pbrt.h:377-389) over the
// light powers; returns the light index (into light_tri)
BRE_TD int sample_light(const DevScene &S, float u, float &pdf) {
    const float *cdf = S.light_cdf;
    const int off = find_interval(S.n_lights + 1, [&](int i) { return cdf[i] <= u; });
    pdf = (S.light_func_int > 0) ? S.light_func[off] / (S.light_func_int * (float)S.n_lights) : 0.f;
    return off;
}

// Sampler draws: the photon pass draws from PCG32 (AwesomeHaltonSampler past its 1000 Halton
// dimensions); the camera pass overloads smp_1d for its AwesomeSampler (bre_camera.hip).
__device__ __forceinline__ float smp_1d(Pcg &r) { return pcg_float(r); }

// HomogeneousMedium::Tr, homogeneous.cpp:44-48
__device__ __forceinline__ void medium_tr(const DevScene &S, f3 d, float tmax, float tr[3]) {
    const float x = smin(tmax * len3(d), kMaxFloat);
    // one expf per distinct argument (a grey medium's three channels share theirs: the same values)
    const float a0 = -S.sigma_t[0] * x, a1 = -S.sigma_t[1] * x, a2 = -S.sigma_t[2] * x;
    tr[0] = bre_expf(a0);
    tr[1] = a1 == a0 ? tr[0] : bre_expf(a1);
    tr[2] = a2 == a1 ? tr[1] : bre_expf(a2);
}

// HomogeneousMedium::Sample distance part, homogeneous.cpp:50-60 (two draws)
template <class Smp>
__device__ __forceinline__ bool medium_sample(const DevScene &S, Smp &rng, f3 d, float tmax, float &t) {
    int ch = (int)(smp_1d(rng) * 3);
    ch = (2 < ch) ? 2 : ch;  // std::min(ch, 2)
    const float st = ch == 0 ? S.sigma_t[0] : (ch == 1 ? S.sigma_t[1] : S.sigma_t[2]);
    const float dist = -bre_logf(1 - smp_1d(rng)) / st;
    t = smin(dist * len3(d), tmax);
    return t < tmax;
}

// ---- GridDensityMedium (src/media/grid.{h,cpp}) ----
BRE_TD float lerp_ref(float t, float v1, float v2) { return (1 - t) * v1 + t * v2; }  // pbrt.h:391

// GridDensityMedium::D, grid.h:84-88 (0 outside [0, n) per axis)
__device__ __forceinline__ float grid_D(const DevScene &S, int x, int y, int z) {
    if (!(x >= 0 && x < S.gn[0] && y >= 0 && y < S.gn[1] && z >= 0 && z < S.gn[2])) return 0.f;
    return S.density[((int64_t)z * S.gn[1] + y) * S.gn[0] + x];
}

// GridDensityMedium::Density, grid.cpp:46-60: trilinear over the sample lattice at cell centres
__device__ __forceinline__ float grid_density(const DevScene &S, f3 p) {
    const float sx = p.x * (float)S.gn[0] - .5f, sy = p.y * (float)S.gn[1] - .5f, sz = p.z * (float)S.gn[2] - .5f;
    const int ix = (int)floorf(sx), iy = (int)floorf(sy), iz = (int)floorf(sz);
    const float dx = sx - (float)ix, dy = sy - (float)iy, dz = sz - (float)iz;
    const float d00 = lerp_ref(dx, grid_D(S, ix, iy, iz), grid_D(S, ix + 1, iy, iz));
    const float d10 = lerp_ref(dx, grid_D(S, ix, iy + 1, iz), grid_D(S, ix + 1, iy + 1, iz));
    const float d01 = lerp_ref(dx, grid_D(S, ix, iy, iz + 1), grid_D(S, ix + 1, iy, iz + 1));
    const float d11 = lerp_ref(dx, grid_D(S, ix, iy + 1, iz + 1), grid_D(S, ix + 1, iy + 1, iz + 1));
    const float d0 = lerp_ref(dy, d00, d10);
    const float d1 = lerp_ref(dy, d01, d11);
    return lerp_ref(dz, d0, d1);
}

// WorldToMedium(Ray(o, Normalize(d), tMax * |d|)) (grid.cpp:66-67) through
// Transform::operator()(Ray) (transform.h:251-264, point with error bound :278-299, vector :236-242),
// then Bounds3f(0, 1)::IntersectP(ray, &t0, &t1) (geometry.h:1386-1408).  Returns false on a miss.
__device__ __forceinline__ bool grid_ray(const DevScene &S, f3 o, f3 d, float tmax, f3 &mo, f3 &md, float &t0,
                                         float &t1) {
    const f3 dn = normalize3(d);
    const float tm = tmax * len3(d);
    const float *m = S.w2m;
    const float xp = m[0] * o.x + m[1] * o.y + m[2] * o.z + m[3];
    const float yp = m[4] * o.x + m[5] * o.y + m[6] * o.z + m[7];
    const float zp = m[8] * o.x + m[9] * o.y + m[10] * o.z + m[11];
    const float wp = m[12] * o.x + m[13] * o.y + m[14] * o.z + m[15];
    const float xs = fabsf(m[0] * o.x) + fabsf(m[1] * o.y) + fabsf(m[2] * o.z) + fabsf(m[3]);
    const float ys = fabsf(m[4] * o.x) + fabsf(m[5] * o.y) + fabsf(m[6] * o.z) + fabsf(m[7]);
    const float zs = fabsf(m[8] * o.x) + fabsf(m[9] * o.y) + fabsf(m[10] * o.z) + fabsf(m[11]);
    const float g3 = gamma_n(3);
    const f3 oerr = mk(g3 * xs, g3 * ys, g3 * zs);
    f3 po = mk(xp, yp, zp);
    if (!(wp == 1)) {
        const float inv = (float)1 / wp;
        po = mk(inv * xp, inv * yp, inv * zp);
    }
    const f3 dv = mk(m[0] * dn.x + m[1] * dn.y + m[2] * dn.z, m[4] * dn.x + m[5] * dn.y + m[6] * dn.z,
                     m[8] * dn.x + m[9] * dn.y + m[10] * dn.z);
    float rt = tm;
    const float l2 = lensq3(dv);
    if (l2 > 0) {
        const float dt = dot3(abs3(dv), oerr) / l2;
        po = add3(po, scale3(dv, dt));
        rt -= dt;
    }
    mo = po;
    md = dv;
    float a = 0, b = rt;
    const float pad = 1 + 2 * gamma_n(3);
    const float oo[3] = {po.x, po.y, po.z}, dd[3] = {dv.x, dv.y, dv.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float inv = 1 / dd[i];
        float tn = (0.f - oo[i]) * inv;
        float tf = (1.f - oo[i]) * inv;
        if (tn > tf) {
            const float x = tn;
            tn = tf;
            tf = x;
        }
        tf *= pad;
        a = tn > a ? tn : a;
        b = tf < b ? tf : b;
        if (a > b) return false;
    }
    t0 = a;
    t1 = b;
    return true;
}

// GridDensityMedium::Sample, grid.cpp:62-89: delta tracking.  On an interaction, t is the
// medium-space distance and the interaction point is rWorld(t) = o + d*t (as the reference).
template <class Smp>
__device__ __forceinline__ bool grid_sample(const DevScene &S, Smp &smp, f3 o, f3 d, float tmax, float &t_out) {
    f3 mo, md;
    float tmin, tm;
    if (!grid_ray(S, o, d, tmax, mo, md, tmin, tm)) return false;
    float t = tmin;
    while (true) {
        t -= bre_logf(1 - smp_1d(smp)) * S.grid_inv_max / S.grid_sigma_t;
        if (t >= tm) break;
        if (grid_density(S, ray_at(mo, md, t)) * S.grid_inv_max > smp_1d(smp)) {
            t_out = t;
            return true;
        }
    }
    return false;
}

// GridDensityMedium::Tr, grid.cpp:91-118: ratio tracking with Russian roulette below 0.1
template <class Smp>
__device__ __forceinline__ float grid_tr(const DevScene &S, Smp &smp, f3 o, f3 d, float tmax) {
    f3 mo, md;
    float tmin, tm;
    if (!grid_ray(S, o, d, tmax, mo, md, tmin, tm)) return 1.f;
    float tr = 1, t = tmin;
    while (true) {
        t -= bre_logf(1 - smp_1d(smp)) * S.grid_inv_max / S.grid_sigma_t;
        if (t >= tm) break;
        const float density = grid_density(S, ray_at(mo, md, t));
        tr *= 1 - smax(0.f, density * S.grid_inv_max);
        const float rr = 0.1f;
        if (tr < rr) {
            const float q = smax(0.05f, 1 - tr);
            if (smp_1d(smp) < q) return 0.f;
            tr /= 1 - q;
        }
    }
    return tr;
}

// Medium::Tr of the world ray (o, d, tmax) for either medium type
template <class Smp>
__device__ __forceinline__ void medium_tr_any(const DevScene &S, Smp &smp, f3 o, f3 d, float tmax, float tr[3]) {
    if (S.medium == BRE_MEDIUM_GRID) {
        const float t = grid_tr(S, smp, o, d, tmax);
        tr[0] = tr[1] = tr[2] = t;
    } else {
        medium_tr(S, d, tmax, tr);
    }
}

// Medium::Sample distance decision; on true the interaction point is o + d*t
template <class Smp>
__device__ __forceinline__ bool medium_sample_any(const DevScene &S, Smp &smp, f3 o, f3 d, float tmax, float &t) {
    if (S.medium == BRE_MEDIUM_GRID) return grid_sample(S, smp, o, d, tmax, t);
    return medium_sample(S, smp, d, tmax, t);
}

BRE_TD bool black3(const float v[3]) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }
BRE_TD float lum3(const float v[3]) { return 0.212671f * v[0] + 0.715160f * v[1] + 0.072169f * v[2]; }

// ---- camera pass (bre_camera.hip) ----
constexpr int kHaltonDims = 1000;  // HaltonSampler's PrimeTableSize = AwesomeSampler's limit (photonbeam.cpp:460)

struct DevCamera {
    f3 pos, dir, right, nup;           // LookAt frame
    float sx0, sx1, sy0, sy1;          // screen window
    float tan_ang, fw, fh;             // tan(fov/2), film size as float
    int width, height;
    int base_scale[2], base_exp[2];    // HaltonSampler baseScales / baseExponents
    int stride;                        // sampleStride
    int mult_inv[2];                   // multInverse
    int primes[kHaltonDims];
    int prime_sums[kHaltonDims];
};

// per-(depth, pixel-slot) camera segments before compaction
struct CamSlots {
    float *o, *p, *d, *t;
    int32_t *pix, *valid;
};

void prepare_camera(const bre_scene *s, int width, int height, DevCamera *c, std::vector<uint16_t> *perms);
int64_t camera_slots(int width, int height);
hipError_t launch_camera(const DevScene *scene, int stack_depth, const DevCamera *cam, const uint16_t *perms, int width,
                         int height, int iteration, int max_depth, int render_surfaces, int render_media,
                         const CamSlots &s, float *surface, unsigned int *flags, int shard_rank, int shard_count,
                         int shard_block, int classes, hipStream_t stream);
size_t camera_scan_temp_bytes(int64_t n);
hipError_t launch_camera_scan(void *tmp, size_t tmp_bytes, const CamSlots &s, int64_t nslots, int max_depth,
                              int64_t *offs, hipStream_t stream, bool slot);
hipError_t launch_camera_compact(const CamSlots &s, int64_t nslots, int max_depth, const int64_t *offs, float *o,
                                 float *p, float *d, float *t, int32_t *pix, int32_t *depth, hipStream_t stream);

// dynamic LDS of a photon / camera launch: the scene traversal stack of every thread of a block
inline size_t scene_stack_bytes(int stack_depth, int block) {
    return (size_t)(stack_depth > 0 ? stack_depth : 1) * (size_t)block * sizeof(int);
}

// photon pass launchers (bre_photon.hip)
// mode 0: count beams per photon; 1: write them at offsets (over > 0: only photons with more than `over`
// beams); 2: write the first `over` beams to per-photon slots and count them all (single-trace form)
hipError_t launch_photons(const DevScene *scene, int stack_depth, int64_t n, uint64_t seq0, int max_depth,
                          float radius, int32_t *counts, const int64_t *offsets, float *start, float *end,
                          float *rad, float *power, int mode, int over, hipStream_t s);
// the single-trace form's copy of each photon's slots to its offsets
hipError_t launch_photon_slots(int64_t n, int cap, const int32_t *counts, const int64_t *offsets, const float *ss,
                               const float *se, const float *sr, const float *sp, float *start, float *end,
                               float *rad, float *power, hipStream_t s);
size_t count_scan_temp_bytes(int64_t n);
hipError_t launch_count_scan(void *tmp, size_t bytes, const int32_t *counts, int64_t *offsets, int64_t n, hipStream_t s,
                             bool slot);

}  // namespace bre
