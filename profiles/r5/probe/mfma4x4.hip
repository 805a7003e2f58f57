// Probe (round 5): operand/result layout of v_mfma_f32_4x4x1_16b_f32 with A broadcast from block 0
// (cbsz 4, abid 0), and whether a K=1 chain of them is bit-identical to the scan's VALU fma chain.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_layout(float *out, int cbsz) {
    const int l = threadIdx.x;
    const float a = 1000.0f * (float)(l + 1);  // A value of lane l
    const float b = (float)(l + 1);            // B value of lane l
    v4f c = {0.f, 0.f, 0.f, 0.f};
    if (cbsz) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 0, 0);
    else c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

// per lane: segment (au, q); per row r: beam r (bu, m0).  VALU: the scan's chains; MFMA: the same order.
__global__ void k_chain(const float *beams, const float *segs, int n, unsigned int *bad, float *ov, float *om) {
    const int l = threadIdx.x;
    const int g = blockIdx.x;  // 4 beams per block
    const float *s = segs + (size_t)(g * 64 + l) * 6;
    const float aux = s[0], auy = s[1], auz = s[2], qx = s[3], qy = s[4], qz = s[5];
    const float *bl = beams + (size_t)(g * 4 + (l & 3)) * 6;  // lane l (l < 4 matters): beam l of the group
    const float bux = bl[0], buy = bl[1], buz = bl[2], mx = bl[3], my = bl[4], mz = bl[5];
    v4f c = {0.f, 0.f, 0.f, 0.f}, t = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(buz, auz, c, 4, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(buy, auy, c, 4, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(bux, aux, c, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(mz, auz, t, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(my, auy, t, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(mx, aux, t, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(buz, -qz, t, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(buy, -qy, t, 4, 0, 0);
    t = __builtin_amdgcn_mfma_f32_4x4x1f32(bux, -qx, t, 4, 0, 0);
    for (int r = 0; r < 4; ++r) {
        const float *b = beams + (size_t)(g * 4 + r) * 6;
        const float cv = __builtin_fmaf(aux, b[0], __builtin_fmaf(auy, b[1], auz * b[2]));
        const float x = __builtin_fmaf(aux, b[3], __builtin_fmaf(auy, b[4], auz * b[5]));
        const float tv = __builtin_fmaf(-b[0], qx, __builtin_fmaf(-b[1], qy, __builtin_fmaf(-b[2], qz, x)));
        const size_t o = ((size_t)g * 64 + l) * 4 + r;
        ov[2 * o] = cv;
        ov[2 * o + 1] = tv;
        om[2 * o] = c[r];
        om[2 * o + 1] = t[r];
        if (__float_as_uint(cv) != __float_as_uint(c[r]) || __float_as_uint(tv) != __float_as_uint(t[r])) atomicAdd(bad, 1u);
    }
}

static unsigned long long rs = 88172645463325252ull;
static float frand() {  // xorshift, uniform [-1, 1)
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (float)((double)(rs >> 11) / (double)(1ull << 53) * 2.0 - 1.0);
}

int main() {
    float *d;
    hipMalloc(&d, 256 * sizeof(float));
    for (int cb = 0; cb < 2; ++cb) {
        k_layout<<<1, 64>>>(d, cb);
        float h[256];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        printf("cbsz=%d:\n", cb ? 4 : 0);
        for (int l = 0; l < 64; l += (l < 8 ? 1 : 9)) {
            printf("  lane %2d:", l);
            for (int r = 0; r < 4; ++r) printf(" %9.0f", h[l * 4 + r]);
            printf("\n");
        }
    }
    const int G = 4096;  // groups of 4 beams
    const int nb = G * 4, ns = G * 64;
    float *hb = (float *)malloc(sizeof(float) * 6 * nb), *hs = (float *)malloc(sizeof(float) * 6 * ns);
    for (int i = 0; i < nb; ++i) {
        float u[3] = {frand(), frand(), frand()};
        float L = sqrtf(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
        float p[3] = {frand() * 2, frand() * 2, frand() * 2};
        for (int k = 0; k < 3; ++k) hb[6 * i + k] = u[k] / L;
        if (i % 97 == 0) hb[6 * i] = 0.f, hb[6 * i + 1] = -0.f;  // zeros of both signs
        hb[6 * i + 3] = hb[6 * i + 1] * p[2] - hb[6 * i + 2] * p[1];
        hb[6 * i + 4] = hb[6 * i + 2] * p[0] - hb[6 * i + 0] * p[2];
        hb[6 * i + 5] = hb[6 * i + 0] * p[1] - hb[6 * i + 1] * p[0];
        if (i % 89 == 0) hb[6 * i + 5] = 1e-39f;  // a denormal
    }
    for (int i = 0; i < ns; ++i) {
        for (int k = 0; k < 6; ++k) hs[6 * i + k] = frand() * (k < 3 ? 1.f : 3.f);
        if (i % 101 == 0) hs[6 * i + 2] = 1e-30f;  // tiny products
    }
    float *db, *dsg, *ov, *om;
    unsigned int *bad;
    hipMalloc(&db, sizeof(float) * 6 * nb);
    hipMalloc(&dsg, sizeof(float) * 6 * ns);
    hipMalloc(&ov, sizeof(float) * 8 * ns);
    hipMalloc(&om, sizeof(float) * 8 * ns);
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    hipMemcpy(db, hb, sizeof(float) * 6 * nb, hipMemcpyHostToDevice);
    hipMemcpy(dsg, hs, sizeof(float) * 6 * ns, hipMemcpyHostToDevice);
    k_chain<<<G, 64>>>(db, dsg, G, bad, ov, om);
    unsigned int hbad = 0;
    hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost);
    float *hv = (float *)malloc(sizeof(float) * 8 * ns), *hm = (float *)malloc(sizeof(float) * 8 * ns);
    hipMemcpy(hv, ov, sizeof(float) * 8 * ns, hipMemcpyDeviceToHost);
    hipMemcpy(hm, om, sizeof(float) * 8 * ns, hipMemcpyDeviceToHost);
    int shown = 0;
    for (size_t i = 0; i < (size_t)8 * ns && shown < 8; ++i)
        if (memcmp(&hv[i], &hm[i], 4) != 0) {
            printf("  diff at %zu: valu %.9g (%08x) mfma %.9g (%08x)\n", i, hv[i], *(unsigned *)&hv[i], hm[i], *(unsigned *)&hm[i]);
            ++shown;
        }
    printf("chain check: %d groups x 4 beams x 64 lanes, %u (lane, beam) values differ from the VALU fma chain\n", G, hbad);
    return hbad != 0;
}
