// bre_check.hip — device self-check of the scalar primitives the passes and the gather share.
//
// The photon and camera passes step every spawned ray origin with NextFloatUp / NextFloatDown
// (OffsetRayOrigin, geometry.h:1438-1458; pbrt.h:215-239) and choose the emitting light with
// FindInterval (Distribution1D::SampleDiscrete, sampling.h:90-100; pbrt.h:377-389); the gather's
// exact stage takes its square roots and its shared-divisor quotient without the compiler's general
// expansions (bre_math.h sqrt_cr_noscale, div_by_shared).  bre_device_check runs those very device
// functions on caller-supplied inputs so the tests can hold them bit for bit against the reference's
// own primitive tests (src/tests/fp_tests.cpp, find_interval.cpp) and against the compiler's sqrtf
// and division -- a toolchain change to the f32 sqrt lowering then fails a test instead of silently
// moving the exact stage off the reference's rounding.
#include <hip/hip_runtime.h>

#include "bre_device.h"
#include "bre_math.h"
#include "bre_trace.h"

namespace bre {

namespace {

// kind 0: next_up; 1: next_down; 2: sqrt_cr_noscale and sqrtf (two outputs per input);
// 3: find_interval over aux[0, n_aux) with pred aux[i] <= x (the index as a float);
// 4: div_by_shared(x, aux[0], 1 / aux[0]) and x / aux[0] (two outputs per input);
// 9: the passes' expf, logf, sinf and cosf (include/bre_fmath.h; four outputs per input)
__global__ __launch_bounds__(256) void k_check(int kind, int64_t n, const float *__restrict__ x, int n_aux,
                                               const float *__restrict__ aux, float *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    switch (kind) {
    case 0: y[i] = next_up(v); break;
    case 1: y[i] = next_down(v); break;
    case 2:
        y[2 * i] = sqrt_cr_noscale(v);
        y[2 * i + 1] = sqrtf(v);
        break;
    case 3: y[i] = (float)find_interval(n_aux, [&](int k) { return aux[k] <= v; }); break;
    case 9:
        y[4 * i] = bre_expf(v);
        y[4 * i + 1] = bre_logf(v);
        bre_sincosf(v, &y[4 * i + 2], &y[4 * i + 3]);
        break;
    default: {
        const float b = aux[0];
        const float inv = 1.0f / b;
        y[2 * i] = div_by_shared(v, b, inv);
        y[2 * i + 1] = v / b;
    }
    }
}

}  // namespace

// outputs per input: 1 for kinds 0, 1, 3; 2 for kinds 2 and 4; 4 for kind 9
hipError_t launch_device_check(int kind, int64_t n, const float *x, int n_aux, const float *aux, float *y,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_check, dim3((unsigned int)((n + 255) / 256)), dim3(256), 0, s, kind, n, x, n_aux, aux, y);
    return hipGetLastError();
}

}  // namespace bre
