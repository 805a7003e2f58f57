"""libbre's own device copies of the scalar primitives, bit for bit (bre_device_check).

* NextFloatUp / NextFloatDown (bre_trace.h next_up / next_down; every photon and camera bounce steps
  its spawned origin with them, OffsetRayOrigin geometry.h:1438-1458): the reference's
  FloatingPoint.NextUpDownFloat test (src/tests/fp_tests.cpp:29-53) on the device, against numpy's
  nextafter and the oracle, on the same RNG() float stream.
* FindInterval (bre_trace.h find_interval, the light choice of the photon pass): the reference's
  FindInterval.Basics (src/tests/find_interval.cpp:8-28), plus random monotone arrays against the oracle.
* The exact stage's square root (bre_math.h sqrt_cr_noscale: v_sqrt_f32 + the residual correction,
  without the compiler's small-input scaling) is bit-identical to sqrtf for every x >= 2^-96, 0, +inf
  and exact squares (a change of the compiler's f32 sqrt lowering must fail a test).
* The shared-reciprocal division (div_by_shared) equals the correctly rounded quotient for the
  divisors the gather uses (R + r).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(bre):
    with bre.BeamGather(0) as g:
        yield g


def test_device_next_up_down(ctx, oracle):
    inf = np.float32(np.inf)
    up = ctx.device_check(0, np.array([-0.0, inf, -inf], np.float32))
    dn = ctx.device_check(1, np.array([0.0, inf, -inf], np.float32))
    assert up[0] > 0.0 and dn[0] < 0.0
    assert up[1] == inf and dn[1] < inf
    assert dn[2] == -inf and up[2] > -inf
    u = oracle.pcg32_default(200_000)
    f = u.view(np.float32)
    f = f[np.isfinite(f)][:100_000]
    for kind, direction, up_ in ((0, inf, True), (1, -inf, False)):
        got = ctx.device_check(kind, f).view(np.uint32)
        assert np.array_equal(got, np.nextafter(f, direction).view(np.uint32))
        assert np.array_equal(got, oracle.next_float(f, up_).view(np.uint32))


def test_device_find_interval(ctx, oracle):
    a = np.arange(10, dtype=np.float32)
    xs = [-1.0, 100.0] + [v for i in range(9) for v in (i, i + 0.5, i - 0.5)]
    x = np.array(xs, np.float32)
    got = ctx.device_check(3, x, aux=a).astype(np.int32)
    assert got[0] == 0 and got[1] == a.size - 2
    for k, i in enumerate(range(9)):
        assert got[2 + 3 * k] == i and got[3 + 3 * k] == i
        if i > 0:
            assert got[4 + 3 * k] == i - 1
    rng = np.random.default_rng(4)
    for n in (2, 3, 17, 129):
        cdf = np.sort(rng.random(n).astype(np.float32))
        cdf[0] = 0.0
        q = np.concatenate([rng.random(4000).astype(np.float32), cdf, np.array([-1.0, 2.0], np.float32)])
        assert np.array_equal(ctx.device_check(3, q, aux=cdf).astype(np.int32), oracle.find_interval(cdf, q))


def test_device_sqrt_noscale_is_sqrtf(ctx):
    rng = np.random.default_rng(6)
    lo, hi = np.uint32(0x0F800000), np.uint32(0x7F7FFFFF)  # 2^-96 .. FLT_MAX
    u = rng.integers(lo, hi, 2_000_000, dtype=np.uint32, endpoint=True)
    edge = np.array([0x0F800000, 0x0F800001, 0x0F7FFFFF + 1, 0x3F800000, 0x7F7FFFFF], np.uint32)
    sq = (np.arange(1, 4097, dtype=np.float32) * np.float32(0.25)) ** 2  # exact squares
    x = np.concatenate([u.view(np.float32), edge.view(np.float32), sq,
                        np.array([0.0, np.inf], np.float32)]).astype(np.float32)
    y = ctx.device_check(2, x)
    assert np.array_equal(y[:, 0].view(np.uint32), y[:, 1].view(np.uint32))
    # sqrtf itself is the correctly rounded root (numpy's, IEEE)
    assert np.array_equal(y[:, 1].view(np.uint32), np.sqrt(x).view(np.uint32))


@pytest.mark.parametrize("b", [0.02, 0.0101, 0.0150625, 0.0030517578, 1.0])
def test_device_div_by_shared(ctx, b):
    rng = np.random.default_rng(7)
    a = np.concatenate([rng.random(500_000).astype(np.float32) * np.float32(b),
                        np.float32(b) * (1 - rng.random(1000).astype(np.float32) * np.float32(1e-6)),
                        np.array([0.0, np.float32(b)], np.float32)]).astype(np.float32)
    y = ctx.device_check(4, a, aux=np.array([b], np.float32))
    assert np.array_equal(y[:, 0].view(np.uint32), y[:, 1].view(np.uint32))
    assert np.array_equal(y[:, 1].view(np.uint32), (a / np.float32(b)).astype(np.float32).view(np.uint32))
