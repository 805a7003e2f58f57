"""Known-answer tests for the oracle, each derived by hand from the cited reference lines.

The reference's own tests hold no case for this path, so these KATs and the
independent Python restatement (test_oracle_crosscheck.py) are what pin the oracle."""
import math

import numpy as np
import pytest

f32 = np.float32


def one_beam(start, end, radius, power=(1.0, 2.0, 4.0)):
    return {"start": np.array([start], f32), "end": np.array([end], f32), "radius": np.array([radius], f32),
            "power": np.array([power], f32)}


def seg(o, p):
    o, p = np.array(o, np.float64), np.array(p, np.float64)
    d = (p - o) / np.linalg.norm(p - o)
    tmax = np.linalg.norm(p - o)
    return {"o": np.array([o], f32), "p": np.array([p], f32), "d": np.array([d], f32),
            "tmax": np.array([tmax], f32)}


def gather1(oracle, beams, segs, R):
    out = oracle.build(beams).gather(segs, R)
    bf = oracle.bruteforce(beams, segs, R)
    assert np.array_equal(out["cand"], bf["cand"])
    assert np.array_equal(out["seg_rgb"], bf["seg_rgb"])  # one beam: no summation-order freedom
    return out


def test_slab_pad_is_1_plus_3ulp(oracle):
    # gamma(3) = 3e/(1-3e), e = 2^-24 (pbrt.h:175,263); 1 + 2*gamma(3) rounds to 1 + 3*2^-23
    assert oracle.slab_pad() == np.float32(1 + 3 * 2.0**-23)


def test_radius_schedule(oracle):
    # R_{i+1} = R_i (i + alpha)/(i + 1)   photonbeam.cpp:354-356, 562
    assert oracle.radius_at(1.0, 0.5, 0) == 1.0
    assert oracle.radius_at(1.0, 0.5, 1) == np.float32(0.5)
    assert oracle.radius_at(1.0, 0.5, 2) == np.float32(np.float32(0.5) * np.float32(1.5 / 2.0))
    r = np.float32(0.01)
    for i in range(9):
        r = np.float32(r * np.float32(np.float32(i + 0.5) / np.float32(i + 1)))
    assert oracle.radius_at(0.01, 0.5, 9) == r


def test_perpendicular_beam_kernel_value(oracle):
    """Segment along +x through the origin region, beam along +z offset by h in y (h < r so the
    box is hit): closest distance h, contribution 1e-5 * P * sqrt(1 - (h/(R+r))^2)."""
    R, r, h = 0.05, 0.05, 0.03
    beams = one_beam((0.5, h, -0.5), (0.5, h, 0.5), r)
    # tilt the ray slightly so no direction component is zero
    segs = seg((0.0, 0.0, 1e-3), (1.0, 0.0, -1e-3))
    out = gather1(oracle, beams, segs, R)
    assert out["cand"][0] == 1 and out["contrib"][0] == 1
    expect = 1e-5 * np.array([1, 2, 4]) * math.sqrt(1 - (h / (R + r)) ** 2)
    np.testing.assert_allclose(out["seg_rgb"][0], expect, rtol=2e-6)


def test_box_miss_gives_zero_even_within_kernel_radius(oracle):
    """r < h < R + r: inside the kernel support, but the beam's box (half-width r around the
    beam in y) is missed, so the reference never considers the beam (photonbeambvh.h:60-72)."""
    R, r, h = 0.05, 0.02, 0.04
    beams = one_beam((0.5, h, -0.5), (0.5, h, 0.5), r)
    segs = seg((0.0, 0.0, 1e-3), (1.0, 0.0, -1e-3))
    out = gather1(oracle, beams, segs, R)
    assert out["cand"][0] == 0 and out["contrib"][0] == 0 and not out["seg_rgb"].any()


def test_negative_direction_box_shrinks(oracle):
    """size_i = dir_i*len + 2r*sqrt(1-dir_i^2) uses the SIGNED dir_i, so along a negative component
    the box is |dir_i|*len - 2r*sqrt(1-dir_i^2) wide: narrower than the beam's own extent."""
    r = 0.05
    start, end = (0.8, 0.5, 0.2), (0.2, 0.5, 1.0)  # dir = (-0.6, 0, 0.8), len = 1
    box = oracle.beam_bounds(np.array([start]), np.array([end]), np.array([r]))[0]
    width_x = box[3] - box[0]
    assert width_x == pytest.approx(0.6 - 2 * r * 0.8, abs=1e-6)
    # mirrored beam (+x): box grows instead
    box2 = oracle.beam_bounds(np.array([(0.2, 0.5, 0.2)]), np.array([(0.8, 0.5, 1.0)]), np.array([r]))[0]
    assert box2[3] - box2[0] == pytest.approx(0.6 + 2 * r * 0.8, abs=1e-6)
    # a ray that passes the negative beam's start within R+r but outside its shrunken box: 0
    R = 0.05
    # beam start x = 0.8; shrunken box max x = 0.5 + (0.6 - 0.08)/2 = 0.76
    segs = seg((0.78, 0.0, 0.2 + 1e-3), (0.78, 1.0, 0.2 - 1e-3))
    out = gather1(oracle, one_beam(start, end, r), segs, R)
    assert out["cand"][0] == 0
    segs2 = seg((0.22, 0.0, 0.2 + 1e-3), (0.22, 1.0, 0.2 - 1e-3))
    out2 = gather1(oracle, one_beam((0.2, 0.5, 0.2), (0.8, 0.5, 1.0), r), segs2, R)
    assert out2["cand"][0] == 1 and out2["contrib"][0] == 1


def test_parallel_segment_contributes_nothing(oracle):
    """cross(A,B) == 0 -> ComputeClosestPoints returns false (photonbeam.cpp:131-156)."""
    beams = one_beam((0.1, 0.5, 0.5), (0.9, 0.5, 0.5), 0.05)
    segs = seg((0.0, 0.5, 0.5), (1.0, 0.5, 0.5))  # collinear
    out = gather1(oracle, beams, segs, 0.05)
    assert out["cand"][0] == 1 and out["contrib"][0] == 0


def test_closest_point_clamped_to_beam_end(oracle):
    """Segment crossing beyond the beam's end: t1 > magB and t0 in range -> the beam point stays
    on the beam LINE (unclamped, photonbeam.cpp:178-181 re-projects only pA)."""
    ok, ac, bc = oracle.closest_points((0, 0.0, 0.0), (0, 2.0, 0.0), (1.0, 1.0, 1.0), (0.5, 1.0, 1.0))
    # lines: A = y-axis, B along -x at (y=1, z=1): line-line closest points (0,1,0) and (0,1,1);
    # t1 = 1.0 > magB = 0.5, t0 = 1 in range -> pB = b0 + B*t1 = (0,1,1) (off the beam), pA = (0,1,0)
    assert ok
    np.testing.assert_allclose(bc, [0.0, 1.0, 1.0], atol=1e-7)
    np.testing.assert_allclose(ac, [0.0, 1.0, 0.0], atol=1e-7)
    # t0 out of range: pA clamps to a1, pB re-projected and clamped onto the beam
    ok, ac, bc = oracle.closest_points((0, 0.0, 0.0), (0, 0.5, 0.0), (0.5, 1.0, 1.0), (-0.5, 1.0, 1.0))
    np.testing.assert_allclose(ac, [0.0, 0.5, 0.0], atol=1e-7)
    np.testing.assert_allclose(bc, [0.0, 1.0, 1.0], atol=1e-7)


def test_zero_length_segment(oracle):
    """magA == 0: aClosest = a0, bClosest = clamped projection on B (photonbeam.cpp:95-108)."""
    ok, ac, bc = oracle.closest_points((0.3, 0.2, 0.0), (0.3, 0.2, 0.0), (0.0, 0.0, 0.0), (1.0, 0.0, 0.0))
    assert ok
    np.testing.assert_allclose(ac, [0.3, 0.2, 0.0])
    np.testing.assert_allclose(bc, [0.3, 0.0, 0.0], atol=1e-7)
    ok, ac, bc = oracle.closest_points((1.5, 0.2, 0.0), (1.5, 0.2, 0.0), (0.0, 0.0, 0.0), (1.0, 0.0, 0.0))
    np.testing.assert_allclose(bc, [1.0, 0.0, 0.0])


def test_zero_length_beam_box_is_nan(oracle):
    box = oracle.beam_bounds(np.array([(0.5, 0.5, 0.5)]), np.array([(0.5, 0.5, 0.5)]), np.array([0.01]))[0]
    assert np.isnan(box).all()


def test_empty_group_box_semantics(oracle):
    """Beams with identical centroids share one SAH leaf (photonbeambvh.cpp:289-297): a beam whose
    own box is missed is still gathered when its twin's box is hit."""
    r = 0.01
    a = ((0.2, 0.5, 0.5), (0.8, 0.5, 0.5))    # +x beam
    b = ((0.5, 0.2, 0.5), (0.5, 0.8, 0.5))    # +y beam, same centre
    beams = {"start": np.array([a[0], b[0]], f32), "end": np.array([a[1], b[1]], f32),
             "radius": np.array([r, r], f32), "power": np.array([(1, 1, 1), (1, 1, 1)], f32)}
    bvh = oracle.build(beams)
    assert bvh.max_leaf() == 2  # one leaf with both beams
    # segment along z at (0.3, 0.5): inside beam a's box (x in [0.2,0.8], y in [0.49,0.51]) only
    segs = seg((0.3, 0.5 + 1e-4, 0.0), (0.3 + 1e-4, 0.5, 1.0))
    out = bvh.gather(segs, 0.05)
    assert out["cand"][0] == 2  # both returned by the leaf
    bf = oracle.bruteforce(beams, segs, 0.05)
    assert bf["cand"][0] == 2
