"""bre_math.h div_by_shared: a / b from a shared correctly rounded reciprocal y = RN(1 / b), by two
Markstein corrections (q0 = a y; q += (a - b q) y, twice, the residuals exact by FMA), returns the
correctly rounded quotient RN(a / b).  The exact stage uses it for r = d / MaxDistance of a
uniform-radius set (one MaxDistance per gather).  Emulated here with exact rational FMAs against
IEEE float32 division, over the exact stage's range (0 <= d < MaxDistance) and its edges."""
import random
from fractions import Fraction as F

import numpy as np

f32 = np.float32


def _rn32(x: F) -> np.float32:
    """Nearest float32 (ties to even) of an exact rational."""
    if x == 0:
        return f32(0.0)
    s = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    while F(2) ** e > x:
        e -= 1
    while F(2) ** (e + 1) <= x:
        e += 1
    ulp = F(2) ** (max(e, -126) - 23)
    m = x / ulp
    n, rem = divmod(m.numerator, m.denominator)
    rem = F(rem, m.denominator)
    if rem > F(1, 2) or (rem == F(1, 2) and n % 2 == 1):
        n += 1
    return f32(s * float(n * ulp))


def _fma(a, b, c):
    return _rn32(F(float(a)) * F(float(b)) + F(float(c)))


def _div_by_shared(a, b, y):
    q0 = f32(a * y)
    q1 = _fma(_fma(-q0, b, a), y, q0)
    return _fma(_fma(-q1, b, a), y, q1)


def test_div_by_shared_is_correctly_rounded():
    rng = random.Random(11)
    n = 0
    for trial in range(60):
        b = f32(rng.uniform(1e-3, 0.05)) if trial % 2 else f32(0.01 * (1 + rng.randint(-8, 8) * 2.0 ** -23))
        y = f32(f32(1.0) / b)
        for k in range(60):
            mode = k % 3
            if mode == 0:
                a = f32(rng.uniform(0.0, float(b)))
            elif mode == 1:  # just below the divisor: quotients next to 1
                a = f32(b * f32(1 - rng.randint(1, 64) * 2.0 ** -24))
            else:  # many binades down
                a = f32(float(b) * 2.0 ** rng.uniform(-60, 0))
            if not (a < b):
                continue
            assert _div_by_shared(a, b, y) == f32(a / b), (a, b)
            n += 1
    assert n > 3000


def test_one_product_alone_is_not_enough():
    """The corrections matter: q0 = a * RN(1/b) alone misses the correctly rounded quotient often."""
    rng = random.Random(12)
    miss = 0
    for _ in range(2000):
        b = f32(rng.uniform(1e-3, 0.05))
        a = f32(rng.uniform(0.0, float(b)))
        miss += f32(a * f32(f32(1.0) / b)) != f32(a / b)
    assert miss > 200
