"""include/bre_fmath.h against the host libm, bit for bit (CPU).

The reference calls std::exp / std::log / std::sin / std::cos on floats: the x86-64 glibc libm's
expf / logf / sinf / cosf (spectrum.h:222-224, homogeneous.cpp:47,74, grid.cpp:76,104,
sampling.cpp:127, medium.cpp:194-213).  bre_fmath.h restates their algorithms (glibc >= 2.28) with
explicit fused multiply-adds where libm's FMA variants have them; the photon and camera passes on the
GPU and the oracle both use it.  tests/fmath_libm_check.c compares every STRIDE-th float bit pattern;
the full sweep (stride 1, all 2^32 inputs, ~40 s on 8 threads) is in
profiles/r6/fmath_libm_exhaustive.txt and runs here with BRE_FMATH_EXHAUSTIVE=1.  The GPU side of
the same functions is tests/test_fmath_gpu.py."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("fmath") / "fmath_libm_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-builtin", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "fmath_libm_check.c"), "-o", exe, "-lm"], check=True)
    return exe


def test_fmath_equals_libm_on_a_sweep_of_all_floats(checker):
    stride = 1 if os.environ.get("BRE_FMATH_EXHAUSTIVE") == "1" else 257
    r = subprocess.run([checker, str(stride), "8"], capture_output=True, text=True, timeout=600)
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 4, r.stdout + r.stderr
    for line in lines:
        assert " 0 of " in line, line
    assert r.returncode == 0
