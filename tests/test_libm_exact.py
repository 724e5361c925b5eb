"""The device restatement of glibc's expf / sinf / cosf (llamacog_amd/csrc/libm_exact.h) is
bit-exact against this host's libm — the functions the reference CPU backend calls in flash
attention (expf), the SiLU tail (expf) and the RoPE cache (cosf / sinf).

The header is compiled for the host by oracle/Makefile (build/libm_check) and compared on a
strided walk over every float bit pattern of the ranges those callers use; the exhaustive walk
(stride 1: 2.24e9 expf inputs in [-104, 89], 1.2e9 sinf / cosf inputs in [0, 2^18]) was run
when the header was written and found no mismatch."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "oracle", "build", "libm_check")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "build/libm_check"], check=True)
    return EXE


@pytest.mark.parametrize("func,lo,hi", [(0, "-0.0", "-104"), (0, "0", "89"), (1, "0", "262144"), (2, "0", "262144"),
                                        (1, "-0.0", "-1000"), (2, "-0.0", "-1000")])
def test_libm_restatement_bit_exact(exe, func, lo, hi):
    out = subprocess.run([exe, str(func), lo, hi, "1009"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "mismatches 0" in out.stdout
