"""CPU: the drop-in shim (shim/*.cc, shim/orbfe_glue.h) compiles against include/orbfe.h. The shim needs
OpenCV / Eigen / Sophus / the ORB-SLAM3 headers, none of which exist here, so it is compiled with
-fsyntax-only against minimal stand-ins of the types it touches (tests/shim_stubs/, declarations with the
reference's names). A change of an orbfe_* signature, struct field or constant that the shim no longer
matches fails this test."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIMS = sorted(glob.glob(os.path.join(ROOT, "shim", "*.cc")))


def _gxx(src, extra=()):
    return subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                           "-Wno-unused-function", "-I", os.path.join(ROOT, "tests", "shim_stubs"), "-I",
                           os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "shim"), *extra, src],
                          capture_output=True, text=True, timeout=120)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("src", SHIMS, ids=[os.path.basename(s) for s in SHIMS])
def test_shim_compiles(src):
    r = _gxx(src)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_shim_set_is_complete():
    # the replacements INTEGRATION.md §2 lists, one file each
    names = {os.path.basename(s) for s in SHIMS}
    assert {"ORBextractor_orbfe.cc", "ORBmatcher_orbfe.cc", "ORBmatcher_backend_orbfe.cc", "Frame_orbfe.cc",
            "Tracking_orbfe.cc"} <= names


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_shim_compile_catches_abi_drift(tmp_path):
    """The check bites: the same shim against a copy of orbfe.h with one argument dropped from
    orbfe_frame_stereo fails to compile."""
    inc = tmp_path / "include"
    inc.mkdir()
    hdr = open(os.path.join(ROOT, "include", "orbfe.h")).read()
    old = "                       int* mono_right, float* uright, float* depth);"
    assert old in hdr
    (inc / "orbfe.h").write_text(hdr.replace(old, "                       int* mono_right, float* uright);"))
    r = subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "shim_stubs"), "-I",
                        str(inc), "-I", os.path.join(ROOT, "shim"), os.path.join(ROOT, "shim", "Frame_orbfe.cc")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "orbfe_frame_stereo" in r.stderr
