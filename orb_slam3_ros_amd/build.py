"""In-tree build of liborbfe.so (hipcc, gfx950). The .so travels to the GPU box with the snapshot."""
from __future__ import annotations

import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, "csrc")
LIB = os.path.join(_HERE, "liborbfe.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["orbfe_engine.hip"]
DEPS = ["orbfe_engine.hip", "orbfe_kernels.hip", "orbfe_types.h", "glibc_sincosf.h", "stl_sort.h",
        "brief_pattern.h", "orbfe_matcher.hip", "orbfe_bow.hip", "glibc_logf.h", "glibc_atan2f.h", "orbfe_remap.hip", "orbfe_backend.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-Wno-unused-function"]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    hdr = os.path.join(os.path.dirname(_HERE), "include", "orbfe.h")
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps + [hdr])


CAPI_SRC = os.path.join(os.path.dirname(_HERE), "tests", "native", "capi_frontend.cpp")
CAPI_BIN = os.path.join(os.path.dirname(_HERE), "tests", "native", "capi_frontend")
TRACK_HDR = os.path.join(os.path.dirname(_HERE), "tests", "native", "tracking_loop.h")
TRACK_KB8_HDR = os.path.join(os.path.dirname(_HERE), "tests", "native", "tracking_kb8.h")
TRACK_CPU_SRC = os.path.join(os.path.dirname(_HERE), "tests", "native", "tracking_cpu.cpp")
TRACK_CPU_BIN = os.path.join(os.path.dirname(_HERE), "tests", "native", "tracking_cpu")
ORACLE_LIB = os.path.join(os.path.dirname(_HERE), "oracle", "liborb_oracle.so")
GLUE_HDR = os.path.join(os.path.dirname(_HERE), "shim", "orbfe_glue.h")


def build_library(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, d) for d in DEPS]
    if force or _stale(LIB, deps):
        cmd = [HIPCC] + FLAGS + ["-o", LIB] + [os.path.join(CSRC, s) for s in SOURCES]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return LIB


def build_capi_consumer(force: bool = False, verbose: bool = False) -> str:
    """The compiled C++ consumer of include/orbfe.h (tests/native/capi_frontend.cpp), linked against the
    in-tree liborbfe.so by name with an $ORIGIN-relative runpath so it runs from the GPU box's copy."""
    if force or _stale(CAPI_BIN, [CAPI_SRC, TRACK_HDR, TRACK_KB8_HDR, LIB, GLUE_HDR]):
        # no contraction: the harness's host-side projections must round as the CPU twin's do
        cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wall", "-I", os.path.join(os.path.dirname(_HERE), "include"),
               "-I", os.path.join(os.path.dirname(_HERE), "shim"),
               "-o", CAPI_BIN, CAPI_SRC, "-L", _HERE, "-lorbfe", "-Wl,-rpath,$ORIGIN/../../orb_slam3_ros_amd",
               "-Wl,-rpath-link,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return CAPI_BIN


def build_tracking_cpu(force: bool = False, verbose: bool = False) -> str:
    """TEST INFRASTRUCTURE: the CPU Tracking-frame timer / parity reference (tests/native/tracking_cpu.cpp),
    tests/native/tracking_loop.h over the oracle's restatement (oracle/liborb_oracle.so, built first by
    oracle/Makefile). Only the CPU-baseline leg of bench.py and the tests run it."""
    if force or _stale(TRACK_CPU_BIN, [TRACK_CPU_SRC, TRACK_HDR, TRACK_KB8_HDR, ORACLE_LIB]):
        # -ffp-contract=off: -march=x86-64-v3 has FMA, and g++ would contract the host-side projections
        # and pose arithmetic of tests/native/tracking_*.h differently from the GPU consumer's build
        cmd = ["g++", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-std=c++17", "-Wall", "-pthread", "-I",
               os.path.join(os.path.dirname(_HERE), "include"), "-o", TRACK_CPU_BIN, TRACK_CPU_SRC, ORACLE_LIB,
               "-Wl,-rpath,$ORIGIN/../../oracle"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return TRACK_CPU_BIN


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
