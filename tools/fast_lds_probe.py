#!/usr/bin/env python3
"""Timing-only k_fast probes (outputs INVALID except `orig` / `cur`): is pass 1 bound by its LDS reads?
  orig:   the kernel source of git HEAD~N (N = $ORIG_REV, default HEAD)      (valid)
  cur:    the working tree's kernel                                        (valid)
  ldsx:   cur + 12 extra dword LDS reads per 4-pixel pass-1 test, consumed by an empty asm (valid
          outputs: the sensitivity of k_fast's time to pass-1 LDS traffic)
  valux:  cur + a 24-instruction dependent VALU chain per 4-pixel pass-1 test, consumed the same way
          (valid outputs: the sensitivity to pass-1 VALU)
All with -DFAST_NO_OVERLAP. usage: python tools/fast_lds_probe.py; then REPS=2 bash tools/gpu_variants_trace.sh"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "orb_slam3_ros_amd", "csrc")

R1 = "                const uint32_t c0w = r0p[0], c2w = r0p[2];\n"
R2 = "                const uint32_t ph[8] = {0u, 0u, c2w, cw, r0p[2 * nd + 2], r0p[-2 * nd + 1], r0p[-2 * nd + 2], r0p[2 * nd + 1]};\n"
R3 = "                const uint32_t pl[8] = {r0p[3 * nd + 1], r0p[-3 * nd + 1], cw, c0w,          // (0, 3), (0, -3), (3, 0), (-3, 0)\n"
R4 = "                                        r0p[2 * nd + 1], r0p[-2 * nd], r0p[-2 * nd + 1], r0p[2 * nd]};   // (2, 2), (-2, -2), (2, -2), (-2, 2)\n"


def nolds1(src: str) -> str:
    for a in (R1, R2, R3, R4):
        assert src.count(a) == 1, a
    rot = lambda k: f"__builtin_amdgcn_alignbit(cw, cw, {k}u)"
    src = src.replace(R1, f"                const uint32_t c0w = {rot(3)}, c2w = {rot(5)};\n")
    src = src.replace(R2, f"                const uint32_t ph[8] = {{0u, 0u, c2w, cw, {rot(7)}, {rot(9)}, {rot(11)}, {rot(13)}}};\n")
    src = src.replace(R3, f"                const uint32_t pl[8] = {{{rot(15)}, {rot(17)}, cw, c0w,\n")
    src = src.replace(R4, f"                                        {rot(19)}, {rot(21)}, {rot(23)}, {rot(25)}}};\n")
    return src


def ldsx(src: str) -> str:
    assert src.count(R1) == 1
    extra = ("                asm volatile(\"\" ::\"v\"(r0p[nd]), \"v\"(r0p[-nd]), \"v\"(r0p[nd + 1]), \"v\"(r0p[-nd + 1]),"
             " \"v\"(r0p[nd + 2]), \"v\"(r0p[-nd + 2]), \"v\"(r0p[3 * nd]), \"v\"(r0p[-3 * nd]), \"v\"(r0p[3 * nd + 2]),"
             " \"v\"(r0p[-3 * nd + 2]), \"v\"(r0p[1]), \"v\"(r0p[4 * nd + 1]));\n")
    return src.replace(R1, R1 + extra)


def valux(src: str) -> str:
    assert src.count(R1) == 1
    chain = ("                { uint32_t z = c0w;\n#pragma unroll\n                  for (int u = 0; u < 24; u++) z = __builtin_amdgcn_alignbit(z, z, 7u + u);\n"
             "                  asm volatile(\"\" ::\"v\"(z)); }\n")
    return src.replace(R1, R1 + chain)


def build(name, src):
    with tempfile.TemporaryDirectory() as d:
        shutil.copytree(CSRC, os.path.join(d, "pkg", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
        open(os.path.join(d, "pkg", "csrc", "orbfe_kernels.hip"), "w").write(src)
        out = os.path.join(ROOT, "variants", f"liborbfe_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-function", "-DFAST_NO_OVERLAP",
                        "-o", out, os.path.join(d, "pkg", "csrc", "orbfe_engine.hip")], check=True)
        print(out)


def main():
    shutil.rmtree(os.path.join(ROOT, "variants"), ignore_errors=True)
    os.makedirs(os.path.join(ROOT, "variants"))
    cur = open(os.path.join(CSRC, "orbfe_kernels.hip")).read()
    orig = subprocess.run(["git", "show", os.environ.get("ORIG_REV", "HEAD") + ":orb_slam3_ros_amd/csrc/orbfe_kernels.hip"],
                          cwd=ROOT, capture_output=True, text=True, check=True).stdout
    build("orig", orig)
    build("cur", cur)
    build("ldsx", ldsx(cur))
    build("valux", valux(cur))


if __name__ == "__main__":
    main()
