#!/usr/bin/env python3
"""Timing-only k_fast census builds (outputs INVALID): patched copies of the kernel sources, compiled
to variants/liborbfe_fast{1..4}.so, so the product source carries no ablation hooks.
  fast1: staging only (every cell returns after its ROI is in LDS)
  fast2: + pass 1 (pretest + group compaction), then the cell stops
  fast3: + entry expansion and pass 2 (exact scores), then the cell stops before NMS
  fast4: + NMS and emission of attempt 0, never the minThFAST fallback
  fast5: the product kernel
All five with -DFAST_NO_OVERLAP (every launch in stream order: isolated kernel times). usage: python tools/fast_census.py"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "orb_slam3_ros_amd", "csrc")

A1 = "    const uint8_t* s_px = s_img + 1;   // ROI pixel (y, x) = s_px[y * RS + x]\n"
A2 = "        WAVE_SYNC();\n        // per chunk of 64 groups: expand into entries"
A3 = "        // NMS over corners (every other pixel has score 0), fused with the emission"
A4 = "        if (nsurv > 0) break;"


def patched(level: int, src: str) -> str:
    for a in (A1, A2, A3, A4):
        assert src.count(a) == 1, a
    if level == 1:
        return src.replace(A1, A1 + "    { asm volatile(\"\" ::\"v\"((int)s_img[lane])); if (lane == 0) "
                           "cellcnt[(size_t)b * g.total_cells + c] = 0; WAVE_SYNC(); return; }\n")
    if level == 2:
        return src.replace(A2, "        WAVE_SYNC();\n        { asm volatile(\"\" ::\"v\"(ngrp)); nsurv = 0; break; }\n"
                           "        // per chunk of 64 groups: expand into entries")
    if level == 3:
        return src.replace(A3, "        { asm volatile(\"\" ::\"v\"((int)s_sc[lane]), \"v\"(ncorner)); nsurv = 0; break; }\n" + A3)
    if level == 4:
        return src.replace(A4, "        break;")
    return src


def main():
    os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
    src = open(os.path.join(CSRC, "orbfe_kernels.hip")).read()
    for level in (1, 2, 3, 4, 5):
        with tempfile.TemporaryDirectory() as d:
            # the sources include ../../include/orbfe.h
            shutil.copytree(CSRC, os.path.join(d, "pkg", "csrc"))
            shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
            open(os.path.join(d, "pkg", "csrc", "orbfe_kernels.hip"), "w").write(patched(level, src))
            out = os.path.join(ROOT, "variants", f"liborbfe_fast{level}.so")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                            "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-function", "-DFAST_NO_OVERLAP",
                            "-o", out, os.path.join(d, "pkg", "csrc", "orbfe_engine.hip")], check=True)
            print(out)


if __name__ == "__main__":
    main()
