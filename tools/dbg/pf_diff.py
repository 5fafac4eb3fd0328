"""Debug: per-level pyramid / raw FAST cell keys of the fused path vs the oracle for one image."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle
from orb_slam3_ros_amd.extractor import ORBextractor
from orb_slam3_ros_amd.synth import synth_stereo
sys.path.insert(0, "tests")
from test_gpu_extractor import _gpu_cell_keys, _cell_geom, _unpack

seed, side, path = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
W, H = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (752, 480)
img = synth_stereo(seed, W, H)[side]
ext = ORBextractor(1000, 1.2, 8, 20, 7)
ext.set_path(path)
ora = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
ext(img)
ora(img)
for l in range(8):
    pg, po = ext.pyramid_level(l), ora.pyramid_level(l)
    npx = int((pg != po).sum())
    raw_o = ora.debug_keys(l, 0)
    ncell, cap = _cell_geom(*po.shape[::-1])
    cnt = np.zeros(ncell, np.int32)
    ext._lib.orbfe_debug_copy(ext.handle, 0, 0, l, cnt.ctypes.data, cnt.nbytes)
    raw_g = _gpu_cell_keys(ext, l, ncell, cap)
    gx, gy, gs = _unpack(raw_g)
    ok = len(raw_g) == len(raw_o) and np.array_equal(gx, raw_o["x"].astype(np.uint32)) and \
        np.array_equal(gy, raw_o["y"].astype(np.uint32)) and np.array_equal(gs, raw_o["response"].astype(np.uint32))
    print(f"level {l}: pyramid px differ {npx}, raw keys gpu {len(raw_g)} oracle {len(raw_o)} match {ok}")
    if not ok:
        # per-cell comparison: oracle keys grouped by cell order are contiguous; walk both
        W, H = po.shape[1], po.shape[0]
        width, height = np.float32(W - 32), np.float32(H - 32)
        ncols, nrows = int(width / np.float32(35)), int(height / np.float32(35))
        wc, hc = int(np.ceil(width / np.float32(ncols))), int(np.ceil(height / np.float32(nrows)))
        ox = raw_o["x"].astype(int); oy = raw_o["y"].astype(int); os_ = raw_o["response"].astype(int)
        i0 = 0
        for c in range(ncell):
            n = cnt[c]
            g = list(zip(gx[i0:i0 + n].tolist(), gy[i0:i0 + n].tolist(), gs[i0:i0 + n].tolist()))
            i0 += n
            ci, cj = divmod(c, ncols)
            # oracle keys of this cell: x,y relative to minB; cell of a key = its detection rect
            sel = [(x, y, s) for x, y, s in zip(ox, oy, os_) if
                   min((x - 3) // wc, ncols - 1) == cj and min((y - 3) // hc, nrows - 1) == ci]
            if g != sel:
                print(f"  cell {c} (row {ci}, col {cj}): gpu {len(g)} oracle {len(sel)}")
                sg = set(g); so = set((int(a), int(b), int(c)) for a, b, c in sel)
                print("   gpu only   ", sorted(sg - so, key=lambda t: (t[1], t[0])))
                print("   oracle only", sorted(so - sg, key=lambda t: (t[1], t[0])))
