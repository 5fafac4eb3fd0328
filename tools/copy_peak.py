"""bench.py's measured copy ceiling alone (TB/s), for copy-kernel A/B builds (ORBFE_LIB)."""
import sys
sys.path.insert(0, ".")
import torch  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
print(" ".join(f"{bench.copy_peak_gbps(torch, dev) / 1e3:.3f}" for _ in range(3)))
