"""orbfe_copy_stream (bench.py's measured HBM ceiling): byte-exact copies of sizes that exercise the
unrolled rounds and the tail, and the argument checks."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [16, 16 * 255, 16 * 4097, (1 << 24) + 16 * 37])
def test_copy_stream_exact(nbytes):
    import torch
    from orb_slam3_ros_amd import _lib
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    b = torch.zeros_like(a)
    s = torch.cuda.current_stream()
    assert lib.orbfe_copy_stream(a.data_ptr(), b.data_ptr(), nbytes, s.cuda_stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_copy_stream_rejects_unaligned():
    import torch
    from orb_slam3_ros_amd import _lib
    lib = _lib.load()
    a = torch.zeros(64, dtype=torch.uint8, device="cuda")
    assert lib.orbfe_copy_stream(a.data_ptr(), a.data_ptr() + 16, 24, None) < 0
