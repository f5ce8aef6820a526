"""CU-masked replica streams (runner.py ``cu_frac``, bench.py --small-cu-frac)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_cu_masked_stream_runs_graphless_work():
    """A stream limited to 3/4 of the CUs (hipExtStreamCreateWithCUMask via
    librnb_runtime.so) runs kernels with the same results as the default
    stream."""
    from rnb_amd.runner import _cu_masked_stream
    dev = torch.device("cuda:0")
    s = _cu_masked_stream(dev, 0.75)
    assert s is not None
    a = torch.randn(512, 512, device=dev)
    ref = a @ a
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        out = a @ a
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    assert torch.allclose(out, ref)
