"""Graph capture holds Python's cyclic GC off (engine._capture): a collection inside a capture ran an earlier engine's
HIP finalizers while the stream recorded and aborted the full GPU suite (profiles/r04ae, first attempt)."""
import gc
import inspect

import pytest
import torch

from twamd import engine


def test_every_capture_site_goes_through_the_gc_guard():
    src = inspect.getsource(engine)
    assert src.count("torch.cuda.graph(") == 1  # the one inside _capture
    assert src.count("_capture(g,") >= 3  # prompt, beam step and the decode step graphs


@pytest.mark.gpu
def test_capture_with_garbage_pending():
    s = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")
    # garbage whose collection would free device memory: reference cycles holding CUDA tensors and events
    for _ in range(200):
        a = {"t": torch.ones(256, device="cuda"), "e": torch.cuda.Event()}
        a["self"] = a
    del a
    g = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with engine._capture(g, s):
            assert not gc.isenabled()
            junk = [[i] for i in range(5000)]  # allocations that would trigger a collection
            junk.append(junk)
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    assert gc.isenabled()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0
