"""Graph capture and engine lifetime: a collection inside a capture ran an earlier engine's HIP finalizers while the
stream recorded and aborted the full GPU suite (profiles/r04ae, first attempt). engine._capture holds the cyclic GC off
(defence in depth); the cause — engines kept alive by reference cycles until a collection — is gone: engines are freed
by their reference count, WhisperEngine.close() releases everything in order, and a capture with the guard off and
collections forced inside it replays correctly."""
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


def test_public_engine_passes_run_on_the_engine_streams():
    """every public entry point that launches work is wrapped by on_engine_streams (ordered after
    the caller's stream on entry, the caller's stream waits on exit)."""
    for name in ("decode_pass", "sample_pass", "beam_pass", "generate", "run_batches", "decoder_step", "encode",
                 "logmel", "set_long_input", "_detect_languages"):
        fn = getattr(engine.WhisperEngine, name)
        assert getattr(fn, "__wrapped__", None) is not None, name


def _mini(seed=1234):
    from twamd.config import PRESETS, GenerationSettings
    from twamd.weights import build_weights
    dims = PRESETS["test-mini"]
    return engine.WhisperEngine(build_weights(dims, seed=seed), GenerationSettings.default(dims), max_batch=2,
                                device="cuda")


def _prime(eng):
    import numpy as np
    from twamd.synth_audio import speech_like
    host = np.stack([speech_like(30.0, 1234), speech_like(30.0, 99)]).astype(np.float32)
    eng.wave[:2].copy_(torch.from_numpy(host))
    eng.logmel(2)
    eng.row_map[:2] = torch.arange(2, dtype=torch.int32, device="cuda")
    eng.seek[:2] = 0
    eng.encode(2)


@pytest.mark.gpu
def test_dropped_engine_leaves_no_cycle_and_capture_needs_no_gc_guard(monkeypatch):
    """an engine that captured graphs is freed by its reference count alone (no cycle keeps it for
    the cyclic GC), so a collection inside a later capture finds no HIP object to finalize: another engine captures
    with the GC guard off and collections forced throughout, and its replayed decode equals the first engine's."""
    import weakref
    a = _mini()
    _prime(a)
    tail = a.prompt_tail("transcribe", True)
    want = a.decode_pass(2, tail, None, 24).tokens
    assert a._graphs  # prompt + step graphs captured
    ref = weakref.ref(a)
    del a
    assert ref() is None  # freed by refcount: its graphs and events are gone now, outside any capture
    monkeypatch.setattr(engine, "CAPTURE_GC_GUARD", False)
    b = _mini()
    _prime(b)
    old = gc.get_threshold()
    gc.set_threshold(1, 1, 1)  # a collection on (almost) every allocation, captures included
    try:
        got = b.decode_pass(2, tail, None, 24).tokens
        again = b.decode_pass(2, tail, None, 24).tokens  # replays of the graphs captured without the guard
    finally:
        gc.set_threshold(*old)
    assert got == want and again == want
    b.close()


@pytest.mark.gpu
def test_close_releases_and_refuses_further_use():
    eng = _mini()
    _prime(eng)
    tail = eng.prompt_tail("transcribe", True)
    first = eng.decode_pass(2, tail, None, 16).tokens
    with _mini() as other:  # the context manager closes on exit
        _prime(other)
        assert other.decode_pass(2, tail, None, 16).tokens == first
    assert other.closed and other._graphs is None
    eng.close()
    eng.close()  # idempotent
    with pytest.raises(RuntimeError, match="closed"):
        eng.decode_pass(2, tail, None, 16)


@pytest.mark.gpu
def test_decode_pass_from_the_callers_stream_equals_engine_stream_call():
    """decode_pass called from the default stream (the wrapper orders it after the caller's work and the
    caller after it) returns what the call on the engine's own stream returns."""
    eng = _mini()
    _prime(eng)
    tail = eng.prompt_tail("transcribe", True)
    with torch.cuda.stream(eng.stream):
        inside = eng.decode_pass(2, tail, None, 32).tokens
    outside = eng.decode_pass(2, tail, None, 32).tokens
    assert outside == inside
    eng.close()
