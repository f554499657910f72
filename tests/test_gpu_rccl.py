"""The RCCL path on hardware (30-s windows sharded over GPUs, ONE all-gather of token arrays; the
reference itself is single-GPU, /root/reference/vocalis/core/audio_pipeline.py:191).

A one-GPU box cannot form a multi-rank RCCL world, so these tests create an nccl (= RCCL) process group of world
size 1 on a TCP store at 127.0.0.1 — exactly as bench.py does for N > 1 — and force the collective path
(twamd.dist force_collective) that a world of one normally skips: the device-tensor all_reduce (agree),
all_gather_into_tensor (gather_tokens) and broadcast (broadcast_waveform) then run through RCCL and must return what
the host path returns. bench.py --force-collective runs the bench's per-batch all-gather the same way."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from twamd import dist as twd

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rccl_group():
    assert not dist.is_initialized()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dev
    dist.destroy_process_group()


def _seqs(n, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 51866, size=int(rng.integers(0, 300))).tolist() for _ in range(n)], \
        [int(x) if x >= 0 else None for x in rng.integers(-1, 100, size=n)]


def test_rccl_agree_gather_broadcast_equal_host_path(rccl_group):
    seqs, langs = _seqs(24, 1)
    host = twd.gather_tokens(seqs, langs, 24)  # world of one, not forced: returned as given
    assert twd.collective_path(True) and not twd.collective_path(False)
    dev = twd.gather_tokens(seqs, langs, 24, force_collective=True)
    assert dev == host == (seqs, langs)
    # a wider minimum width is honoured and changes nothing
    assert twd.gather_tokens(seqs, langs, 24, width=448, force_collective=True) == host
    assert twd.agree(False, 17) == (False, 17) and twd.agree(True, 3) == (True, 3)
    # a shard-size mismatch is reported before the gather (the agreement runs first)
    with pytest.raises(ValueError):
        twd.gather_tokens(seqs[:5], langs[:5], 24, force_collective=True)
    wav = np.random.default_rng(2).standard_normal(123457).astype(np.float32)
    buf = twd.broadcast_waveform(wav, as_tensor=True, force_collective=True)
    assert buf.device.type == "cuda" and torch.equal(buf.cpu(), torch.from_numpy(wav))
    assert np.array_equal(twd.broadcast_waveform(wav, force_collective=True), wav)
    assert twd.broadcast_waveform(wav, failed=True, force_collective=True) is None


def test_rccl_transcribe_sharded_equals_direct(rccl_group):
    windows = list(range(7))
    rng = np.random.default_rng(3)
    out = {w: rng.integers(0, 51866, size=int(rng.integers(1, 200))).tolist() for w in windows}
    times = {w: np.sort(rng.random(len(out[w])).astype(np.float32) * 30).tolist() for w in windows}

    def run(wav, ws):
        return [out[w] for w in ws]

    def run_timed(wav, ws):
        return [(out[w], times[w]) for w in ws]

    assert twd.transcribe_sharded(run, None, windows, force_collective=True) == run(None, windows)
    got = twd.transcribe_sharded(run_timed, None, windows, timed=True, force_collective=True)
    assert got == [(out[w], times[w]) for w in windows]  # float32 times travel bit-exactly

    def broken(wav, ws):
        raise RuntimeError("engine failure")

    with pytest.raises(RuntimeError, match="engine failure"):
        twd.transcribe_sharded(broken, None, windows, force_collective=True)


def test_rccl_transcriber_call_equals_single_gpu_call(rccl_group, monkeypatch):
    """The product call (TurboTranscriber.__call__: waveform broadcast from rank 0 in device memory, window shards,
    the token all-gather) through RCCL equals the plain single-GPU call."""
    from twamd.pipeline import TurboTranscriber
    from twamd.synth_audio import speech_like

    tr = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=4, device="cuda:0")
    wav = np.concatenate([speech_like(30.0, 5), speech_like(25.0, 6)]).astype(np.float32)
    kw = dict(chunk_length_s=30, stride_length_s=5, batch_size=4, return_timestamps=True,
              generate_kwargs={"task": "transcribe", "max_new_tokens": 24})
    plain = tr(wav, **kw)
    monkeypatch.setattr(twd, "FORCE_COLLECTIVE", True)
    assert twd.collective_path()
    forced = tr(wav, **kw)
    assert forced == plain


def test_bench_force_collective_line():
    """bench.py --force-collective (its own process: an nccl group of one around the engine's run_batches, one
    device-tensor all-gather per batch) prints a line that says so, with parity true."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-collective", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=280, env=env,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["collectives"] == "rccl (group of one, forced)"
    assert line["n_gpus"] == 1 and line["parity"] is True
