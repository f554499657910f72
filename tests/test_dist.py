"""Chunk data parallelism (twamd.dist) on CPU: world_size-2 (and C3's 8-way) gloo process groups over 127.0.0.1.

The engine itself needs the GPU, so the per-rank window work is a deterministic stand-in that turns each window's
samples into a valid Whisper token sequence; what is under test is the sharding, the waveform broadcast, the
all-gather reassembly and the stitched transcript, which must equal the single-process result exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from twamd import dist as twd
from twamd.config import GenerationSettings, PRESETS
from twamd.frontend import chunk_windows, time_precision
from twamd.tokenizer import WhisperVocab, decode_asr

ST = GenerationSettings.default(PRESETS["large-v3-turbo"]).special


def fake_windows(wav, windows):
    """Deterministic per-window 'generate' output: <ts> text... <ts> pairs derived from the samples."""
    out = []
    for w in windows:
        seg = wav[w.start: w.start + min(w.length, 480000)]
        h = int(abs(float(seg[::997].sum())) * 1000) % 5000
        n = 1 + h % 7
        toks = [ST.timestamp_begin]
        for i in range(n):
            toks.append(300 + (h + 37 * i) % 20000)
        toks.append(ST.timestamp_begin + 50 + h % 1400)
        out.append(toks)
    return out


def fake_timed_windows(wav, windows):
    """(tokens, per-token float32 times) pairs, as the word-timestamp path returns them."""
    return [(t, [float(np.float32(0.02 * (i + 1) + 1e-3 * (j % 7))) for i in range(len(t))])
            for j, t in enumerate(fake_windows(wav, windows))]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, n_samples, chunk, stride, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        rng = np.random.default_rng(3)
        wav = rng.standard_normal(n_samples).astype(np.float32) if rank == 0 else None
        wav = twd.broadcast_waveform(wav)
        windows = list(chunk_windows(len(wav), chunk, stride, 16000))
        seqs = twd.transcribe_sharded(fake_windows, wav, windows)
        langs = [None] * len(windows)
        lo, hi = twd.shard_range(len(windows), ws, rank)
        g_seqs, g_langs = twd.gather_tokens(seqs[lo:hi], [rank] * (hi - lo), len(windows))
        timed = twd.transcribe_sharded(fake_timed_windows, wav, windows, timed=True)
        q.put((rank, seqs, g_langs, float(wav.sum()), timed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_samples,chunk,stride", [(3600 * 16000 // 10, 30, 0), (200 * 16000, 60, 5),
                                                     (16000 * 20, 30, 0)])
def test_two_rank_gather_equals_single_process(n_samples, chunk, stride):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_samples, chunk, stride, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rng = np.random.default_rng(3)
    wav = rng.standard_normal(n_samples).astype(np.float32)
    windows = list(chunk_windows(len(wav), chunk, stride, 16000))
    ref = fake_windows(wav, windows)
    sizes = twd.shard_sizes(len(windows), 2)
    sizes = twd.shard_sizes(len(windows), 2)
    ref_timed = []
    for r in range(2):  # each rank's stand-in numbers its windows from 0
        lo, hi = twd.shard_range(len(windows), 2, r)
        ref_timed += fake_timed_windows(wav, windows[lo:hi])
    for rank, seqs, g_langs, wsum, timed in res:
        assert wsum == pytest.approx(float(wav.sum()))
        assert seqs == ref
        assert timed == ref_timed  # float32 times travel bit-exactly
        assert g_langs == [0] * sizes[0] + [1] * sizes[1]
    # the stitched transcript is the single-process one
    vocab = WhisperVocab.synthetic(ST)
    mo = [{"tokens": t, "stride": (w.length / 16000, w.stride_left / 16000, w.stride_right / 16000)}
          for w, t in zip(windows, res[0][1])]
    mo_ref = [{"tokens": t, "stride": (w.length / 16000, w.stride_left / 16000, w.stride_right / 16000)}
              for w, t in zip(windows, ref)]
    assert decode_asr(vocab, mo, True, False, time_precision(1500)) == decode_asr(vocab, mo_ref, True, False,
                                                                                  time_precision(1500))


def test_shard_ranges_cover_in_order():
    for n in (0, 1, 7, 24, 120, 121):
        for ws in (1, 2, 3, 8):
            rs = [twd.shard_range(n, ws, r) for r in range(ws)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(ws - 1))
            assert max(twd.shard_sizes(n, ws)) - min(twd.shard_sizes(n, ws)) <= 1


def test_pack_unpack_roundtrip_and_limits():
    seqs = [[1, 2, 3], [], list(range(448))]
    arr = twd.pack_tokens(seqs, [5, None, 7], 4)
    s2, l2 = twd.unpack_tokens(arr, 3)
    assert s2 == seqs and l2 == [5, None, 7]
    with pytest.raises(ValueError):
        twd.pack_tokens([list(range(449))], None, 1)
    with pytest.raises(ValueError):
        twd.pack_tokens([[1], [2]], None, 1)


class _RecordingASR:
    def __init__(self):
        self.calls = []

    def __call__(self, inputs, **kw):
        rank, ws = twd.world()
        wav = np.asarray(inputs, np.float32) if rank == 0 else None
        wav = twd.broadcast_waveform(wav)
        windows = list(chunk_windows(len(wav), kw["chunk_length_s"], kw.get("stride_length_s"), 16000))
        seqs = twd.transcribe_sharded(fake_windows, wav, windows)
        self.calls.append(kw)
        return seqs


def _serve_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        fe = twd.RankZeroFrontend(_RecordingASR())
        if rank == 0:
            rng = np.random.default_rng(9)
            outs = [fe(rng.standard_normal(16000 * s).astype(np.float32), chunk_length_s=30, stride_length_s=0)
                    for s in (95, 40)]
            fe.close()
            q.put((0, outs))
        else:
            q.put((rank, fe.follow()))
    finally:
        dist.destroy_process_group()


def long_windows(wav, windows):
    """Windows whose 'generate' output ran several seek passes: more tokens than one pass can return (> 448)."""
    return [[ST.timestamp_begin] + [300 + (w.start // 997 + i) % 20000 for i in range(600 + 37 * j)]
            + [ST.timestamp_begin + 1400] for j, w in enumerate(windows)]


def failing_on_rank1(wav, windows):
    if twd.world()[0] == 1:
        raise RuntimeError("engine fault on rank 1")
    return fake_windows(wav, windows)


def malformed_on_rank1(wav, windows):
    """Rank 1 returns items that are not (tokens, times) pairs: a local failure that must still be collective."""
    if twd.world()[0] == 1:
        return [object() for _ in windows]
    return fake_timed_windows(wav, windows)


def _edge_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        rng = np.random.default_rng(5)
        wav = rng.standard_normal(16000 * 150).astype(np.float32)
        windows = list(chunk_windows(len(wav), 30, 0, 16000))
        res = {"long": twd.transcribe_sharded(long_windows, wav, windows)}
        try:
            twd.transcribe_sharded(failing_on_rank1, wav, windows)
            res["fail"] = None
        except twd.PeerError as e:
            res["fail"] = ("peer", str(e))
        except RuntimeError as e:
            res["fail"] = ("own", str(e))
        try:  # a malformed result on one rank (timed mode) is reported on every rank
            twd.transcribe_sharded(malformed_on_rank1, wav, windows, timed=True)
            res["malformed"] = None
        except twd.PeerError:
            res["malformed"] = "peer"
        except (TypeError, ValueError):
            res["malformed"] = "own"
        # gather_tokens with an explicit width and a shard-size mismatch on one rank raises on every rank
        lo, hi = twd.shard_range(len(windows), ws, rank)
        mine = fake_windows(wav, windows[lo:hi])
        if rank == 1:
            mine = mine[:-1]
        try:
            twd.gather_tokens(mine, None, len(windows), width=8)
            res["mismatch"] = None
        except twd.PeerError:
            res["mismatch"] = "peer"
        except ValueError:
            res["mismatch"] = "own"
        # an explicit width narrower than the sequences is widened to the agreed maximum
        full = fake_windows(wav, windows[lo:hi])
        res["narrow"] = twd.gather_tokens(full, None, len(windows), width=1)[0]
        # the collectives still line up after a failed call
        res["after"] = twd.transcribe_sharded(fake_windows, wav, windows)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_two_rank_long_windows_and_collective_failure():
    """a window can return more than 448 tokens (several seek passes): the gather width is agreed over
    the ranks instead of fixed; an engine failure on one rank raises on every rank instead of leaving the others
    blocked in the all-gather, and the group stays usable."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_edge_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rng = np.random.default_rng(5)
    wav = rng.standard_normal(16000 * 150).astype(np.float32)
    windows = list(chunk_windows(len(wav), 30, 0, 16000))
    ref_long = []
    for r in range(2):
        lo, hi = twd.shard_range(len(windows), 2, r)
        ref_long += long_windows(wav, windows[lo:hi])
    assert max(len(s) for s in ref_long) > twd.MAX_TOKENS
    for r in (0, 1):
        assert res[r]["long"] == ref_long
        assert res[r]["after"] == fake_windows(wav, windows)
    assert res[1]["fail"] == ("own", "engine fault on rank 1")
    assert res[0]["fail"][0] == "peer"
    assert (res[0]["malformed"], res[1]["malformed"]) == ("peer", "own")
    assert (res[0]["mismatch"], res[1]["mismatch"]) == ("peer", "own")
    assert res[0]["narrow"] == res[1]["narrow"] == fake_windows(wav, windows)


class _LoadingASR(_RecordingASR):
    """Decodes like TurboTranscriber.__call__: rank 0 loads the input (here: None is a broken upload) and tells the
    other ranks through broadcast_waveform whether it failed."""

    def __call__(self, inputs, **kw):
        rank, ws = twd.world()
        wav, err = None, None
        if rank == 0:
            try:
                if inputs is None:
                    raise ValueError("corrupt upload")
                wav = np.asarray(inputs, np.float32)
            except ValueError as e:
                err = e
        wav = twd.broadcast_waveform(wav, failed=err is not None)
        if err is not None:
            raise err
        windows = list(chunk_windows(len(wav), kw["chunk_length_s"], kw.get("stride_length_s"), 16000))
        seqs = twd.transcribe_sharded(fake_windows, wav, windows)
        self.calls.append(kw)
        return seqs


def _serve_bad_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        fe = twd.RankZeroFrontend(_LoadingASR())
        if rank == 0:
            out = []
            try:
                fe(None, chunk_length_s=30, stride_length_s=0)
            except ValueError as e:
                out.append(str(e))
            rng = np.random.default_rng(9)
            out.append(fe(rng.standard_normal(16000 * 40).astype(np.float32), chunk_length_s=30, stride_length_s=0))
            fe.close()
            q.put((0, out))
        else:
            q.put((rank, fe.follow()))
    finally:
        dist.destroy_process_group()


def test_rank_zero_frontend_survives_bad_input():
    """rank 0 failing to decode an upload must not leave the followers blocked in the waveform broadcast:
    rank 0 raises (-> the reference's error dict upstream), followers skip the call and keep serving."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_bad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][0] == "corrupt upload"
    assert res[1] == 1  # the good call was served, the failed one skipped
    rng = np.random.default_rng(9)
    wav = rng.standard_normal(16000 * 40).astype(np.float32)
    assert res[0][1] == fake_windows(wav, list(chunk_windows(len(wav), 30, 0, 16000)))


def test_rank_zero_frontend_serves_followers():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[1] == 2
    rng = np.random.default_rng(9)
    for s, out in zip((95, 40), res[0]):
        wav = rng.standard_normal(16000 * s).astype(np.float32)
        assert out == fake_windows(wav, list(chunk_windows(len(wav), 30, 0, 16000)))


# ---------------------------------------------------------------- the product call path, sharded (bench --config c3)
class _FakeEngine:
    """WhisperEngine's surface as TurboTranscriber.transcribe_windows drives it (max_batch, wave, run_batches with
    load(k) filling wave[:n]); each window's tokens are fake_windows' function of the samples that load() put in
    wave, so the test sees exactly what the sharded upload delivered."""

    def __init__(self, max_batch, tokens=None):
        self.tokens = tokens or (lambda wav, windows, idx: fake_windows(wav, windows))
        self.max_batch = max_batch
        self.wave = torch.zeros(max_batch, 480000)
        self.gen = GenerationSettings.default(PRESETS["large-v3-turbo"])
        self.device = torch.device("cpu")
        self.sizes = []
        self.done = 0  # windows run so far (rank-local)

        class d:
            max_source_positions = 1500
        self.d = d

    def run_batches(self, sizes, load=None, batch_kwargs=None, **kw):
        from twamd.frontend import Window
        out, self.batch_langs, self.batch_passes, self.batch_token_timestamps = [], [], [], []
        self.batch_prefixes = []
        for k, n in enumerate(sizes):
            load(k)
            rows = self.wave[:n].numpy()
            base = self.done
            toks = self.tokens(rows.reshape(-1), [Window(j * 480000, 480000, 0, 0, False) for j in range(n)],
                               [base + j for j in range(n)])
            self.done += n
            out.append(toks)
            self.batch_langs.append([None] * n)
            self.batch_passes.append([[t] for t in toks])
            self.batch_prefixes.append([[None] for _ in toks])
        self.sizes.append(list(sizes))
        return out


def _call_kwargs():
    return dict(chunk_length_s=30, stride_length_s=0, batch_size=24, return_timestamps=True,
                generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 128, "max_passes": 1})


def _call_worker(rank, ws, port, n_samples, max_batch, q):
    from twamd.pipeline import TurboTranscriber
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        eng = _FakeEngine(max_batch)
        tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
        wav = np.random.default_rng(5).standard_normal(n_samples).astype(np.float32) if rank == 0 else None
        q.put((rank, tr(wav, **_call_kwargs()), eng.sizes))
    finally:
        dist.destroy_process_group()


def test_sharded_transcriber_call_equals_single_process():
    """TurboTranscriber.__call__ at world size 2 (gloo), the path `bench.py --config c3` times: rank 0 decodes the
    input, the waveform is broadcast (kept as the collective's tensor), each rank uploads its windows from it into
    engine batches, the token arrays are all-gathered and stitched. Rank 0's transcript equals the single-process
    call's, and each rank ran its own half of the 24 windows."""
    from twamd.pipeline import TurboTranscriber
    n_samples = 24 * 480000 - 16000 * 7  # 24 windows, the last one ragged
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_call_worker, args=(r, 2, port, n_samples, 8, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    eng = _FakeEngine(8)
    tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
    ref = tr(np.random.default_rng(5).standard_normal(n_samples).astype(np.float32), **_call_kwargs())
    assert eng.sizes == [[8, 8, 8]]
    assert res[0][1] == ref and res[1][1] == ref  # every rank returns the stitched result
    assert res[0][2] == [[6, 6]] and res[1][2] == [[6, 6]]  # 12 windows per rank: two near-equal batches


def fake_open_windows(wav, windows, idx):
    """fake_windows whose closing timestamp is dropped (a segment left open into the next window) on every window
    that ends a 15-window shard of C3's 8-way split and on the windows whose first text token is 0 mod 3; `idx` are
    the global window indices of the batch."""
    out = fake_windows(wav, windows)
    for k, t in zip(idx, out):
        if k % 15 == 14 or t[1] % 3 == 0:
            t.pop()
    return out


def _c3_worker(rank, ws, port, n_samples, q):
    from twamd.pipeline import TurboTranscriber
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        eng = _FakeEngine(24, tokens=lambda wav, w, idx: fake_open_windows(wav, w, [i + 15 * rank for i in idx]))
        tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
        wav = np.random.default_rng(11).standard_normal(n_samples).astype(np.float32) if rank == 0 else None
        out = tr(wav, **_call_kwargs())
        q.put((rank, out, eng.sizes, twd.merge_pieces.last_restitched))
    finally:
        dist.destroy_process_group()


def test_c3_eight_rank_split_equals_single_process():
    """BASELINE config 3's exact partition, rehearsed on the CPU: one hour at 30-s windows (120 windows) over 8 gloo
    ranks, 15 windows and one engine batch per rank, transcribe_sharded + stitch_sharded with timestamps, segments
    left open across every rank boundary (the merge must re-stitch those shards). Every rank's result equals the
    single-process call's."""
    from twamd.pipeline import TurboTranscriber
    n_samples, ws = 3600 * 16000, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c3_worker, args=(r, ws, port, n_samples, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    eng = _FakeEngine(24, tokens=fake_open_windows)
    tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
    ref = tr(np.random.default_rng(11).standard_normal(n_samples).astype(np.float32), **_call_kwargs())
    assert eng.sizes == [[24] * 5] and len(ref["chunks"]) > 60
    for r, out, sizes, restitched in res:
        assert sizes == [[15]], (r, sizes)
        assert out == ref, r
        assert restitched >= 7  # every shard after the first opened with a segment in flight


def test_batch_sizes_policy():
    from twamd.pipeline import batch_sizes
    assert batch_sizes(0, 24) == []
    assert batch_sizes(120, 24) == [24] * 5
    assert batch_sizes(30, 24) == [15, 15]
    assert batch_sizes(49, 24) == [17, 16, 16]
    assert batch_sizes(15, 24) == [15]
    assert batch_sizes(15, 24, sub_batch_min=4) == [8, 7]
    assert batch_sizes(7, 24, sub_batch_min=4) == [7]
    for n in range(1, 100):
        s = batch_sizes(n, 24, 6)
        assert sum(s) == n and max(s) <= 24 and max(s) - min(s) <= 1


def test_fallback_keys_are_global_window_indices():
    """the fallback sampler's row keys come from global window indices (batch offset + rank shard
    base), so window j of batch 0 and window j of batch 1 draw different noise."""
    from twamd.engine import fallback_row_key
    from twamd.pipeline import TurboTranscriber
    from twamd.segments import FallbackConfig
    keys = {fallback_row_key(w, p, f) for w in range(200) for p in range(3) for f in range(6)}
    assert len(keys) == 200 * 3 * 6
    with pytest.raises(ValueError):
        fallback_row_key(2 ** 21, 0, 0)
    with pytest.raises(ValueError):  # a field past its width would alias another row's stream
        fallback_row_key(0, 1024, 0)
    with pytest.raises(ValueError):
        fallback_row_key(0, 0, 16)

    seen = []

    class Eng(_FakeEngine):
        def run_batches(self, sizes, load=None, batch_kwargs=None, **kw):
            seen.append((list(sizes), kw.get("window_offset")))
            return super().run_batches(sizes, load, batch_kwargs)

    eng = Eng(8)
    tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
    fb = FallbackConfig(temperatures=(0.0, 0.2), compression_ratio_threshold=2.4, logprob_threshold=-1.0,
                        no_speech_threshold=None, top_k=50, seed=0)
    wav = np.random.default_rng(5).standard_normal(20 * 480000).astype(np.float32)
    from twamd.frontend import chunk_windows
    ws = list(chunk_windows(len(wav), 30, 0, 16000))
    tr.transcribe_windows(wav, ws[10:], task="transcribe", lang_id=None, return_timestamps=True, fallback=fb,
                          window_base=10)
    assert seen == [([5, 5], 10)]  # run_batches adds each batch's offset: keys of windows 10..19


def test_checkpoint_thresholds_turn_the_fallback_on():
    """a checkpoint whose generation_config sets a fallback threshold turns the fallback on for every
    call; with the pipeline's default beam-5 the call runs (beam rounds inside the fallback) as with greedy passes,
    and the engine receives the checkpoint's criteria."""
    from twamd.pipeline import TurboTranscriber
    eng = _FakeEngine(8)
    eng.gen.logprob_threshold = -1.0
    seen = []
    orig = eng.run_batches

    def rb(sizes, load=None, batch_kwargs=None, **kw):
        seen.append((kw.get("num_beams"), kw.get("fallback")))
        return orig(sizes, load, batch_kwargs, **kw)

    eng.run_batches = rb
    tr = TurboTranscriber(eng, WhisperVocab.synthetic(ST))
    wav = np.zeros(16000, np.float32)
    for nb in (None, 1):
        gk = {"task": "transcribe", "max_passes": 1, **({"num_beams": nb} if nb else {})}
        out = tr(wav, chunk_length_s=30, generate_kwargs=gk, return_timestamps=True)
        assert "text" in out
    assert [nb for nb, _ in seen] == [5, 1] and all(f.logprob_threshold == -1.0 for _, f in seen)
