"""Host-side logic of the drop-in (CPU): chunk windows, seek-segment bookkeeping, _decode_asr stitching and
the full TurboTranscriber.__call__ flow with the oracle standing in for the GPU engine."""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as hs

from oracle import whisper_oracle as wo
from twamd import audio
from twamd.config import PRESETS, GenerationSettings, SpecialTokens
from twamd.frontend import chunk_windows, dft_basis, mel_filterbank, mel_table, pack_k8
from twamd.pipeline import TurboTranscriber
from twamd.segments import retrieve_segment, strip_generated
from twamd.synth_audio import speech_like, white_noise
from twamd.tokenizer import WhisperVocab, decode_asr

G = os.path.join(os.path.dirname(__file__), "golden")


def test_special_token_layouts():
    for v, tb in ((51866, 50365), (51865, 50364), (51864, 50363)):
        st = SpecialTokens.for_vocab(v)
        assert st.timestamp_begin == tb and st.timestamp_begin + 1501 == v
    st = SpecialTokens.for_vocab(51866)
    assert st.lang_to_id()["<|en|>"] == 50259 and st.lang_to_id()["<|yue|>"] == 50358
    assert (st.translate, st.transcribe, st.notimestamps) == (50359, 50360, 50364)


def test_decode_asr_matches_transformers():
    cases = json.load(open(os.path.join(G, "decode_asr.json")))
    vocab = WhisperVocab.synthetic(SpecialTokens.for_vocab(51866))
    for c in cases:
        outs = [{"tokens": o["tokens"], "stride": tuple(o["stride"])} for o in c["outputs"]]
        text, opt = decode_asr(vocab, outs, return_timestamps=c["return_timestamps"],
                               return_language=c["return_language"])
        assert text == c["text"]
        got = json.loads(json.dumps(opt))
        assert got == c["optional"]


@given(n=hs.integers(0, 3_000_000), chunk=hs.sampled_from([30, 60, 10.5]), stride=hs.sampled_from([0, 5, 2.5, None]))
@settings(max_examples=200, deadline=None)
def test_chunk_windows_match_chunk_iter(n, chunk, stride):
    from transformers.pipelines.automatic_speech_recognition import chunk_iter

    class FE:  # records chunk lengths instead of featurising
        sampling_rate = 16000

        def __call__(self, chunk, **kw):
            class R(dict):
                def to(self, dtype):
                    return self
            return R(n=len(chunk))

    sl = chunk / 6 if stride is None else stride
    cl, st_ = int(round(chunk * 16000)), int(round(sl * 16000))
    if cl < 2 * st_:
        return
    ref = [(it["stride"], it["is_last"]) for it in chunk_iter(np.zeros(n, np.float32), FE(), cl, st_, st_)]
    got = [((w.length, w.stride_left, w.stride_right), w.is_last)
           for w in chunk_windows(n, chunk, stride)]
    assert got == ref


@given(seq=hs.lists(hs.sampled_from([5, 6, 7, 100, 101, 150, 50257]), max_size=30))
@settings(max_examples=300, deadline=None)
def test_retrieve_segment_matches_oracle(seq):
    seq = strip_generated(seq, 50257)
    a = retrieve_segment(seq, 0, 3000, 100)
    b = wo.retrieve_segment(seq, 3000, 100)
    assert a == b
    assert a[0] == list(seq[: len(a[0])])


def test_strip_generated():
    assert strip_generated([1, 2, 50257, 50257, 50257], 50257) == [1, 2]
    assert strip_generated([1, 2, 50257], 50257) == [1, 2]
    assert strip_generated([1, 2], 50257) == [1, 2]


def test_frontend_tables():
    fb = mel_filterbank(128)
    from transformers.audio_utils import mel_filter_bank

    ref = mel_filter_bank(201, 128, 0.0, 8000.0, 16000, norm="slaney", mel_scale="slaney")
    np.testing.assert_allclose(fb, ref, rtol=1e-12, atol=1e-15)
    c, s = dft_basis()
    assert c.shape == (400, 224) and not c[:, 201:].any() and not s[:, 201:].any()
    t = mel_table(80)
    assert t.shape == (224, 96) and not t[201:].any() and not t[:, 80:].any()


def test_pack_k8_index_formula():
    """tw_logmel's "k8" operand order (include/tw_whisper.h): [k][c] at ((k/8 * C + c) * 2 + k%2) * 4 + (k%8)/2."""
    a = np.arange(400 * 224, dtype=np.float32).reshape(400, 224)
    p = pack_k8(a).ravel()
    k, c = np.meshgrid(np.arange(400), np.arange(224), indexing="ij")
    idx = ((k // 8 * 224 + c) * 2 + k % 2) * 4 + (k % 8) // 2
    assert np.array_equal(p[idx], a)


def test_wav_roundtrip(tmp_path):
    x = speech_like(1.5, 3)
    p = str(tmp_path / "a.wav")
    audio.write_wav(p, x)
    y = audio.load_input(p)
    np.testing.assert_allclose(y, x, atol=1.0 / 32767)
    y2 = audio.load_input({"array": x, "sampling_rate": 16000})
    np.testing.assert_array_equal(y2, x)
    y3 = audio.load_input({"raw": np.stack([x, x]), "sampling_rate": 16000})  # channels-first -> mean
    np.testing.assert_allclose(y3, x, atol=1e-7)


class _OracleTranscriber(TurboTranscriber):
    """TurboTranscriber whose per-window model work is the fp32 oracle (CPU test of the host flow)."""

    def __init__(self, dims):
        gen = GenerationSettings.default(dims)
        self.gen = gen
        self.vocab = WhisperVocab.synthetic(gen.special)
        self.sampling_rate = 16000
        st = gen.special
        self.g = wo.GenCfg(dims.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                           st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)
        sd = wo.synth_state_dict(dims.d_model, dims.encoder_layers, dims.decoder_layers, dims.ffn, dims.n_mels,
                                 dims.vocab, 1234)
        self.m = wo.WhisperOracle(sd, dims.heads)
        self.n_mels = dims.n_mels

        class _E:
            class d:
                max_source_positions = 1500
        self.engine = _E()

    def transcribe_windows(self, wav, windows, task, lang_id, return_timestamps, max_new_tokens=None, num_beams=1,
                           word_timestamps=False, num_frames=None, group=None, max_passes=None):
        if word_timestamps:  # batches of `group` windows: the product passes the pipeline's batch_size
            out, self.last_window_token_timestamps = [], []
            B = group or 1
            heads = getattr(self, "alignment_heads", None) or self.gen.alignment_heads
            for b0 in range(0, len(windows), B):
                feats = [wo.log_mel(wav[w.start: w.start + min(w.length, 480000)], self.n_mels)
                         for w in windows[b0: b0 + B]]
                for toks, _, tts in wo.generate_batch_word(self.m, feats, self.g, heads, num_frames[b0: b0 + B],
                                                           task=task, language=lang_id,
                                                           max_new_tokens=max_new_tokens):
                    out.append(toks)
                    self.last_window_token_timestamps.append(tts)
            return out
        out = []
        for w in windows:
            f = wo.log_mel(wav[w.start: w.start + min(w.length, 480000)], self.n_mels)
            toks, _ = wo.generate(self.m, f, self.g, task=task, language=lang_id,
                                  return_timestamps=return_timestamps, max_new_tokens=max_new_tokens,
                                  num_beams=num_beams)
            out.append(toks)
        return out


@pytest.mark.slow
def test_pipeline_host_flow_matches_transformers_pipeline():
    gold = json.load(open(os.path.join(G, "pipeline.json")))
    tr = _OracleTranscriber(PRESETS["test-mini"])
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    for case in gold["cases"]:
        xx = x if case["name"] != "short_nochunk" else x[: 20 * 16000]
        r = tr(xx, generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40},
               return_timestamps=True, **case["kwargs"])
        assert json.loads(json.dumps(r)) == case["output"], case["name"]


@pytest.mark.slow
def test_pipeline_word_timestamps_host_flow_matches_transformers():
    """return_timestamps="word" through the host flow (num_frames per window, per-token times, LCS merge with
    times, word collation) with the batched oracle as the model: equals the transformers ASR pipeline output."""
    gold = json.load(open(os.path.join(G, "word.json")))
    tr = _OracleTranscriber(PRESETS["test-mini"])
    tr.alignment_heads = [tuple(h) for h in gold["alignment_heads"]]
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    for case in gold["cases"]:
        r = tr(x[: case["n_samples"]], generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40},
               return_timestamps="word", **case["kwargs"])
        assert json.loads(json.dumps(r)) == case["output"], case["name"]


# ---- temperature fallback criteria (generation_whisper.py:1243-1287) vs transformers' own values --------------------
def _fallback_golden():
    import json

    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fallback.json")))


def test_fallback_compression_ratio_and_decisions_match_transformers():
    """twamd.segments: _retrieve_compression_ratio exactly, and _need_fallback's decisions (incl. the no-speech skip)
    from transformers' own criteria values, for every seek pass of the spied generate() runs."""
    from twamd.segments import FallbackConfig, compression_ratio, need_fallback

    z = _fallback_golden()
    for name in ("metrics", "skip"):
        kw = z[name]["kwargs"]
        cfg = FallbackConfig(temperatures=tuple(kw["temperature"]),
                             compression_ratio_threshold=kw["compression_ratio_threshold"],
                             logprob_threshold=kw["logprob_threshold"], no_speech_threshold=kw["no_speech_threshold"])
        for c in z[name]["calls"]:
            assert compression_ratio(c["tokens"], 51866) == c["compression_ratio"]
            got = need_fallback(c["tokens"], c["avg_logprob"] * len(c["tokens"]), c["no_speech_prob"], 51866, cfg)
            assert got == (c["needs_fallback"], c["should_skip"]), (name, c["index"])


def test_fallback_sequence_cut():
    from twamd.segments import fallback_sequence

    assert fallback_sequence([5, 6, 50257, 50257, 50257], 50257, 50257) == [5, 6, 50257]
    assert fallback_sequence([5, 6, 7], 50257, 50257) == [5, 6, 7]
    assert fallback_sequence([5, 6, 50257], 50257, 50257) == [5, 6, 50257]
    assert fallback_sequence([5, 0, 0], 0, 50257) == [5]


def test_lcs_vectorised_scan_equals_sequential_scan():
    """find_longest_common_sequence's diagonal-sum form (no token timestamps) picks the same overlap as the
    sequential scan of tokenization_whisper.py:1153-1270 (restated here) on random and planted-overlap runs."""
    from twamd.tokenizer import find_longest_common_sequence

    def scan(sequences):
        left, total = sequences[0], []
        for right in sequences[1:]:
            L, R = len(left), len(right)
            best, idx = 0.0, (L, L, 0, 0)
            for i in range(1, L + R):
                ls, le, rs, re_ = max(0, L - i), min(L, L + R - i), max(0, i - L), min(R, i)
                m = sum(1 for k in range(le - ls) if left[ls + k] == right[rs + k])
                if m > 1 and m / i + i / 10000.0 > best:
                    best, idx = m / i + i / 10000.0, (ls, le, rs, re_)
            ls, le, rs, re_ = idx
            total.extend(left[:(le + ls) // 2])
            left = right[(re_ + rs) // 2:]
        return total + list(left)

    rng = np.random.default_rng(11)
    for _ in range(1500):
        V = int(rng.choice([2, 4, 16, 50000]))
        seqs = [[int(x) for x in rng.integers(0, V, rng.integers(0, 40))] for _ in range(int(rng.integers(2, 5)))]
        if len(seqs[0]) > 4 and rng.random() < 0.5:
            seqs[1] = seqs[0][-int(rng.integers(1, len(seqs[0]))):] + seqs[1]
        assert find_longest_common_sequence(seqs) == scan(seqs), seqs


def _sharded_stitch(vocab, outs, n_shards, **kw):
    """twamd.dist.stitch_sharded without a process group: every shard's piece computed here, then the merge."""
    from twamd import dist as twd
    bounds = [twd.shard_range(len(outs), n_shards, r) for r in range(n_shards)]
    pieces = [twd.shard_piece(vocab, outs, lo, hi, **kw) for lo, hi in bounds]
    return twd.merge_pieces(vocab, outs, pieces, bounds, **kw)


def test_sharded_stitching_equals_decode_asr_on_transformers_cases():
    """_decode_asr split over ranks (each stitches its window shard from the state it expects, the
    pieces merged) equals the serial stitching — and so transformers — on every decode_asr.json case, every shard
    count."""
    cases = json.load(open(os.path.join(G, "decode_asr.json")))
    vocab = WhisperVocab.synthetic(SpecialTokens.for_vocab(51866))
    for c in cases:
        outs = [{"tokens": o["tokens"], "stride": tuple(o["stride"])} for o in c["outputs"]]
        kw = dict(return_timestamps=c["return_timestamps"], return_language=c["return_language"])
        for n in range(1, len(outs) + 2):
            text, opt = _sharded_stitch(vocab, outs, n, **kw)
            assert text == c["text"]
            assert json.loads(json.dumps(opt)) == c["optional"]


@given(data=hs.data())
@settings(max_examples=300, deadline=None)
def test_sharded_stitching_equals_serial_random_windows(data):
    """Random window token streams (text, timestamps in and out of order, open segments across windows, language
    switches, strides) and random shard counts: the merged pieces equal the serial decode_asr."""
    st = SpecialTokens.for_vocab(51866)
    vocab = WhisperVocab.synthetic(st)
    langs = [st.lang_begin, st.lang_begin + 1, st.lang_begin + 7]
    n_win = data.draw(hs.integers(1, 9))
    stride = data.draw(hs.sampled_from([(30.0, 0.0, 0.0), (30.0, 5.0, 5.0), (20.0, 2.5, 0.0)]))
    outs = []
    for w in range(n_win):
        toks = []
        if data.draw(hs.booleans()):
            toks += [st.sot, data.draw(hs.sampled_from(langs)), st.transcribe]
        for _ in range(data.draw(hs.integers(0, 10))):
            kind = data.draw(hs.integers(0, 2))
            if kind == 0:
                toks.append(data.draw(hs.integers(200, 240)))  # text (repeats: LCS overlaps)
            elif kind == 1:
                toks.append(st.timestamp_begin + data.draw(hs.integers(0, 1500)))
            else:
                toks.append(data.draw(hs.sampled_from(langs)))
        left = 0.0 if w == 0 else stride[1]
        right = 0.0 if w == n_win - 1 else stride[2]
        tts = sorted(data.draw(hs.lists(hs.floats(0, 30, allow_nan=False), min_size=len(toks), max_size=len(toks))))
        outs.append({"tokens": toks, "stride": (stride[0], left, right), "token_timestamps": tts})
    rt = data.draw(hs.sampled_from([True, False, "word"]))
    rl = data.draw(hs.booleans())
    want = decode_asr(vocab, outs, return_timestamps=rt, return_language=rl)
    for n in range(1, n_win + 1):
        assert _sharded_stitch(vocab, outs, n, return_timestamps=rt, return_language=rl) == want
