"""The production load path: a LOCAL Hugging Face Whisper checkpoint directory (config.json, generation_config.json,
model.safetensors, vocab.json / merges.txt / added_tokens.json) -> GenerationSettings, WhisperVocab, the safetensors
loader and TurboTranscriber.from_pretrained(checkpoint=...); and the decode the boundary runs by default.

References: load_transcription_model builds `transformers.pipeline("automatic-speech-recognition", model=name)`
(/root/reference/vocalis/core/audio_pipeline.py:195-200) and calls it with generate_kwargs={"task": task} only
(:351-358); the pipeline's decode defaults come from $TF/pipelines/automatic_speech_recognition.py:160-163 and
$TF/pipelines/base.py:887-908 (pinned here by tests/golden/defaults.json, which transformers itself produced).
The checkpoint is written by tests/ckpt_util.py from the seeded synthetic weights (no real checkpoints offline)."""
import json
import os

import numpy as np
import pytest

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings

import ckpt_util as cu

G = os.path.join(os.path.dirname(__file__), "golden")
D = PRESETS["test-mini"]


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    return cu.write_checkpoint(str(tmp_path_factory.mktemp("ckpt")), generation={"num_beams": 3})


def test_resolve_decode_matches_transformers_pipeline():
    """The boundary's default decode is what the HF ASR pipeline resolves: beam-5 whatever the checkpoint's
    generation_config.json says, max_length-bounded unless max_length is unset (then max_new_tokens=256)."""
    from twamd.pipeline import resolve_decode

    gold = json.load(open(os.path.join(G, "defaults.json")))
    assert len(gold["cases"]) == 15
    for c in gold["cases"]:
        gs = GenerationSettings.default(D)
        cfg = c["checkpoint_generation_config"]
        if "num_beams" in cfg:
            gs.num_beams = cfg["num_beams"]
        if "max_length" in cfg and cfg["max_length"] is None:
            gs.max_length_set = False
        got = resolve_decode(gs, dict(c["generate_kwargs"]))
        want = c["resolved"]
        assert got == {"num_beams": want["num_beams"], "max_new_tokens": want["max_new_tokens"]}, c


def test_generation_settings_from_checkpoint(ckpt):
    gs = GenerationSettings.from_checkpoint(ckpt, D)
    ref = GenerationSettings.default(D)
    assert gs.num_beams == 3 and gs.max_length == 448 and gs.max_length_set
    assert gs.suppress_tokens == ref.suppress_tokens
    assert gs.begin_suppress_tokens == ref.begin_suppress_tokens
    assert gs.max_initial_timestamp_index == 50
    assert gs.alignment_heads == ref.alignment_heads
    assert gs.median_filter_width == 7


def test_generation_settings_without_max_length(tmp_path):
    d = str(tmp_path)
    with open(os.path.join(d, "generation_config.json"), "w") as f:
        json.dump({"suppress_tokens": [1, 2], "begin_suppress_tokens": [220]}, f)
    gs = GenerationSettings.from_checkpoint(d, D)
    assert not gs.max_length_set and gs.num_beams == 1 and gs.suppress_tokens == [1, 2]
    from twamd.pipeline import resolve_decode

    assert resolve_decode(gs, {"task": "transcribe"}) == {"num_beams": 5, "max_new_tokens": 256}


def test_dims_from_checkpoint(ckpt):
    from twamd.pipeline import _dims_from_checkpoint

    d = _dims_from_checkpoint(ckpt)
    assert (d.d_model, d.encoder_layers, d.decoder_layers, d.heads, d.ffn, d.n_mels, d.vocab,
            d.max_source_positions, d.max_target_positions) == \
        (D.d_model, D.encoder_layers, D.decoder_layers, D.heads, D.ffn, D.n_mels, D.vocab, 1500, 448)


def test_vocab_from_checkpoint_decodes_like_transformers(ckpt):
    """WhisperVocab.from_checkpoint(dir).decode equals transformers' WhisperTokenizer.from_pretrained(dir).decode
    (tests/golden/ckpt_decode.json): multi-byte UTF-8 tokens, UTF-8 sequences split across byte tokens, invalid
    byte runs (U+FFFD)."""
    from twamd.tokenizer import WhisperVocab

    gold = json.load(open(os.path.join(G, "ckpt_decode.json"), encoding="utf-8"))
    st = GenerationSettings.default(D).special
    v = WhisperVocab.from_checkpoint(ckpt, st)
    assert gold["vocab_size"] == st.vocab and gold["all_special_ids"] == st.special_ids()
    lay = gold["layout"]
    assert (lay["<|endoftext|>"], lay["<|startoftranscript|>"], lay["<|en|>"], lay["<|transcribe|>"],
            lay["<|notimestamps|>"], lay["<|0.00|>"], lay["<|30.00|>"]) == \
        (st.eot, st.sot, st.lang_begin, st.transcribe, st.notimestamps, st.timestamp_begin, st.vocab - 1)
    for c in gold["cases"]:
        assert v.decode(c["ids"]) == c["text"], c
    # the checkpoint's vocabulary, not the preset's, was loaded
    assert v.decode([cu.MB_BASE]) == cu.MULTIBYTE_WORDS[0]
    assert WhisperVocab.synthetic(st).decode([cu.MB_BASE]) != cu.MULTIBYTE_WORDS[0]


@pytest.mark.parametrize("dtype", [np.float32, np.float16], ids=["f32", "f16"])
def test_safetensors_loader_maps_every_parameter(tmp_path, dtype):
    """load_checkpoint_state_dict reads every parameter the engine packs, by HF name and shape, into bf16
    matrices / f32 vectors; with an f32 checkpoint of bf16-exact values the result is the seeded parameter
    bit for bit."""
    import torch

    from twamd.weights import load_checkpoint_state_dict, param_shapes

    d = cu.write_checkpoint(str(tmp_path), dtype=dtype)
    sd = load_checkpoint_state_dict(d, D, device="cpu")
    ref = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    names = [n for n, _ in param_shapes(D)]
    assert sorted(sd) == sorted(names)
    for n, shape in param_shapes(D):
        t = sd[n]
        assert tuple(t.shape) == shape
        assert t.dtype == (torch.float32 if len(shape) == 1 else torch.bfloat16)
        r = ref[n].astype(dtype).astype(np.float32)
        got = t.float().numpy()
        if dtype == np.float32:
            assert np.array_equal(got, ref[n]), n
        else:  # f16 storage then bf16: within one bf16 ulp of the f16 value
            assert np.allclose(got, r, rtol=2 ** -8, atol=1e-7), n


def test_loader_rejects_missing_and_misshaped(tmp_path):
    from safetensors.numpy import save_file

    from twamd.weights import load_checkpoint_state_dict

    with pytest.raises(FileNotFoundError):
        load_checkpoint_state_dict(str(tmp_path), D, device="cpu")
    save_file({"model.encoder.conv1.weight": np.zeros((D.d_model, D.n_mels, 3), np.float32)},
              os.path.join(str(tmp_path), "model.safetensors"))
    with pytest.raises(KeyError, match="lacks"):
        load_checkpoint_state_dict(str(tmp_path), D, device="cpu")
    save_file({"model.encoder.conv1.weight": np.zeros((D.d_model, D.n_mels, 5), np.float32)},
              os.path.join(str(tmp_path), "model.safetensors"))
    with pytest.raises(ValueError, match="shape"):
        load_checkpoint_state_dict(str(tmp_path), D, device="cpu")


@pytest.mark.gpu
def test_checkpoint_transcriber_equals_preset(ckpt):
    """TurboTranscriber.from_pretrained(checkpoint=dir) runs the same kernels on the same weights as the seeded
    preset: identical tokens for greedy generate() and for the callable's default (beam-5) decode; its texts come
    from the checkpoint's vocabulary."""
    import torch

    from twamd.pipeline import TurboTranscriber
    from twamd.synth_audio import speech_like, white_noise
    from twamd.tokenizer import WhisperVocab

    a = TurboTranscriber.from_pretrained(checkpoint=ckpt, max_batch=2)
    assert a.gen.num_beams == 3
    host = np.zeros((2, 480000), np.float32)
    host[0] = speech_like(30.0, 1234)
    n = white_noise(12.3, 7)
    host[1, : len(n)] = n

    def run(tr):
        tr.engine.wave[:2].copy_(torch.from_numpy(host))
        tr.engine.logmel(2)
        g = tr.engine.generate(2, task="transcribe", max_new_tokens=40, return_timestamps=True)
        out = tr(np.concatenate([host[0], host[1][:16000 * 12]]), chunk_length_s=30, stride_length_s=0,
                 generate_kwargs={"task": "transcribe", "max_new_tokens": 24}, return_timestamps=True)
        return g, out, [t for w in tr.last_window_passes for p in w for t in p]

    ga, oa, pa = run(a)
    del a
    torch.cuda.empty_cache()
    b = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=2)
    gb, ob, pb = run(b)
    gold = np.load(os.path.join(G, "model.npz"))
    for i in range(2):
        ref = [int(t) for t in gold["gen_sequences"][i]]
        while ref and ref[-1] == 50257:
            ref.pop()
        assert ga[i] == ref
    assert ga == gb and pa == pb
    assert [c["timestamp"] for c in oa["chunks"]] == [c["timestamp"] for c in ob["chunks"]]
    st = GenerationSettings.default(D).special
    if any(cu.MB_BASE <= t < cu.MB_BASE + len(cu.MULTIBYTE_WORDS) for t in pa):
        assert oa["text"] != ob["text"]  # decoded with the checkpoint's vocabulary
    assert isinstance(WhisperVocab.from_checkpoint(ckpt, st).decode([t for t in pa if t < st.eot]), str)
    del b
