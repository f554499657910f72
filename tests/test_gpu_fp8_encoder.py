"""BASELINE config 5 end to end: the MX fp8 encoder (tw_layernorm_mx / tw_gemm_mx / tw_quant_mx) + the bf16
decoder, test-mini dims with seeded weights, against the oracle's encode_mx (the same MX quantisation points in
float32/float64 numpy) and, for the tokens, replay_generate(mx=True).

Tolerances: the GPU keeps q/k/v and the attention output in bf16 and accumulates in f32, so an MX element may
round to the neighbouring e4m3 value where numpy's is a near-tie (one e4m3 step is 12.5 % of the element): encoder
output |diff| <= 0.3 abs, mean <= 0.04 (LayerNorm-scale outputs, mean |x| ~0.8; measured 0.19 / 0.026 — about half
the oracle's own MX-vs-fp32 distance, 0.35 / 0.052, so the two MX realisations share most of their quantisation). Against the fp32 encoder (what fp8 costs):
mean |diff| <= 0.1. Greedy decisions: within TAU = 0.3 logits of the reference's choice (as the bf16 pipeline
test)."""
import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, white_noise

pytestmark = pytest.mark.gpu
D = PRESETS["test-mini"]


@pytest.fixture(scope="module")
def tr8():
    return TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=4, enc_fp8=True)


@pytest.fixture(scope="module")
def oracle():
    sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    return wo.WhisperOracle(sd, D.heads)


def _gcfg():
    gen = GenerationSettings.default(D)
    st = gen.special
    return wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                     st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def _load(tr, clips):
    eng = tr.engine
    host = np.zeros((len(clips), 480000), np.float32)
    for i, c in enumerate(clips):
        host[i, : min(len(c), 480000)] = c[:480000]
    eng.wave[: len(clips)].copy_(torch.from_numpy(host))
    eng.logmel(len(clips))


def test_fp8_encoder_vs_oracle_mx(tr8, oracle):
    eng = tr8.engine
    assert eng.enc_fp8 and len(eng.enc_mx) == D.encoder_layers
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7)]
    _load(tr8, clips)
    R = 2
    eng.row_map[:R] = torch.arange(R, dtype=torch.int32)
    eng.seek[:R] = 0
    eng.encode(R)
    enc = eng.encoder_output(R).float().cpu().numpy()
    for i, c in enumerate(clips):
        feats = wo.log_mel(c, D.n_mels)
        d = np.abs(enc[i] - oracle.encode_mx(feats))
        print(f"clip {i}: vs encode_mx max {d.max():.4f} mean {d.mean():.5f}")
        assert d.max() < 0.3 and d.mean() < 0.04, (i, d.max(), d.mean())
        d32 = np.abs(enc[i] - oracle.encode(feats))
        print(f"clip {i}: vs fp32 encode max {d32.max():.4f} mean {d32.mean():.5f}")
        assert d32.mean() < 0.1, (i, d32.mean())


def test_fp8_transcript_decisions_within_tau(tr8, oracle):
    TAU = 0.3
    x = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    r = tr8(x, chunk_length_s=30, stride_length_s=0,
            generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 40}, return_timestamps=True)
    assert "text" in r and "chunks" in r
    g = _gcfg()
    segs = [x[k * 480000: (k + 1) * 480000] for k in range((len(x) + 479999) // 480000)]
    assert len(segs) == len(tr8.last_window_passes)
    for k, seg in enumerate(segs):
        st = wo.replay_generate(oracle, wo.log_mel(seg, D.n_mels), g, tr8.last_window_passes[k],
                                tr8.last_window_langs[k], max_new_tokens=40, tau=TAU, mx=True)
        print(k, st)
        assert st["ok"], (k, st)
