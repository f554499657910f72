"""Diagnostic (not product code): where does the engine's beam-5 translate decode of tests/golden/options.json's
audio leave the oracle's fp32 beam search (pinned to transformers)? Per 60/5 window: device vs oracle final tokens."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import whisper_oracle as wo  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.frontend import chunk_windows  # noqa: E402
from twamd.pipeline import TurboTranscriber  # noqa: E402
from twamd.synth_audio import speech_like, white_noise  # noqa: E402

D = PRESETS["test-mini"]
gen = GenerationSettings.default(D)
st = gen.special
g = wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate, st.notimestamps,
              gen.suppress_tokens, gen.begin_suppress_tokens)
sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
orc = wo.WhisperOracle(sd, D.heads)
audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
tr = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=4, max_beams=5)
r = tr(audio, generate_kwargs={"task": "translate", "max_new_tokens": 24}, return_timestamps=True,
       chunk_length_s=60, stride_length_s=5, batch_size=32)
wins = list(chunk_windows(len(audio), 60, 5, 16000))
for k, w in enumerate(wins):
    seg = audio[w.start: w.start + min(w.length, 480000)]
    feats = wo.log_mel(seg, D.n_mels)
    otoks, olang = wo.generate(orc, feats, g, task="translate", max_new_tokens=24, num_beams=5)
    dev = tr.last_window_passes[k]
    print(f"window {k}: lang device {tr.last_window_langs[k]} oracle {olang}")
    print("  oracle final:", list(otoks))
    print("  device passes:", [list(p) for p in dev])
