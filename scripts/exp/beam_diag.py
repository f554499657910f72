"""Diagnostic (not product code): sweep case nochunk_beam5 (25 s, no chunking, beam 5): device first pass vs the fp32
oracle's beam search, with per-position fp32 log-probs of both hypotheses."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

from make_golden import sweep_audio  # noqa: E402
from oracle import whisper_oracle as wo  # noqa: E402
from twamd.config import PRESETS, GenerationSettings  # noqa: E402
from twamd.pipeline import TurboTranscriber  # noqa: E402

D = PRESETS["test-mini"]
gen = GenerationSettings.default(D)
st = gen.special
g = wo.GenCfg(D.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate, st.notimestamps,
              gen.suppress_tokens, gen.begin_suppress_tokens)
orc = wo.WhisperOracle(wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab,
                                           1234), D.heads)
audio = sweep_audio([("speech", 25.0, 36)])
tr = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=8, max_beams=5)
r = tr(audio, generate_kwargs={"task": "transcribe", "num_beams": 5, "max_new_tokens": 24}, return_timestamps=True)
feats = wo.log_mel(audio[:480000], D.n_mels)
enc = orc.encode(feats)
lang = tr.last_window_langs[0]
prompt = [st.sot, lang, st.transcribe]
ora = wo.beam_pass(orc, enc, prompt, 24, g, True, 5)
dev = [int(x) for x in tr.last_window_passes[0][0]]
print("lang", lang, "oracle lang", wo.detect_language(orc, enc, g))
print("oracle", ora)
print("device", dev)
fs = tr.engine._beam_buffers(5)["fin_score"][:5].cpu().numpy()
print("device fin scores", fs)


def lps(toks):
    cache = orc.new_cache(enc)
    for t in prompt[:-1]:
        orc.decoder_step(t, cache)
    lg = orc.decoder_step(prompt[-1], cache)
    out, hist = [], []
    for t in toks:
        out.append(float(wo.process_logits(wo._log_softmax32(lg), hist, g, True)[t]))
        hist.append(t)
        lg = orc.decoder_step(t, cache)
    return out


a, b = lps(ora), lps(dev)
print("fp32 oracle hyp avg", sum(a) / len(a), "device hyp avg", sum(b) / len(b))
for i, (x, y) in enumerate(zip(a, b)):
    print(i, ora[i] if i < len(ora) else None, round(x, 3), dev[i] if i < len(dev) else None, round(y, 3))

# device teacher-forced processed log-probs of the device hypothesis (one row, window re-encoded at seek 0)
import torch  # noqa: E402

eng = tr.engine
host = np.zeros((1, 480000), np.float32)
host[0, : len(audio)] = audio[:480000]
eng.wave[:1].copy_(torch.from_numpy(host))
eng.logmel(1)
eng.row_map[0] = 0
eng.seek[0] = 0
eng.encode(1)
full = prompt + dev
dl = []
for pos in range(len(full) - 1):
    eng.ids[0] = full[pos]
    eng.pos[0] = pos
    eng.decoder_step(1)
    lg = eng.logits[0].cpu().numpy()
    j = pos + 1 - len(prompt)
    if j >= 0:
        dl.append(float(wo.process_logits(wo._log_softmax32(lg), dev[:j], g, True)[dev[j]]))
print("device teacher-forced avg", sum(dl) / len(dl))
for i, (x, y) in enumerate(zip(b, dl)):
    print(i, dev[i], "fp32", round(x, 3), "device", round(y, 3))
