"""BASELINE.json configs beyond the bench line, through the product path on the MI355X:

  configs[0]  whisper-tiny.en (English-only vocabulary 51864, 80 mels, d 384): no language detection, no task token;
              teacher-forced logits vs the f32 oracle and the greedy decode replayed through the oracle within tau
  configs[2]  chunk-sharded transcription across ranks: two ranks (gloo) share this box's one GPU, each runs its own
              engine on its shard of the windows, one all-gather reassembles; the transcript must equal the
              single-process transcript exactly (same kernels, same inputs per window)

Weights are the seeded synthetic ones (no checkpoints offline); the oracle restates the transformers path and is
pinned by tests/test_oracle_golden.py."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd.config import PRESETS, GenerationSettings
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, white_noise

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcfg(dims):
    gen = GenerationSettings.default(dims)
    st = gen.special
    return wo.GenCfg(dims.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                     st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens,
                     multilingual=st.is_multilingual)


@pytest.fixture(scope="module")
def tiny():
    d = PRESETS["tiny.en"]
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=2)
    sd = wo.synth_state_dict(d.d_model, d.encoder_layers, d.decoder_layers, d.ffn, d.n_mels, d.vocab, 1234)
    return tr, wo.WhisperOracle(sd, d.heads), d


def test_tiny_en_special_tokens(tiny):
    tr, _, d = tiny
    st = tr.gen.special
    assert (st.eot, st.sot, st.notimestamps, st.timestamp_begin, st.is_multilingual) == (50256, 50257, 50362, 50363,
                                                                                            False)
    with pytest.raises(ValueError, match="English-only"):
        tr(np.zeros(16000, np.float32), generate_kwargs={"task": "transcribe"})


def test_tiny_en_teacher_forced_logits(tiny):
    tr, oracle, d = tiny
    eng = tr.engine
    clip = speech_like(30.0, 4321)
    eng.wave[:1].copy_(torch.from_numpy(clip[None, :480000]))
    eng.logmel(1)
    eng.row_map[0] = 0
    eng.seek[0] = 0
    eng.encode(1)
    enc_ref = oracle.encode(wo.log_mel(clip, d.n_mels))
    enc = eng.encoder_output(1)[0].float().cpu().numpy()
    assert np.abs(enc - enc_ref).max() < 0.08
    cache = oracle.new_cache(enc_ref)
    st = tr.gen.special
    ids = [st.sot, st.timestamp_begin, 1000, 2000, 3000, st.timestamp_begin + 20, 400, 500]
    for t, tok in enumerate(ids):
        eng.ids[0] = tok
        eng.pos[0] = t
        eng.decoder_step(1)
        got = eng.logits[0].cpu().numpy()
        ref = oracle.decoder_step(tok, cache)
        assert np.abs(got - ref).max() < 0.15, (t, np.abs(got - ref).max())


@pytest.fixture(scope="module")
def tiny_z():
    return np.load(os.path.join(ROOT, "tests", "golden", "tiny.npz"))


def test_tiny_en_vs_transformers_goldens(tiny, tiny_z):
    """The engine at tiny.en against transformers fp32 itself (tests/golden/tiny.npz, make_golden.py tiny): encoder
    rows (0.08 abs, as test-mini), the 16 fp32-top teacher-forced logits and their log-sum-exp (0.15 abs), and
    generate() (English-only prompt, seek loop, 48 new tokens) pass by pass: equal, or diverging first at a near-tie
    within tau = 0.3 (the tolerance of the oracle replay above)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import turbo_parity as tp

    tr, _, d = tiny
    z = tiny_z
    eng = tr.engine
    clips = [speech_like(30.0, 1234), white_noise(12.3, 7)]
    host = np.zeros((2, 480000), np.float32)
    for i, c in enumerate(clips):
        host[i, : len(c)] = c[:480000]
    eng.wave[:2].copy_(torch.from_numpy(host))
    eng.logmel(2)
    eng.row_map[:2] = torch.arange(2, dtype=torch.int32)
    eng.seek[:2] = 0
    eng.encode(2)
    enc = eng.encoder_output(2).float().cpu().numpy()
    for i in range(2):
        assert np.abs(enc[i][z["enc_rows_idx"]] - z["enc_rows"][i]).max() < 0.08
        assert abs(enc[i].mean() - z["enc_mean"][i]) < 2e-3 and abs(enc[i].std() - z["enc_std"][i]) < 2e-3
    for t, tok in enumerate(z["tf_input_ids"]):
        eng.ids[0] = int(tok)
        eng.pos[0] = t
        eng.decoder_step(1, r_enc=2)  # (cross K/V encoded with batch stride 2)
        lg = eng.logits[0].cpu().numpy().astype(np.float64)
        m = lg.max()
        assert np.abs(lg[z["tf_top_idx"][t]] - z["tf_top_val"][t]).max() < 0.15, t
        assert abs(m + np.log(np.exp(lg - m).sum()) - z["tf_lse"][t]) < 0.15, t
    eng.logmel(2)
    seqs = eng.generate(2, task=None, max_new_tokens=48, return_timestamps=True)
    st = tr.gen.special
    for i in range(2):
        ref = [int(x) for x in z["gen_sequences"][i]]
        while ref and ref[-1] == st.eot:
            ref.pop()
        if seqs[i] == ref:
            continue
        lens, o = z[f"gen{i}_pass_len"], 0
        for k, n in enumerate(lens):
            dev = [int(x) for x in eng.last_passes[i][k]] if k < len(eng.last_passes[i]) else []
            dev = dev[: dev.index(st.eot) + 1] if st.eot in dev else dev
            r = tp.check_pass(dev, z[f"gen{i}_pass_tokens"][o: o + n], z[f"gen{i}_top_idx"][o: o + n],
                              z[f"gen{i}_top_val"][o: o + n], z[f"gen{i}_ts_margin"][o: o + n], tau=0.3,
                              ts_begin=st.timestamp_begin)
            o += n
            if r["status"] != "exact":
                assert r["status"] == "within_tau", (i, k, r)
                break


def test_tiny_en_generate_is_tolerance_greedy(tiny):
    tr, oracle, d = tiny
    eng = tr.engine
    clips = [speech_like(30.0, 11), white_noise(17.0, 12)]
    host = np.zeros((2, 480000), np.float32)
    for i, c in enumerate(clips):
        host[i, : len(c)] = c[:480000]
    eng.wave[:2].copy_(torch.from_numpy(host))
    eng.logmel(2)
    eng.generate(2, task=None, max_new_tokens=48, return_timestamps=True)
    g = _gcfg(d)
    for i in range(2):
        st = wo.replay_generate(oracle, wo.log_mel(host[i], d.n_mels), g, eng.last_passes[i], None, task=None,
                                max_new_tokens=48, tau=0.3)
        assert st["ok"], (i, st)
        assert st["exact"] >= 0.8 * st["decisions"], st


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, q):
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from twamd.pipeline import TurboTranscriber as TT
        from twamd.synth_audio import speech_like as sl

        tr = TT.from_pretrained("test-mini", seed=1234, max_batch=2)
        x = sl(160.0, 77) if rank == 0 else None
        out = tr(x, chunk_length_s=30, stride_length_s=0, generate_kwargs={"task": "transcribe", "max_new_tokens": 24},
                 return_timestamps=True)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_transcript_equals_single_process():
    import torch.multiprocessing as mp

    ref_tr = TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=2)
    ref = ref_tr(speech_like(160.0, 77), chunk_length_s=30, stride_length_s=0,
                 generate_kwargs={"task": "transcribe", "max_new_tokens": 24}, return_timestamps=True)
    del ref_tr
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert outs[0] == ref and outs[1] == ref
