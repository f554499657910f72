"""Beam search on the MI355X (tw_beam_step + tw_kv_reorder, WhisperEngine.beam_pass) against the oracle's
restatement of transformers' _beam_search (oracle/whisper_oracle.py: beam_search_core, itself pinned token-for-token
to transformers generate(num_beams=5) by tests/test_oracle_golden.py)."""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle import whisper_oracle as wo
from twamd import _lib
from twamd.config import PRESETS, GenerationSettings

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(__file__), "golden")


def _gcfg(dims):
    gen = GenerationSettings.default(dims)
    st = gen.special
    return gen, wo.GenCfg(dims.vocab, st.eot, st.sot, st.lang_begin, st.n_languages, st.transcribe, st.translate,
                          st.notimestamps, gen.suppress_tokens, gen.begin_suppress_tokens)


def _synthetic_logits(history, V, tsb, eot, salt):
    """Deterministic logits for a beam's token history: seeded Gaussian plus a few boosted tokens, with EOS and
    timestamps likely enough that beams finish and the timestamp rules act."""
    h = hash((salt,) + tuple(history)) & 0xFFFFFFFF
    rng = np.random.default_rng(h)
    x = rng.standard_normal(V).astype(np.float32) * 2.0
    x[rng.integers(0, tsb, 6)] += 7.0
    x[tsb + rng.integers(0, 60, 3)] += 6.5
    x[eot] += 5.0 + 0.4 * len(history)
    return x


@pytest.mark.parametrize("nb,W,use_ts,max_new", [(5, 3, True, 24), (2, 4, True, 30), (5, 2, False, 16),
                                                 (3, 3, True, 5)])
def test_beam_step_matches_oracle_core(nb, W, use_ts, max_new):
    d = PRESETS["test-mini"]
    gen, g = _gcfg(d)
    st = gen.special
    V, T, R = d.vocab, 448, W * nb
    P = 3
    # device state
    logits = torch.empty(R, V, device=DEV)
    state = torch.zeros(R, _lib.TW_STATE_STRIDE, dtype=torch.int32, device=DEV)
    state[:, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
    tokens = torch.zeros(R, T, dtype=torch.int32, device=DEV)
    ids = torch.zeros(R, dtype=torch.int32, device=DEV)
    pos = torch.full((R,), P, dtype=torch.int32, device=DEV)
    run_score = torch.full((W, nb), -1e9, device=DEV)
    run_score[:, 0] = 0
    fin_score = torch.full((R,), -1e9, device=DEV)
    fin_flag = torch.zeros(R, dtype=torch.int32, device=DEV)
    fin_len = torch.zeros(R, dtype=torch.int32, device=DEV)
    fin_tokens = torch.zeros(R, T, dtype=torch.int32, device=DEV)
    win = torch.tensor([[1, 0, 0, 0]] * W, dtype=torch.int32, device=DEV)
    src_rows = torch.zeros(R, dtype=torch.int32, device=DEV)
    ws = torch.empty(int(_lib.load().tw_beam_workspace_bytes(R)), dtype=torch.uint8, device=DEV)
    bits = np.zeros((V + 31) // 32, np.uint32)
    for t in gen.suppress_tokens:
        bits[t >> 5] |= np.uint32(1 << (t & 31))
    sup = torch.from_numpy(bits.view(np.int32)).to(DEV)
    bs_ = list(gen.begin_suppress_tokens)[:8]
    sel = _lib.TwSelectParams(V, st.eot, st.eot, st.timestamp_begin, st.notimestamps, 50, int(use_ts), max_new, 0, 0, 0,
                              len(bs_), (ctypes.c_int32 * 8)(*(bs_ + [0] * (8 - len(bs_)))))
    bp = _lib.TwBeamParams(nb, max_new, 1.0, T)
    bst = _lib.TwBeamState(run_score.data_ptr(), fin_score.data_ptr(), fin_flag.data_ptr(), fin_len.data_ptr(),
                           fin_tokens.data_ptr(), win.data_ptr(), src_rows.data_ptr())
    tsb = st.timestamp_begin
    # GPU loop: logits of every row from its history (window salt w)
    hist = [[] for _ in range(R)]
    steps = 0
    while steps < max_new:
        host = np.stack([_synthetic_logits(hist[r], V, tsb, st.eot, r // nb) for r in range(R)])
        logits.copy_(torch.from_numpy(host))
        _lib.call("tw_beam_step", logits.data_ptr(), W, V, sup.data_ptr(), ctypes.byref(sel), ctypes.byref(bp),
                  ctypes.byref(bst), state.data_ptr(), tokens.data_ptr(), ids.data_ptr(), pos.data_ptr(),
                  ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
        steps += 1
        tk = tokens.cpu().numpy()
        hist = [list(tk[r, :steps]) for r in range(R)]
        assert (pos.cpu().numpy() == P + steps).all()
        if bool(win[:, 1].all().item()):
            break
    # oracle: the same logits function, per window
    for w in range(W):
        first = _synthetic_logits([], V, tsb, st.eot, w)

        def step(srcs, toks, _st={"h": [[] for _ in range(nb)]}):
            _st["h"] = [_st["h"][s] + [t] for s, t in zip(srcs, toks)]
            return [_synthetic_logits(h, V, tsb, st.eot, w) for h in _st["h"]]

        ref, tr = wo.beam_search_core(first, step, P, max_new, g, use_ts, nb)
        got = fin_tokens[w * nb, : int(fin_len[w * nb])].tolist()
        assert got == ref, (w, got, ref)
        np.testing.assert_allclose(fin_score.view(W, nb)[w].cpu().numpy(), tr["fin_score"], rtol=1e-5, atol=1e-4)
        assert [bool(x) for x in fin_flag.view(W, nb)[w].cpu().numpy()] == [bool(x) for x in tr["fin_flag"]]


def test_kv_reorder_matches_gather():
    L, cap, H, T, R = 2, 12, 3, 40, 10
    k = torch.randn(L, cap, H, T, 64, device=DEV).to(torch.bfloat16)
    v = torch.randn(L, cap, H, T, 64, device=DEV).to(torch.bfloat16)
    k0, v0 = k.clone(), v.clone()
    src = torch.tensor([0, 0, 1, 4, 4, 5, 9, 2, 8, 3], dtype=torch.int32, device=DEV)
    pos = torch.full((R,), 17, dtype=torch.int32, device=DEV)
    ks, vs = torch.empty_like(k), torch.empty_like(v)
    _lib.call("tw_kv_reorder", k.data_ptr(), v.data_ptr(), ks.data_ptr(), vs.data_ptr(), L, cap, H, T, R, src.data_ptr(),
              pos.data_ptr(), torch.cuda.current_stream().cuda_stream)
    sl = src.long()
    assert torch.equal(k[:, :R, :, :17], k0[:, sl, :, :17]) and torch.equal(v[:, :R, :, :17], v0[:, sl, :, :17])
    assert torch.equal(k[:, :R, :, 17:], k0[:, :R, :, 17:])  # positions past pos untouched
    assert torch.equal(k[:, R:], k0[:, R:])


def test_kv_reorder_large_window_permutations():
    """Beam-shaped reorder at the turbo decoder's scale (60 rows = 12 windows x 5 beams, 20 heads, 448 positions):
    sources inside each window, rows at different positions, the LDS-tile path of the in-place kernel."""
    L, cap, H, T, R, nb = 2, 64, 20, 448, 60, 5
    g = torch.Generator(device="cpu").manual_seed(7)
    k = torch.randn(L, cap, H, T, 64, generator=g).to(torch.bfloat16).to(DEV)
    v = torch.randn(L, cap, H, T, 64, generator=g).to(torch.bfloat16).to(DEV)
    k0, v0 = k.clone(), v.clone()
    src = torch.tensor([w * nb + int(j) for w in range(R // nb) for j in torch.randint(0, nb, (nb,), generator=g)],
                       dtype=torch.int32)
    pos = torch.tensor([int(p) for p in torch.randint(1, T + 1, (R // nb,), generator=g) for _ in range(nb)],
                       dtype=torch.int32)
    assert int(src.min()) >= 0 and int(src.max()) < R and int(pos.max()) <= T  # the kernel trusts them
    src_d, pos_d = src.to(DEV), pos.to(DEV)  # held: a temporary's memory could be reused before the launch
    _lib.call("tw_kv_reorder", k.data_ptr(), v.data_ptr(), None, None, L, cap, H, T, R, src_d.data_ptr(),
              pos_d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for r in range(R):
        p, s = int(pos[r]), int(src[r])
        assert torch.equal(k[:, r, :, :p], k0[:, s, :, :p]) and torch.equal(v[:, r, :, :p], v0[:, s, :, :p]), r
        assert torch.equal(k[:, r, :, p:], k0[:, r, :, p:]) and torch.equal(v[:, r, :, p:], v0[:, r, :, p:]), r
    assert torch.equal(k[:, R:], k0[:, R:])


@pytest.mark.parametrize("t_max", [40, 300])  # the one-round-trip path (< 256 keys) and the two-pass path
def test_self_attention_position_table_equals_gathered_history(t_max):
    """tw_attn_decode_self_tab (beam search's copy-free K/V history) against tw_attn_decode_self on caches where each
    row's history has been gathered through the table: same outputs bit for bit (only the addresses differ), the
    step's own K/V written to its own row. A view offset (row0) and sources in other views are included."""
    H, T, cap, R, row0 = 4, 448, 24, 10, 6
    gen = torch.Generator(device="cpu").manual_seed(t_max)
    k = torch.randn(cap, H, T, 64, generator=gen).to(torch.bfloat16).to(DEV)
    v = torch.randn(cap, H, T, 64, generator=gen).to(torch.bfloat16).to(DEV)
    qkv = (torch.randn(R, 3 * H * 64, generator=gen) * 0.125).to(torch.bfloat16).to(DEV)
    pos = torch.randint(t_max // 2, t_max, (R,), generator=gen, dtype=torch.int32)
    tab = torch.arange(cap, dtype=torch.int32)[:, None].repeat(1, T)
    for r in range(R):  # positions < pos of view row r come from random global rows; pos itself stays own
        tab[row0 + r, : int(pos[r])] = torch.randint(0, cap, (int(pos[r]),), generator=gen, dtype=torch.int32)
    for r in range(R):  # (row0 + r2, pos[r2]) is written by this very launch: no history entry may read it. Beam
        for r2 in range(R):  # search never builds such a table (a window's beams share one position), the random
            p2 = int(pos[r2])  # per-row positions here could, and the read would race the write
            if p2 < int(pos[r]) and int(tab[row0 + r, p2]) == row0 + r2:
                tab[row0 + r, p2] = row0 + r
    kg, vg = k.clone(), v.clone()  # gathered: row0 + r holds its logical history contiguously
    for r in range(R):
        for q in range(int(pos[r])):
            kg[row0 + r, :, q] = k[int(tab[row0 + r, q]), :, q]
            vg[row0 + r, :, q] = v[int(tab[row0 + r, q]), :, q]
    tab_d, pos_d = tab.to(DEV), pos.to(DEV)
    a = torch.empty(R, H * 64, dtype=torch.bfloat16, device=DEV)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("tw_attn_decode_self", qkv.data_ptr(), R, H, T, pos_d.data_ptr(), kg[row0].data_ptr(), vg[row0].data_ptr(),
              a.data_ptr(), s)
    _lib.call("tw_attn_decode_self_tab", qkv.data_ptr(), R, H, T, pos_d.data_ptr(), k[row0].data_ptr(),
              v[row0].data_ptr(), tab_d.data_ptr(), row0, b.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    for r in range(R):  # the step's K/V appended to the row's own cache at pos
        p = int(pos[r])
        assert torch.equal(k[row0 + r, :, p], kg[row0 + r, :, p]) and torch.equal(v[row0 + r, :, p], vg[row0 + r, :, p])


@pytest.mark.parametrize("group,first,B",[(5, 0, 30), (5, 3, 32), (5, 2, 28), (2, 1, 7), (8, 0, 32), (3, 2, 2)])
def test_cross_grouped_matches_lean(group, first, B):
    """tw_attn_decode_cross_grouped (one K/V read per beam group) against tw_attn_decode_cross row for row on a beam
    row map (rows of a group share their window's encoder slot), including a leading partial group; the
    keys split in slices merged by a second launch (another softmax merge order), so equal to within 4 bf16 ulps (of max(|x|, 0.02))
    (tolerance written here; measured on MI355X in profiles/r03q_beam_kernels.txt)."""
    H, S, Bt = 20, 1500, 12
    gen = torch.Generator(device="cpu").manual_seed(group * 100 + first)
    q = (torch.randn(B, H * 64, generator=gen) * 0.125).to(torch.bfloat16).to(DEV)
    ckv = torch.randn(2, Bt, H, S, 64, generator=gen).to(torch.bfloat16).to(DEV)
    rows = [0] * first + [1 + (r // group) for r in range(B - first)]
    rmap = torch.tensor([x % Bt for x in rows], dtype=torch.int32, device=DEV)
    a = torch.empty(B, H * 64, dtype=torch.bfloat16, device=DEV)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("tw_attn_decode_cross", q.data_ptr(), B, H, S, Bt, rmap.data_ptr(), ckv.data_ptr(), a.data_ptr(), s)
    ws = torch.empty(int(_lib.load().tw_attn_decode_cross_grouped_ws_bytes(B, H)) // 4, device=DEV)
    _lib.call("tw_attn_decode_cross_grouped", q.data_ptr(), B, H, S, Bt, rmap.data_ptr(), group, first, ckv.data_ptr(),
              ws.data_ptr(), b.data_ptr(), s)
    torch.cuda.synchronize()
    d = (a.float() - b.float()).abs()
    # bf16 ulp of the larger magnitude, floored at that of 0.02 (outputs here are ~0.05: near-zero entries would
    # otherwise count a rounding step of their neighbours' scale as many ulps)
    ulp = torch.maximum(a.float().abs(), b.float().abs()).clamp_min(0.02) * 2.0 ** -7
    print(f"grouped vs lean: {int((d > 0).sum())} of {d.numel()} differ, max {d.max().item():.2e}, "
          f"max in ulps {(d / ulp).max().item():.2f}")
    assert bool((d <= 4 * ulp).all())
    # and against an fp32 reference of softmax(q K^T) V
    kf, vf = ckv[0].float(), ckv[1].float()
    for r in (0, B - 1):
        sc = torch.einsum("hd,hsd->hs", q[r].float().view(H, 64), kf[rmap[r]])
        ref = torch.einsum("hs,hsd->hd", sc.softmax(-1), vf[rmap[r]]).reshape(-1)
        assert (b[r].float() - ref).abs().max().item() < 2e-2


@pytest.fixture(scope="module")
def mini():
    from twamd.pipeline import TurboTranscriber

    return TurboTranscriber.from_pretrained("test-mini", seed=1234, max_batch=3, max_beams=5)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_engine_beam_search_matches_transformers(mini, case):
    """generate(num_beams=5) on the engine vs transformers' own beam search (tests/golden/beam.json)."""
    from twamd.synth_audio import silence, speech_like, white_noise

    gold = json.load(open(os.path.join(G, "beam.json")))
    c = gold["cases"][case]
    clips = {"speech30": speech_like(30.0, 1234), "noise12": white_noise(12.3, 7), "zeros30": silence(30.0)}
    eng = mini.engine
    host = np.zeros((3, 480000), np.float32)
    for i, name in enumerate(c["clips"]):
        x = clips[name][:480000]
        host[i, : len(x)] = x
    eng.wave[:3].copy_(torch.from_numpy(host))
    eng.logmel(3)
    seqs = eng.generate(3, task="transcribe", max_new_tokens=c["max_new_tokens"],
                        return_timestamps=c["return_timestamps"], num_beams=5)
    for got, ref in zip(seqs, c["sequences"]):
        while ref and ref[-1] == 50257:
            ref = ref[:-1]
        assert list(got) == ref


@pytest.mark.parametrize("name", ["ref_60_5", "mode_30_0"])
def test_pipeline_beam5_matches_transformers_pipeline(mini, name):
    """The drop-in callable with the reference's call and the ASR pipeline's default num_beams=5 reproduces the
    transformers pipeline's output (tests/golden/beam.json)."""
    from twamd.synth_audio import speech_like, white_noise

    gold = json.load(open(os.path.join(G, "beam.json")))
    case = next(c for c in gold["pipeline"] if c["name"] == name)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    kw = {k: v for k, v in case["kwargs"].items()}
    r = mini(audio, generate_kwargs={"task": "transcribe", "num_beams": 5, "max_new_tokens": 40},
             return_timestamps=True, **kw)
    _same_or_beam_within_tau(mini, r, case["output"], audio, kw, 40)


@pytest.mark.parametrize("name", ["ref_60_5", "mode_30_0"])
def test_pipeline_beam5_exact_with_enc4_attention(mini, name):
    """one exact-match run of the beam-5 pipeline goldens. With the encoder attention at k_attn_enc4
    (tw_attn_set_variant 16, bit-identical to the enc2 form these goldens were first matched with) the drop-in's
    output equals the transformers pipeline's exactly — no tolerance — so a host-side beam or segment regression
    cannot hide behind the near-tie allowance the default (enc5) runs need."""
    from twamd.synth_audio import speech_like, white_noise

    gold = json.load(open(os.path.join(G, "beam.json")))
    case = next(c for c in gold["pipeline"] if c["name"] == name)
    audio = np.concatenate([speech_like(40.0, 5), white_noise(35.0, 11)])
    eng = mini.engine
    saved = eng.attn_kernel
    eng.attn_kernel = (16, 16)
    try:
        r = mini(audio, generate_kwargs={"task": "transcribe", "num_beams": 5, "max_new_tokens": 40},
                 return_timestamps=True, **case["kwargs"])
    finally:
        eng.attn_kernel = saved
    ref = case["output"]
    assert r["text"] == ref["text"]
    assert [(tuple(c["timestamp"]), c["text"]) for c in r["chunks"]] == \
        [(tuple(c["timestamp"]), c["text"]) for c in ref["chunks"]]


def _same_or_beam_within_tau(t, r, ref, audio, kw, max_new):
    """The transformers pipeline's output exactly, or — where a bf16 near-tie ranks two fp32 candidates the other way
    (the random-weight model's beams lie within hundredths of a logit) — every device seek pass equal to the fp32
    oracle's beam search up to one whose first differing decision is among the fp32 search's candidates or within
    0.3 logits (test_gpu_e2e._beam_passes_within_tau, the tolerance every other beam pipeline test uses)."""
    got = (r["text"], [(tuple(c["timestamp"]), c["text"]) for c in r["chunks"]])
    want = (ref["text"], [(tuple(c["timestamp"]), c["text"]) for c in ref["chunks"]])
    if got == want:
        return
    from test_gpu_e2e import D, _beam_passes_within_tau

    sd = wo.synth_state_dict(D.d_model, D.encoder_layers, D.decoder_layers, D.ffn, D.n_mels, D.vocab, 1234)
    n = _beam_passes_within_tau(t, wo.WhisperOracle(sd, D.heads), audio, kw, "transcribe", max_new)
    assert n > 0, "outputs differ but every device pass equals the fp32 beam search"  # (then it is a host bug)


def test_default_callable_long_audio_matches_transformers_pipeline():
    """The drop-in as from_pretrained builds it by default (engine batches of 24 windows, beam-5 rows) with the
    reference's call on 8 minutes of audio (10 windows: 50 decoder rows in one batch) reproduces the transformers
    pipeline (tests/golden/beam_long.json)."""
    from twamd.pipeline import TurboTranscriber
    from twamd.synth_audio import speech_like, white_noise

    gold = json.load(open(os.path.join(G, "beam_long.json")))
    tr = TurboTranscriber.from_pretrained("test-mini", seed=1234)
    audio = np.concatenate([speech_like(200.0, 21), white_noise(80.0, 22), speech_like(200.0, 23)])
    r = tr(audio, generate_kwargs={"task": "transcribe", "max_new_tokens": gold["max_new_tokens"]},
           return_timestamps=True, **gold["kwargs"])
    _same_or_beam_within_tau(tr, r, gold["output"], audio, gold["kwargs"], gold["max_new_tokens"])


def _racy_table(R, cap, T, row0, seed):
    """Random per-row positions and history sources, WITHOUT removing the entries that name a (row, position) the
    same launch writes (the contract tw_attn_decode_self_tab states), plus the host count of such entries per row."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    pos = torch.randint(20, 60, (R,), generator=gen, dtype=torch.int32)
    tab = torch.arange(cap, dtype=torch.int32)[:, None].repeat(1, T)
    for r in range(R):
        tab[row0 + r, : int(pos[r])] = torch.randint(row0, row0 + R, (int(pos[r]),), generator=gen, dtype=torch.int32)
    bad = [sum(1 for q in range(int(pos[r])) if 0 <= int(tab[row0 + r, q]) - row0 < R
               and int(pos[int(tab[row0 + r, q]) - row0]) == q) for r in range(R)]
    return tab, pos, bad


def test_kv_tab_check_counts_contract_violations():
    """tw_kv_tab_check against a host count of the entries that would race, on a racy table and on the same table
    with those entries pointed back at the row itself (0 everywhere)."""
    R, cap, T, row0 = 12, 20, 448, 5
    tab, pos, bad = _racy_table(R, cap, T, row0, 11)
    assert sum(bad) > 0
    out = torch.full((R,), -1, dtype=torch.int32, device=DEV)
    tab_d, pos_d = tab.to(DEV), pos.to(DEV)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("tw_kv_tab_check", tab_d.data_ptr(), pos_d.data_ptr(), row0, R, T, out.data_ptr(), s)
    assert out.cpu().tolist() == bad
    for r in range(R):
        for q in range(int(pos[r])):
            r2 = int(tab[row0 + r, q]) - row0
            if 0 <= r2 < R and int(pos[r2]) == q:
                tab[row0 + r, q] = row0 + r
    tab_d = tab.to(DEV)
    _lib.call("tw_kv_tab_check", tab_d.data_ptr(), pos_d.data_ptr(), row0, R, T, out.data_ptr(), s)
    assert out.cpu().tolist() == [0] * R


def test_debug_build_refuses_racy_position_table():
    """the -DTW_DEBUG=1 library (libtwhip_dbg.so) checks the position-table contract before the
    launch and fails loudly (TW_ERR_ARG naming the row) instead of racing; a valid table runs and gives the product
    library's output bit for bit."""
    if not os.path.exists(_lib.DEBUG_LIB_PATH):
        pytest.skip("libtwhip_dbg.so not built (make -C turbo-whisper-workspace_amd/csrc debug)")
    dbg = _lib.load_debug()
    R, cap, T, row0, H = 12, 20, 448, 5, 4
    tab, pos, bad = _racy_table(R, cap, T, row0, 12)
    assert sum(bad) > 0
    gen = torch.Generator(device="cpu").manual_seed(3)
    k = torch.randn(cap, H, T, 64, generator=gen).to(torch.bfloat16).to(DEV)
    v = torch.randn(cap, H, T, 64, generator=gen).to(torch.bfloat16).to(DEV)
    qkv = (torch.randn(R, 3 * H * 64, generator=gen) * 0.125).to(torch.bfloat16).to(DEV)
    out = torch.empty(R, H * 64, dtype=torch.bfloat16, device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    tab_d, pos_d = tab.to(DEV), pos.to(DEV)
    k1, v1 = k.clone(), v.clone()
    rc = dbg.tw_attn_decode_self_tab(qkv.data_ptr(), R, H, T, pos_d.data_ptr(), k1[row0].data_ptr(),
                                     v1[row0].data_ptr(), tab_d.data_ptr(), row0, out.data_ptr(), s)
    assert rc == 1, rc
    first = next(r for r in range(R) if bad[r])
    msg = dbg.tw_last_error().decode()
    assert "precondition violated" in msg and f"row {row0 + first}" in msg, msg
    assert torch.equal(k1, k) and torch.equal(v1, v)  # refused before the launch: nothing written
    for r in range(R):  # repaired table: runs, same output as the product library
        for q in range(int(pos[r])):
            r2 = int(tab[row0 + r, q]) - row0
            if 0 <= r2 < R and int(pos[r2]) == q:
                tab[row0 + r, q] = row0 + r
    tab_d = tab.to(DEV)
    k2, v2 = k.clone(), v.clone()
    out2 = torch.empty_like(out)
    assert dbg.tw_attn_decode_self_tab(qkv.data_ptr(), R, H, T, pos_d.data_ptr(), k1[row0].data_ptr(),
                                       v1[row0].data_ptr(), tab_d.data_ptr(), row0, out.data_ptr(), s) == 0
    _lib.call("tw_attn_decode_self_tab", qkv.data_ptr(), R, H, T, pos_d.data_ptr(), k2[row0].data_ptr(),
              v2[row0].data_ptr(), tab_d.data_ptr(), row0, out2.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(out, out2) and torch.equal(k1, k2) and torch.equal(v1, v2)


def test_kv_reorder_row_limit():
    """tw_kv_reorder stages one position of every moved row in LDS (R * 128 B <= 56 KiB): R = 448 runs,
    R = 449 is refused up front instead of asking for more LDS than the launch may use."""
    L, H, T = 1, 1, 4
    for R, ok in ((448, True), (449, False)):
        k = torch.randn(L, R, H, T, 64, device=DEV).to(torch.bfloat16)
        v = torch.randn(L, R, H, T, 64, device=DEV).to(torch.bfloat16)
        k0 = k.clone()
        src = torch.arange(R, dtype=torch.int32, device=DEV).flip(0)
        pos = torch.full((R,), 3, dtype=torch.int32, device=DEV)
        rc = _lib.load().tw_kv_reorder(k.data_ptr(), v.data_ptr(), None, None, L, R, H, T, R, src.data_ptr(),
                                       pos.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (rc == 0) == ok, (R, rc)
        if ok:
            assert torch.equal(k[:, :, :, :3], k0[:, src.long(), :, :3])
