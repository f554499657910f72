"""tw_dec_fused (csrc/decfused.hip): the decoder's layers for one token as one persistent launch, against the launch
chain it replaces (WhisperEngine.decoder_step's 45 kernels: resid_ln, q/k/v, self-attention, out_proj, cross-q,
cross-attention, out_proj, fc1, fc2, final LayerNorm) at large-v3-turbo dims with the seeded synthetic weights.

What is compared (the two paths differ in the f32 summation order of the projections and of the self-attention
softmax, and so in which bf16 activations round up or down; the LayerNorm and cross-attention arithmetic is the
chain's):
  * one decoder step at R = 1 .. 32 rows from random caches (positions 0 .. 447, i.e. one and two key chunks of the
    self-attention) against a plain PyTorch fp32 restatement of the step from the same bf16 weights, caches and
    cross K/V (activations unrounded): the fused logits no further from it than REL_TO_CHAIN x the chain's distance +
    ABS_SLACK, the K/V appended at pos within KV_REL of the chain's (two bf16 ulps of the largest), every other cache
    position untouched;
  * bit-identical results from a second launch and with an agent-scope acquire after every phase wait
    (tw_dec_fused_set_acquire): a stale read of a handed-off line or a hand-off race would show as a difference here;
    a 37-workgroup grid (items re-dealt and re-sliced over fewer workgroups) within the chain tolerance;
  * a greedy pass over the bench workload (24 windows, 128 tokens, EOS suppressed) with the fused launch: windows
    0 and 23 against the fp32 goldens as the bench's parity leg checks them (exact or within tau), and the tokens of
    every window equal to the chain's up to near-ties;
  * the sticky error word stays 0 (no phase wait timed out).
"""
import os
import sys

import pytest
import torch

from twamd import _lib
from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import workload

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import turbo_parity as tp  # noqa: E402

pytestmark = pytest.mark.gpu
LOGIT_ABS = 0.1     # fused vs chain logits, any step (random caches; the bench pass is judged against the goldens)
REL_TO_CHAIN = 1.5  # fused distance to the fp32 step <= REL_TO_CHAIN x the chain's + ABS_SLACK
ABS_SLACK = 0.01
KV_REL = 1.0 / 64  # appended K/V vs the chain's, relative to the largest appended value (two bf16 ulps)


@pytest.fixture(scope="module")
def turbo():
    tr = TurboTranscriber.from_pretrained("large-v3-turbo", seed=1234, max_batch=32, max_beams=1)
    yield tr
    tr.engine.dec_fused_alone = type(tr.engine).dec_fused_alone
    tr.engine.dec_fused_max_rows = type(tr.engine).dec_fused_max_rows
    tr.engine._dec_context()
    del tr
    torch.cuda.empty_cache()


def _random_state(eng, R, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    gd = torch.Generator(device=eng.device).manual_seed(seed)
    d = eng.d
    for t in (eng.kcache, eng.vcache, eng.cross_kv):
        t.copy_(torch.randn(t.shape, generator=gd, device=eng.device, dtype=torch.float32) * 0.5)
    pos = torch.randint(0, d.max_target_positions, (R,), generator=g, dtype=torch.int32)
    pos[0] = 0
    if R > 1:
        pos[1] = d.max_target_positions - 1
    eng.pos[:R] = pos.to(eng.device)
    eng.ids[:R] = torch.randint(0, d.vocab, (R,), generator=g, dtype=torch.int32).to(eng.device)
    return pos


def _step(eng, R, fused, grid=0, acquire=0):
    eng.dec_fused_alone = fused
    eng.dec_fused_max_rows = 32
    eng._dec_context()
    _lib.call("tw_dec_fused_set_grid", grid)
    _lib.call("tw_dec_fused_set_acquire", acquire)
    k0, v0 = eng.kcache.clone(), eng.vcache.clone()
    eng.decoder_step(R, r_enc=R)
    torch.cuda.synchronize()
    out = (eng.logits[:R].clone(), eng.kcache.clone(), eng.vcache.clone(), eng.xd[:R].clone())
    eng.kcache.copy_(k0)
    eng.vcache.copy_(v0)
    _lib.call("tw_dec_fused_set_grid", 0)
    _lib.call("tw_dec_fused_set_acquire", 0)
    return out


def _ref_step(eng, R, pos):
    """fp32 restatement of one decoder step (WhisperDecoderLayer.forward, $TF/models/whisper/modeling_whisper.py:
    448-505, + the final layer_norm and the tied proj_out) from the engine's bf16 weights, its self K/V caches (keys
    < pos) and cross K/V, activations kept in f32. Logits [R][V]."""
    d, w = eng.d, eng.w
    D, H = d.d_model, d.heads
    fn = torch.nn.functional
    f = lambda t: t.float()  # noqa: E731
    dev = eng.device
    pos_l = [int(p) for p in pos]
    ids = eng.ids[:R].long()
    x = f(w.emb[ids]) + f(w.pos_dec[torch.as_tensor(pos_l, device=dev)])
    ln = lambda v, g, b: fn.layer_norm(v, (D,), g, b, 1e-5)  # noqa: E731

    def attend(q, K, V):  # q [H][64], K / V [H][n][64]
        p = torch.softmax(torch.einsum("hd,hnd->hn", q, K), dim=-1)
        return torch.einsum("hn,hnd->hd", p, V).reshape(D)

    for li, L in enumerate(w.dec):
        qkv = ln(x, L.ln1_g, L.ln1_b) @ f(L.wqkv).T + L.bqkv
        q, k, v = qkv.split(D, dim=1)
        a = torch.stack([attend(q[r].view(H, 64),
                                torch.cat([f(eng.kcache[li, r, :, : pos_l[r]]), k[r].view(H, 1, 64)], 1),
                                torch.cat([f(eng.vcache[li, r, :, : pos_l[r]]), v[r].view(H, 1, 64)], 1))
                         for r in range(R)])
        x = x + (a @ f(L.wo).T + L.bo)
        q2 = ln(x, L.ln2_g, L.ln2_b) @ f(L.wq_x).T + L.bq_x
        # the slot's cross K/V as encoded for r_enc = R rows: [layers][k | v][R][H][S][64], contiguous
        blk = eng.cross_kv.reshape(-1)[li * 2 * R * H * 1500 * 64:(li + 1) * 2 * R * H * 1500 * 64]
        xk, xv = blk.view(2, R, H, 1500, 64)
        a2 = torch.stack([attend(q2[r].view(H, 64), f(xk[r]), f(xv[r])) for r in range(R)])
        x = x + (a2 @ f(L.wo_x).T + L.bo_x)
        h = fn.gelu(ln(x, L.ln3_g, L.ln3_b) @ f(L.w1).T + L.b1)
        x = x + (h @ f(L.w2).T + L.b2)
    return ln(x, w.dec_ln_g, w.dec_ln_b) @ f(w.emb).T


@pytest.mark.parametrize("R", [1, 7, 16, 17, 24, 32])
def test_fused_step_matches_chain(turbo, R):
    eng = turbo.engine
    pos = _random_state(eng, R, 100 + R)
    ref = _ref_step(eng, R, pos)
    lc, kc, vc, xc = _step(eng, R, False)
    lf, kf, vf, xf = _step(eng, R, True)
    assert torch.isfinite(lf).all()
    d = (lf - lc).abs().max().item()
    scale = lc.abs().max().item()
    xd = ((xf - xc).abs().max() / xc.abs().max()).item()
    ec, ef = (lc - ref).abs().max().item(), (lf - ref).abs().max().item()
    # the appended K/V at pos and nothing else
    kd = vd = kmax = vmax = 0.0
    for r in range(R):
        p = int(pos[r])
        kd = max(kd, (kf[:, r, :, p] - kc[:, r, :, p]).float().abs().max().item())
        vd = max(vd, (vf[:, r, :, p] - vc[:, r, :, p]).float().abs().max().item())
        kmax = max(kmax, kc[:, r, :, p].float().abs().max().item())
        vmax = max(vmax, vc[:, r, :, p].float().abs().max().item())
        kf[:, r, :, p] = kc[:, r, :, p]
        vf[:, r, :, p] = vc[:, r, :, p]
    print(f"R={R}: logits max|d| vs fp32 step: chain {ec:.2e}, fused {ef:.2e}; fused vs chain {d:.2e} (|logit| max "
          f"{scale:.1f}), residual rel {xd:.1e}, k {kd:.1e} v {vd:.1e}")
    assert ef <= REL_TO_CHAIN * ec + ABS_SLACK, (ef, ec)
    assert d <= LOGIT_ABS and kd <= KV_REL * kmax and vd <= KV_REL * vmax
    assert torch.equal(kf, kc) and torch.equal(vf, vc)  # no other cache position written
    # argmax agrees wherever the chain's top-2 margin is clear
    top2 = lc.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 4 * LOGIT_ABS
    assert torch.equal(lf.argmax(1)[clear], lc.argmax(1)[clear])
    # deterministic: again, with the items dealt over 37 workgroups, and with an acquire fence after every wait
    lf2, kf2, vf2, xf2 = _step(eng, R, True)
    lg, kg, vg, xg = _step(eng, R, True, grid=37)
    la, ka, va, xa = _step(eng, R, True, acquire=1)
    assert torch.equal(lf2, lf) and torch.equal(xf2, xf) and torch.equal(kf2, ka) and torch.equal(vf2, va)
    assert torch.equal(la, lf) and torch.equal(xa, xf)
    # (a 37-workgroup grid re-slices the attention items: the same sums in another order)
    assert (lg - lf).abs().max().item() <= LOGIT_ABS and torch.isfinite(lg).all()
    assert (kg.float() - ka.float()).abs().max().item() <= KV_REL * kmax
    assert (vg.float() - va.float()).abs().max().item() <= KV_REL * vmax
    assert int(eng._fused_err[0].item()) == 0


def test_fused_repeated_steps_stable(turbo):
    """30 launches back to back over changing inputs, each against the chain (hand-offs under a busy device)."""
    eng = turbo.engine
    R = 24
    worst = 0.0
    for it in range(30):
        if it % 10 == 0:
            _random_state(eng, R, 1000 + it)
        eng.ids[:R] = torch.randint(0, eng.d.vocab, (R,), dtype=torch.int32, device=eng.device)
        lc = _step(eng, R, False)[0]
        lf = _step(eng, R, True)[0]
        worst = max(worst, (lf - lc).abs().max().item())
    print(f"fused vs chain, 30 launches at R={R}: worst logits max|d| {worst:.2e}")
    assert worst <= LOGIT_ABS
    eng.check_fused()


def test_fused_bench_pass_vs_goldens(turbo):
    """The bench workload decoded alone with the fused launch: windows 0 and 23 against the fp32 goldens (as bench.py's
    parity leg), every window's tokens equal to the chain's or leaving them at a near-tie."""
    z = tp.load()
    eng = turbo.engine
    gen = turbo.gen
    B, T = 24, 128
    audio = workload(B, 30.0, seed=1234)
    eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])
    try:
        out = {}
        eng.dec_fused_max_rows = 32
        for fused in (False, True):
            eng.dec_fused_alone = fused
            eng.wave[:B].copy_(torch.from_numpy(audio))
            eng.logmel(B)
            eng.generate(B, task="transcribe", max_new_tokens=T, max_passes=1)
            out[fused] = ([p[0] for p in eng.last_passes], list(eng.last_langs))
        passes, langs = out[True]
        assert all(len(p) == T for p in passes)
        for w in tp.BENCH_WINDOWS:
            r = tp.check_bench_window(z, w, passes[w], langs[w])
            print(f"fused bench window {w}: {r}")
            assert r["lang_ok"] and r["status"] in ("exact", "within_tau"), (w, r)
        same = sum(a == b for a, b in zip(out[False][0], passes))
        first = [next((k for k, (x, y) in enumerate(zip(a, b)) if x != y), None) for a, b in zip(out[False][0], passes)]
        print(f"fused vs chain tokens: {same}/{B} windows identical; first differences {first}")
        assert out[False][1] == langs
        assert same >= B // 2
        eng.check_fused()
    finally:
        eng.set_suppress_tokens(list(gen.suppress_tokens))
        eng.dec_fused_alone = type(eng).dec_fused_alone
        eng.dec_fused_max_rows = type(eng).dec_fused_max_rows
