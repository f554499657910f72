"""WhisperEngineF32: the engine at fp32 arithmetic (BASELINE configs[0], whisper-tiny.en fp32: the reference loads
the pipeline with `torch_dtype=torch.float32` on the CPU, /root/reference/vocalis/core/audio_pipeline.py:195-200).

The generation machinery is WhisperEngine's unchanged (decode / sample / beam passes, seek loop, temperature
fallback, timestamp rules, the selection and beam kernels, graph capture): they act on f32 logits and int32 state,
whatever precision produced them. What changes is every producer of those logits — the encoder and the decoder step
run on csrc/f32path.hip (tw_gemm_f32 on v_mfma_f32_16x16x4_f32, f32 LayerNorm, f32 attention with f32 K/V caches), with
the weights held as f32 (build_weights(dtype=torch.float32)). Module map as the bf16 path:
WhisperEncoder.forward / WhisperDecoder.forward ($TF/models/whisper/modeling_whisper.py:600-640, 690-795)."""
import ctypes
from typing import Optional

import torch

from . import _lib
from .frontend import N_FRAMES
from .engine import LN_EPS, S_ENC, VIEW_ROWS, DecView, WhisperEngine, on_engine_streams

__all__ = ["WhisperEngineF32"]


class WhisperEngineF32(WhisperEngine):
    F32 = True

    def __init__(self, weights, gen, max_batch: int = 24, device: str = "cuda", use_graphs: bool = True,
                 max_beams: int = 1, enc_fp8: Optional[bool] = None):
        if enc_fp8:
            raise ValueError("the fp32 path has no MX fp8 encoder")
        super().__init__(weights, gen, max_batch=max_batch, device=device, use_graphs=use_graphs,
                         max_beams=max_beams, enc_fp8=False)

    # ------------------------------------------------------------------ launches
    def _g32(self, A, W, M, N, K, epi, out, stream, bias=None, aux=None, aux_rows=0, kv_geom=None, lda=None):
        """tw_gemm_f32: out (epi) = A[:M] (K columns, row stride lda) x W^T (N rows of K)."""
        rec = self._begin_timer(("gemm_f32", epi), 2.0 * M * N * K, stream)
        _lib.call("tw_gemm_f32", A.data_ptr(), W.data_ptr(), M, N, K, K if lda is None else lda, W.shape[1], epi,
                  out.data_ptr(), N, _lib.ptr(bias), _lib.ptr(aux), aux_rows,
                  None if kv_geom is None else (ctypes.c_int * 4)(*kv_geom), stream.cuda_stream)
        self._end_timer(rec, stream)

    def _ln32(self, x, g, b, M, out, stream):
        _lib.call("tw_layernorm_f32", x.data_ptr(), g.data_ptr(), b.data_ptr(), M, self.d.d_model, LN_EPS,
                  out.data_ptr(), stream.cuda_stream)

    # ------------------------------------------------------------------ encoder
    def _encode_chunks(self, R: int, row_map=True, seek=True, slot: Optional[int] = None, sync: bool = True):
        """WhisperEncoder.forward at f32: conv stem (im2col + GEMM, GELU, + positions), the layers, the final
        LayerNorm and every decoder layer's cross-attention K/V (f32, [layer][k|v][R][H][S][64]) into
        cross_kv_buf[slot]; yields after the stem and after every layer, as the bf16 path."""
        d, w = self.d, self.w
        slot = self._slot if slot is None else slot
        D, F, H = d.d_model, d.ffn, d.heads
        M3, M15 = R * N_FRAMES, R * S_ENC
        st = self._enc_begin(sync)
        s = st.cuda_stream
        rm = self.row_map.data_ptr() if row_map else None
        E = _lib
        if self._long is not None:  # a long-form input's features (set_long_input): one row of T frames
            lf = self._long
            _lib.call("tw_im2col_conv1_f32", lf["feats"].data_ptr(), d.n_mels, lf["ld"], lf["max_frames"].data_ptr(),
                      rm, self.seek.data_ptr(), R, w.kpad1, self.a1.data_ptr(), s)
        else:
            _lib.call("tw_im2col_conv1_f32", self.feats_buf[slot].data_ptr(), d.n_mels, N_FRAMES, None, rm,
                      self.seek.data_ptr() if seek else None, R, w.kpad1, self.a1.data_ptr(), s)
        self._g32(self.a1, w.conv1_w, M3, D, w.kpad1, E.TW_EPI_GELU_F32, self.h1, st, bias=w.conv1_b)
        _lib.call("tw_im2col_conv2_f32", self.h1.data_ptr(), R, D, self.a2.data_ptr(), s)
        self._g32(self.a2, w.conv2_w, M15, D, 3 * D, E.TW_EPI_GELU_POS_F32, self.x, st, bias=w.conv2_b,
                  aux=w.pos_enc, aux_rows=S_ENC)
        yield
        for L in w.enc:
            self._ln32(self.x, L.ln1_g, L.ln1_b, M15, self.hln, st)
            self._g32(self.hln, L.wqkv, M15, 3 * D, D, E.TW_EPI_F32, self.qkv, st, bias=L.bqkv)
            rec = self._begin_timer(("attn_encoder_f32", 0), 4.0 * S_ENC * S_ENC * 64 * H * R, st)
            _lib.call("tw_attn_encoder_f32", self.qkv.data_ptr(), R, S_ENC, H, self.att.data_ptr(), s)
            self._end_timer(rec, st)
            self._g32(self.att, L.wo, M15, D, D, E.TW_EPI_RESID_F32, self.x, st, bias=L.bo)
            self._ln32(self.x, L.ln2_g, L.ln2_b, M15, self.hln, st)
            self._g32(self.hln, L.w1, M15, F, D, E.TW_EPI_GELU_F32, self.ffn, st, bias=L.b1)
            self._g32(self.ffn, L.w2, M15, D, F, E.TW_EPI_RESID_F32, self.x, st, bias=L.b2)
            yield
        self._ln32(self.x, w.enc_ln_g, w.enc_ln_b, M15, self.hln, st)  # encoder last_hidden_state (f32)
        self._g32(self.hln, w.wkv_x, M15, d.decoder_layers * 2 * D, D, E.TW_EPI_CROSSKV, self.cross_kv_buf[slot], st,
                  bias=w.bkv_x, kv_geom=(S_ENC, R, D, H))
        self._enc_end(sync, slot)

    # ------------------------------------------------------------------ decoder
    @on_engine_streams
    def decoder_step(self, R: int, with_logits: bool = True, v: Optional[DecView] = None, r_enc: Optional[int] = None,
                     pre_embedded: bool = False) -> None:
        """WhisperDecoder.forward for one token per row at f32 (as WhisperEngine.decoder_step: ids[b] at pos[b] ->
        logits[b]): embedding, per layer LayerNorm -> q/k/v -> self-attention (K/V cache append) -> out_proj +
        residual -> LayerNorm -> cross q -> cross-attention -> out_proj + residual -> LayerNorm -> fc1 (GELU) -> fc2 +
        residual; final LayerNorm and the tied proj_out. The residual stream xd is updated in place by the GEMMs'
        RESID epilogue."""
        if pre_embedded:
            raise ValueError("the fp32 path has no fused select + embedding (fused_select is off)")
        if v is None and R > VIEW_ROWS:
            r_enc = R if r_enc is None else r_enc
            for r0 in range(0, R, VIEW_ROWS):
                n = min(VIEW_ROWS, R - r0)
                self.decoder_step(n, with_logits, self._view(r0, n), r_enc)
            return
        v = v or self._view(0, R)
        r_enc = R if r_enc is None else r_enc
        d, w, E = self.d, self.w, _lib
        D, F, H, T = d.d_model, d.ffn, d.heads, d.max_target_positions
        st = v.stream
        s = st.cuda_stream
        hp, fp = v.hp[: R * D].view(R, D), v.fp[: R * F].view(R, F)
        _lib.call("tw_embed_decoder_f32", w.emb.data_ptr(), w.pos_dec.data_ptr(), v.ids.data_ptr(), v.pos.data_ptr(),
                  R, D, v.xd.data_ptr(), s)
        xkv_stride = 2 * r_enc * H * S_ENC * 64
        ks = self._kv_start[v.r0:].data_ptr() if self._masked else None  # left-padded prompts (prefill)
        tab = self._kv_tab.data_ptr() if self._kv_tab is not None else None  # beam pass: the position table
        for li, L in enumerate(w.dec):
            kc, vc = self.kcache[li, v.r0:].data_ptr(), self.vcache[li, v.r0:].data_ptr()
            self._ln32(v.xd, L.ln1_g, L.ln1_b, R, hp, st)
            self._g32(hp, L.wqkv, R, 3 * D, D, E.TW_EPI_F32, v.qkvd, st, bias=L.bqkv)
            _lib.call("tw_attn_decode_self_f32", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc, tab, v.r0, ks,
                      v.attd.data_ptr(), s)
            self._g32(v.attd, L.wo, R, D, D, E.TW_EPI_RESID_F32, v.xd, st, bias=L.bo)
            self._ln32(v.xd, L.ln2_g, L.ln2_b, R, hp, st)
            self._g32(hp, L.wq_x, R, D, D, E.TW_EPI_F32, v.qd, st, bias=L.bq_x)
            ckv, rmap = self._cross_ptrs(li, xkv_stride, v)
            self._cross_attend_f32(li, R, r_enc, rmap, ckv, v)
            self._g32(v.attd, L.wo_x, R, D, D, E.TW_EPI_RESID_F32, v.xd, st, bias=L.bo_x)
            self._ln32(v.xd, L.ln3_g, L.ln3_b, R, hp, st)
            self._g32(hp, L.w1, R, F, D, E.TW_EPI_GELU_F32, fp, st, bias=L.b1)
            self._g32(fp, L.w2, R, D, F, E.TW_EPI_RESID_F32, v.xd, st, bias=L.b2)
        if with_logits:
            self._ln32(v.xd, w.dec_ln_g, w.dec_ln_b, R, hp, st)
            self._g32(hp, w.emb, R, d.vocab, D, E.TW_EPI_F32, v.logits, st)

    def _cross_attend_f32(self, li: int, R: int, r_enc: int, rmap, ckv, v: DecView) -> None:
        """Cross-attention of the view's rows (beam rows through dec_row_map); with token-level timestamps requested
        the alignment heads of this layer also write their attention probabilities (as tw_attn_decode_cross_probs)."""
        H, s = self.d.heads, v.stream.cuda_stream
        al = self._align
        probs, mask, slot0, n_slots, pos0, n_steps = None, 0, 0, 0, 0, 0
        if al is not None and li in al["layers"]:
            mask, slot0 = al["layers"][li]
            n_slots, pos0, n_steps = al["n_slots"], al["pos0"], al["n_steps"]
            probs = al["buf"].data_ptr() + v.r0 * n_steps * n_slots * S_ENC * 4
        rec = self._begin_timer(("attn_decode_cross_f32", 0), 4.0 * R * H * S_ENC * 64 * 2, v.stream)
        _lib.call("tw_attn_decode_cross_f32", v.qd.data_ptr(), R, H, S_ENC, r_enc, rmap, ckv, v.attd.data_ptr(), probs,
                  mask, slot0, n_slots, v.pos.data_ptr(), pos0, n_steps, s)
        self._end_timer(rec, v.stream)

    def _embed_head(self, v: DecView) -> None:
        """The head of a decoder step alone (embedding + layer 0's self_attn_layer_norm) for view v."""
        D = self.d.d_model
        L0 = self.w.dec[0]
        _lib.call("tw_embed_decoder_f32", self.w.emb.data_ptr(), self.w.pos_dec.data_ptr(), v.ids.data_ptr(),
                  v.pos.data_ptr(), v.n, D, v.xd.data_ptr(), v.stream.cuda_stream)
        self._ln32(v.xd, L0.ln1_g, L0.ln1_b, v.n, v.hp[: v.n * D].view(v.n, D), v.stream)

    def _select(self, R: int, params, tokens: bool = True, v: Optional[DecView] = None,
                embed_next: bool = False) -> None:
        if embed_next:
            raise ValueError("the fp32 path has no fused select + embedding (fused_select is off)")
        super()._select(R, params, tokens, v)
