"""WhisperEngine: HBM-resident weights and activations, and the hot path as a sequence of C-ABI calls.

Stage map (reference executed path -> this engine):
  WhisperFeatureExtractor (host CPU in the reference)            -> logmel()          tw_logmel
  WhisperEncoder.forward  (modeling_whisper.py:592-646)          -> encode()          im2col + GEMM + LN + attention
  cross-attention K/V of EncoderDecoderCache (:312-335)          -> encode()          one stacked GEMM (CROSSKV)
  detect_language + _sample loop (generation_whisper.py:1610-1673,
    $TF/generation/utils.py:2783-2941)                          -> decode_pass()     decoder step + tw_logits_select
  seek loop of WhisperGenerationMixin.generate (:785-903)         -> generate()        host bookkeeping (segments.py)

Every compute stage is a HIP kernel from libtwhip.so; torch only provides device allocations, the
stream, and (optionally) hipGraph capture of the per-token decoder step.
"""
from __future__ import annotations

import contextlib
import ctypes
import dataclasses
import gc
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib, _ops, alignment
from .config import GenerationSettings, WhisperDims
from .frontend import CHUNK_SAMPLES, N_FRAMES, dft_basis, mel_table, pack_k8
from .segments import (FallbackConfig, condition_prefixes, fallback_sequence, need_fallback, retrieve_segment,
                       segment_slices, strip_generated)
from .weights import PackedWeights

import functools

LN_EPS = 1e-5
S_ENC = 1500


# Python's cyclic GC held off while a graph records (defence in depth): a collection inside a capture that finds an
# unreachable engine in a reference cycle runs its graphs' / events' finalizers (HIP destroys, illegal while a stream
# captures), which aborted a full GPU suite run in r04ae. The cause is gone — engines hold no reference cycles (the
# encoder pump is dropped in run_batches' finally, step hooks are reset by their setters) and WhisperEngine.close()
# releases graphs, events and buffers in order — and tests/test_gpu_capture.py captures with the guard off
# (CAPTURE_GC_GUARD = False) after dropping an engine, with a collection forced inside the capture.
CAPTURE_GC_GUARD = True


@contextlib.contextmanager
def _capture(g: "torch.cuda.CUDAGraph", stream):
    """torch.cuda.graph, with the cyclic GC held off while the graph records when CAPTURE_GC_GUARD is set."""
    guard = CAPTURE_GC_GUARD
    was = gc.isenabled()
    if guard:
        gc.collect()
        gc.disable()
    try:
        with torch.cuda.graph(g, stream=stream):
            yield
    finally:
        if guard and was:
            gc.enable()


# how the decode loop waits for a queued step: polling the event rather than a blocking event synchronize, whose
# wake-up latency depends on the runtime's scheduling mode (a process that has an RCCL communicator up paid ~10 ms per
# bench step with the blocking wait: profiles/r05l_*). The poll yields (sleep(0), which releases the GIL: the C4
# diarizer thread keeps running) for the first _SPIN_POLLS checks — a decode step is ~0.4-0.7 ms — and then backs off
# to 50 us sleeps, so a long wait does not hold a host core at 100 % beside other ranks' host work.
_SPIN_POLLS = 2000


def _wait(ev: "torch.cuda.Event") -> None:
    n = 0
    while not ev.query():
        time.sleep(0 if n < _SPIN_POLLS else 5e-5)
        n += 1


def _pad256(n: int) -> int:
    return (n + 255) // 256 * 256
DEC_SPLITS = 4   # split-K factor of the decoder's d_model-wide projections (out_proj, fc2); 2 or 8: bench 93.0-93.4 / 92.8-95.6 vs 90.4-90.5 ms (profiles/r05ag_dec_splits_ab.txt)
# rows per decoder view: the packed GEMVs stream each weight byte once for up to 64 rows (four 16-row m-tiles; config
# 5's 64 windows, beam-5 over 12 windows); more rows run as consecutive views
VIEW_ROWS = 64


def on_engine_streams(fn):
    """Public engine calls run on the engine's own streams: ordered after the caller's current stream on entry,
    and the caller's stream waits for the engine's decoder stream on exit (so torch ops the caller issues on
    its stream see the results). Nested calls are already on the engine stream."""

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        if self.closed:
            raise RuntimeError("WhisperEngine is closed")
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream in self._own_streams:
            return fn(self, *args, **kwargs)
        self.stream.wait_stream(cur)
        try:
            with torch.cuda.stream(self.stream):
                return fn(self, *args, **kwargs)
        finally:
            cur.wait_stream(self.stream)

    return wrapper


@dataclasses.dataclass
class DecView:
    """Decoder rows [r0, r0 + n) of the engine batch: views of the per-row decoder buffers, their own split-K
    partial buffer and the HIP stream their steps launch on. The full batch is one view; the generation loop
    splits it into chains that run concurrently (each chain's kernels are latency-bound, so two chains fill
    each other's gaps)."""
    r0: int
    n: int
    stream: torch.cuda.Stream
    xd: torch.Tensor
    qkvd: torch.Tensor
    qd: torch.Tensor
    attd: torch.Tensor
    logits: torch.Tensor
    parts: torch.Tensor
    sel_ws: torch.Tensor
    state: torch.Tensor
    tokens: torch.Tensor
    ids: torch.Tensor
    pos: torch.Tensor
    hp: torch.Tensor   # packed-activation LayerNorm output (tw_gemv_packed A operand), <= VIEW_ROWS rows
    fp: torch.Tensor   # packed-activation fc1 output (fc2's A operand)
    fsync: Optional[torch.Tensor] = None  # tw_dec_fused's counter words for this view's launches


class _EncoderPump:
    """Paced queueing of a pipelined encoder prefetch (run_batches). ROCm's launch call costs ~60 us of host time
    once a queue holds more than a few ms of pending work (~7 us otherwise; measured with rocprofv3
    --hip-runtime-trace), and a decode step is 49 launches replayed node by node from the host: queueing the whole
    next-batch encoder up front made every launch of the overlapped decode steps slow (2.8 ms per step instead of
    ~0.5). The pump instead queues the encoder one chunk (conv stem / layer) at a time, keeping at most `ahead`
    chunks pending on enc_stream, and is called from the decode loop between steps."""

    def __init__(self, eng: "WhisperEngine", steps, ahead: int = 2):
        self.eng, self.steps, self.ahead = eng, steps, ahead
        self.pending: List[torch.cuda.Event] = []
        self.done = False

    def __call__(self) -> bool:
        """Queue chunks while fewer than `ahead` are unfinished; True if anything was queued."""
        queued = False
        while not self.done:
            while self.pending and self.pending[0].query():
                self.pending.pop(0)
            if len(self.pending) >= self.ahead:
                break
            self._one()
            queued = True
        return queued

    def _one(self) -> None:
        try:
            next(self.steps)
        except StopIteration:
            self.done = True
            return
        ev = torch.cuda.Event()
        ev.record(self.eng.enc_stream)
        self.pending.append(ev)

    def drain(self) -> None:
        while not self.done:
            self._one()
        self.pending.clear()


def fallback_row_key(window: int, pass_no: int, fi: int) -> int:
    """The fallback sampler's row key (int32): one counter-based noise stream per (global window, seek pass,
    temperature index)."""
    if not (0 <= int(pass_no) < 1024 and 0 <= int(fi) < 16):  # (fields would alias another row's noise stream)
        raise ValueError(f"sampler key fields out of range: pass {pass_no} (< 1024), temperature index {fi} (< 16)")
    key = (int(window) * 1024 + int(pass_no)) * 16 + int(fi)
    if not 0 <= key < 2 ** 31:
        raise ValueError(f"sampler key out of range: window {window}, pass {pass_no}")
    return key


@dataclasses.dataclass
class PassResult:
    tokens: List[List[int]]      # generated tokens per row (as _sample returns them, before stripping)
    lang_ids: Optional[List[int]]
    token_ts: Optional[List[np.ndarray]] = None  # per row, token-level times (prompt zeros first; word timestamps)
    sum_logprob: Optional[List[float]] = None  # per row, sum of the chosen tokens' log-probs (sample_pass)
    no_speech_prob: Optional[List[float]] = None  # per row, softmax at the SOT position of <|nospeech|> (sample_pass)


class WhisperEngine:
    def __init__(self, weights: PackedWeights, gen: GenerationSettings, max_batch: int = 24,
                 device: str = "cuda", use_graphs: bool = True, max_beams: int = 1,
                 enc_fp8: Optional[bool] = None):
        _lib.load()
        self.ops = _ops.load()  # torch.ops.tw (the encoder path's launches)
        # (False: the same encoder kernels through the C-ABI directly, without the dispatcher; bench-equal, r05o)
        self.enc_via_ops = True
        # Large-M GEMM kernel per encoder context (tw_gemm_set_variant): the 8-phase ping-pong k_gemm_8p (5) is 6-19 %
        # faster than k_gemm_big (1) on every encoder shape when it has the GPU to itself (scripts/gemm_bench.py), but
        # beside a running decode it slows the latency-bound decoder kernels more than it gains (bench step 117.1 vs
        # 113.4 ms). An encoder chunk that runs alone uses 5, one queued beside a decode (run_batches' overlap) uses 1.
        # The encoder attention beside a decode reserves LDS for one workgroup per CU (tw_attn_set_lds_pad 4) so the
        # decoder's kernels find free wave slots.
        d = weights.dims
        d.validate()
        if self.F32 != (weights.conv1_w.dtype == torch.float32):
            raise ValueError(f"{type(self).__name__} needs {'f32' if self.F32 else 'bf16'} weights "
                             "(build_weights(..., dtype=...))")
        self.d, self.w, self.gen = d, weights, gen
        self.max_batch = max_batch
        # decoder rows: windows x beams (beam search decodes num_beams rows per window against one cross-K/V)
        self.max_beams = max(1, int(max_beams))
        self.max_rows = max_batch * self.max_beams
        self.device = torch.device(device)
        self.use_graphs = use_graphs
        # a high-priority decoder stream and a default-priority stream for the front end + encoder: the
        # MFMA-bound encoder of the next window batch fills the CUs the latency-bound decode of this one leaves idle,
        # and the dispatcher serves the decoder's small grids first (CU-masked partitions measured slower: DESIGN §4)
        self.stream = torch.cuda.Stream(self.device, priority=-1)
        self.enc_stream = torch.cuda.Stream(self.device, priority=0)
        self._enc_ev = [torch.cuda.Event(), torch.cuda.Event()]
        D, F, H, V, B = d.d_model, d.ffn, d.heads, d.vocab, max_batch
        dev, bf, f32, i32 = self.device, torch.bfloat16, torch.float32, torch.int32
        act = f32 if self.F32 else bf  # activation / cache dtype of the encoder and decoder
        c, s = dft_basis()
        self.basis_cos = torch.from_numpy(pack_k8(c)).to(dev)
        self.basis_sin = torch.from_numpy(pack_k8(s)).to(dev)
        self.mel_fb = torch.from_numpy(pack_k8(mel_table(d.n_mels))).to(dev)
        # front end
        self.wave = torch.zeros(B, CHUNK_SAMPLES, dtype=f32, device=dev)
        self.feats_buf = torch.zeros(2, B, d.n_mels, N_FRAMES, dtype=f32, device=dev)  # [slot]
        self.feats = self.feats_buf[0]
        self.maxkeys = torch.zeros(B, dtype=torch.int32, device=dev)
        # encoder activations
        M3, M15 = B * N_FRAMES, B * S_ENC
        self.a1 = torch.empty(M3, weights.kpad1, dtype=act, device=dev)
        # conv1's output with one row in front: tw_conv2_gemm reads it in place as an operand of row stride 2 D
        # starting one row early (the t = 0 rows it then recomputes; the row in front only has to be readable)
        self._h1_rows = torch.zeros(M3 + 1, D, dtype=act, device=dev)
        self.h1 = self._h1_rows[1:]
        # (True: materialise conv2's im2col operand, 276 MB at B = 24, as before round 4; the f32 path always does)
        self._conv2_im2col = False
        self.a2 = torch.empty(M15, 3 * D, dtype=act, device=dev) if self._conv2_im2col or self.F32 else None
        self.x = torch.empty(M15, D, dtype=f32, device=dev)
        self.hln = torch.empty(M15, D, dtype=act, device=dev)
        self.qkv = torch.empty(M15, 3 * D, dtype=act, device=dev)
        self.att = torch.empty(M15, D, dtype=act, device=dev)
        self.ffn = torch.empty(M15, F, dtype=act, device=dev)
        # cross-attention K/V of the encoded windows, one buffer per pipeline slot
        # BASELINE config 5: the encoder projections on MX fp8 operands (tw_gemm_mx); TW_ENC_FP8=1 (or enc_fp8=True)
        self.enc_fp8 = (os.environ.get("TW_ENC_FP8", "0") == "1") if enc_fp8 is None else bool(enc_fp8)
        if self.F32 and self.enc_fp8:
            raise ValueError("the fp32 path has no MX fp8 encoder")
        self.enc_mx: List[Dict[str, tuple]] = []
        if self.enc_fp8:
            u8 = torch.uint8
            self.m15p = _pad256(M15)
            self.hq = torch.empty(M15, D, dtype=u8, device=dev)
            self.hq_s = torch.zeros(D // 128, self.m15p, 4, dtype=u8, device=dev)
            self.attq = torch.empty(M15, D, dtype=u8, device=dev)
            self.attq_s = torch.zeros(D // 128, self.m15p, 4, dtype=u8, device=dev)
            self.ffnq = torch.empty(M15, F, dtype=u8, device=dev)
            self.ffnq_s = torch.zeros(F // 128, self.m15p, 4, dtype=u8, device=dev)
            with torch.cuda.device(self.device):
                self.enc_mx = [{k: self._quant_weight(getattr(L, k)) for k in ("wqkv", "wo", "w1", "w2")}
                               for L in weights.enc]
                torch.cuda.synchronize(self.device)
        self.cross_kv_buf = torch.empty(2, d.decoder_layers, 2, B, H, S_ENC, 64, dtype=act, device=dev)
        self.cross_kv = self.cross_kv_buf[0]
        self._slot = 0  # slot the decoder reads
        # decoder state (max_rows = max_batch * max_beams rows)
        T = d.max_target_positions
        B = self.max_rows
        self.kcache = torch.zeros(d.decoder_layers, B, H, T, 64, dtype=act, device=dev)
        self.vcache = torch.zeros(d.decoder_layers, B, H, T, 64, dtype=act, device=dev)
        self.xd = torch.empty(B, D, dtype=f32, device=dev)
        self.qkvd = torch.empty(B, 3 * D, dtype=act, device=dev)
        self.qd = torch.empty(B, D, dtype=act, device=dev)
        self.attd = torch.empty(B, D, dtype=act, device=dev)
        self.logits = torch.empty(B, V, dtype=f32, device=dev)
        self.parts = torch.empty(DEC_SPLITS, B, D, dtype=f32, device=dev)   # split-K partials (decoder)
        self.sel_ws = torch.empty(B, _lib.TW_SELECT_WS_PER_ROW, dtype=f32, device=dev)
        self.state = torch.zeros(B, _lib.TW_STATE_STRIDE, dtype=i32, device=dev)
        self.tokens = torch.zeros(B, T, dtype=i32, device=dev)
        self.ids = torch.zeros(B, dtype=i32, device=dev)
        self.pos = torch.zeros(B, dtype=i32, device=dev)
        self.row_map = torch.zeros(max_batch, dtype=i32, device=dev)
        self.seek = torch.zeros(max_batch, dtype=i32, device=dev)
        self.dec_row_map = torch.zeros(B, dtype=i32, device=dev)  # decoder row -> cross-K/V row (beam search)
        self._use_dec_row_map = False
        self._row_group = 1
        self._xws: Optional[torch.Tensor] = None
        self._kv_tab: Optional[torch.Tensor] = None  # beam pass: the self-attention K/V position table
        self._long: Optional[dict] = None  # long-form input features (set_long_input)
        # prompts conditioned on previous segments (condition_on_prev_tokens): per row the left-pad count of the pass's
        # prefix; while _masked, the self-attention masks those positions (tw_attn_decode_self_masked)
        self._kv_start = torch.zeros(self.max_rows, dtype=torch.int32, device=dev)
        self._masked = False
        # the library's (tw_gemv_set_wide_slices, tw_gemv_set_variant) state (its defaults) and whether the decoder's
        # layers run as one persistent launch (tw_dec_fused) in the current pass
        self._dec_ctx = (1, 0, False)
        self._fused_dims = (not self.F32 and bool(_lib.load().tw_dec_fused_supported(D, H, d.ffn, 1)))
        self._fused_tab: Optional[torch.Tensor] = None  # device TwDecLayerW table (below, with the packed weights)
        self._fused_err = torch.zeros(4, dtype=torch.int32, device=dev)  # sticky phase-timeout word
        self._fused_xpart = (torch.empty(int(_lib.load().tw_dec_fused_xpart_bytes(32)) // 4, dtype=torch.float32,
                                         device=dev) if self._fused_dims else None)  # cross-attention slice states
        self._beam: Optional[dict] = None  # beam-search buffers, allocated on first use
        self._align: Optional[dict] = None  # token-level timestamps: alignment-head attention recording
        self._align_buf: Optional[torch.Tensor] = None
        self.suppress_bits = torch.zeros((V + 31) // 32, dtype=torch.int32, device=dev)
        self.set_suppress_tokens(gen.suppress_tokens)
        # concurrent decode chains in the generation loop (measured: two 12-row chains on two streams run no faster
        # than one 24-row chain on MI355X, so one by default; re-measured in round 3 for a pass with no encoder
        # beside it, scripts/exp/chains_ab.py: 15 rows 48.3 ms with one chain vs 52.7-194 ms with two, 24 rows 57.4 vs
        # 50.7-56.2 ms: no dependable gain)
        self.n_chains = 1
        self._chain_streams = [torch.cuda.Stream(self.device, priority=-1) for _ in range(self.n_chains)]
        self._own_streams = {x.cuda_stream for x in [self.stream, self.enc_stream] + self._chain_streams}
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._chain_cache: Dict[tuple, List[DecView]] = {}
        self._pump: Optional[_EncoderPump] = None  # paced next-batch encoder (run_batches)
        # decode steps queued ahead of the host before it pumps encoder chunks or waits, and encoder chunks pending
        # beside a decode: 1 and 2 (queue depths 1-3 re-measured within +-0.5 %)
        self.dec_ahead = 1
        self.pump_ahead = 2
        # greedy steps end with the fused select + next-step embedding + first LayerNorm (tw_logits_select_embed):
        # 47 launches per token instead of 49 (False: the separate launches; the tests check both decode alike)
        self.fused_select = not self.F32
        # decoder steps per graph replay in the generation loop: alone (no encoder chunks pumped between steps) and
        # beside run_batches' encoder pump
        self.graph_steps_alone = 1
        self.graph_steps_beside = 1
        # the prompt phase of a decode pass replayed as one captured graph (False: eager)
        self.prompt_graph = True
        # encoder attention kernel (tw_attn_set_variant) and its LDS cap in 16 KiB units (tw_attn_set_lds_pad) for an
        # encoder chunk alone / beside a running decode
        self.attn_kernel = (32, 32)  # k_attn_enc5 (round 4; 16 = k_attn_enc4, bit-identical to the enc2 form)
        self.attn_pad = (0, 4)
        # the encoder LayerNorm's LDS request in KiB (tw_layernorm_set_lds_pad), alone / beside a decode
        self.ln_pad = (0, 0)
        # run_batches encodes batch k+1 beside the decode of batch k (sequential 138.6 vs overlapped 114.5 ms per
        # bench step, round 1); False: strictly in turn
        self.overlap = True
        # decoder projections in the packed fragment layout (tw_pack_weight; +~342 MB at large-v3-turbo): every
        # wave-load of the per-token GEMVs is one contiguous 1 KiB fragment
        self.dec_p: List[Dict[str, torch.Tensor]] = []
        self.emb_p: Optional[torch.Tensor] = None
        if not self.F32:  # (the fp32 path's decoder runs tw_gemm_f32 on the row-major weights)
            with torch.cuda.device(self.device):
                self.dec_p = [{k: self._pack(getattr(L, k)) for k in ("wqkv", "wo", "wq_x", "wo_x", "w1", "w2")}
                              for L in weights.dec]
                self.emb_p = self._pack(weights.emb)
                if self._fused_dims:
                    self._fused_tab = self._fused_table()
                torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ lifetime
    closed = False
    F32 = False  # the fp32 arithmetic path (twamd/engine_f32.py WhisperEngineF32)

    def close(self) -> None:
        """Release the engine's GPU state in order, deterministically (no finalizer left for the cyclic GC): wait for
        its streams, destroy every captured graph (newest first), drop timers / events, the decode views and the
        encoder pump, then the buffers and weights (back to torch's caching allocator). The engine is unusable
        afterwards; a second close() is a no-op. Also the context-manager exit."""
        if self.closed:
            return
        for st in [self.stream, self.enc_stream] + list(getattr(self, "_chain_streams", [])):
            st.synchronize()
        for key in reversed(list(self._graphs)):
            self._graphs.pop(key).reset()
        self._graphs.clear()
        self._pump = None
        self.step_hook = None
        self.pass_events = None
        self.replay_host = None
        self.timers = None
        self._enc_ev = []
        self._chain_cache.clear()
        keep = {"d", "gen", "max_batch", "max_beams", "max_rows", "device", "closed", "_own_streams"}
        for name in list(vars(self)):
            if name not in keep and isinstance(getattr(self, name), (torch.Tensor, list, dict, tuple)):
                setattr(self, name, None)
        self.w = None
        self.closed = True

    def __enter__(self) -> "WhisperEngine":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def _quant_weight(self, W: torch.Tensor) -> tuple:
        """bf16 [N][K] -> (fp8 [N][K], e8m0 scales [K/128][Np][4], Np) in the MX layout of tw_gemm_mx."""
        N, K = W.shape
        Np = _pad256(N)
        q = torch.empty(N, K, dtype=torch.uint8, device=self.device)
        sc = torch.zeros(K // 128, Np, 4, dtype=torch.uint8, device=self.device)
        _lib.call("tw_quant_mx", W.data_ptr(), N, K, K, q.data_ptr(), sc.data_ptr(), Np,
                  torch.cuda.current_stream(self.device).cuda_stream)
        return q, sc, Np

    def _gemm_mx(self, A, As, Wt, M, N, K, epi, out, bias=None, sout=None, stream=None):
        """MX fp8 GEMM: A fp8 [M][K] + scales As [K/128][m15p][4]; Wt = _quant_weight(W)."""
        st = stream or self.stream
        Wq, Ws, Np = Wt
        rec = self._begin_timer(("gemm_mx", epi), 2.0 * M * N * K, st)
        _lib.call("tw_gemm_mx", A.data_ptr(), As.data_ptr(), Wq.data_ptr(), Ws.data_ptr(), M, N, K, K, K, self.m15p,
                  Np, epi, out.data_ptr(), N, _lib.ptr(bias), _lib.ptr(sout), self.m15p if sout is not None else 0,
                  st.cuda_stream)
        self._end_timer(rec, st)

    def _pack(self, W: torch.Tensor) -> torch.Tensor:
        N, K = W.shape
        Wp = torch.empty((N + 15) // 16 * 16 * K, dtype=torch.bfloat16, device=self.device)
        _lib.call("tw_pack_weight", W.data_ptr(), N, K, K, Wp.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return Wp

    def _gemv(self, A, a_packed: bool, Wp, M, N, K, epi, out, v: DecView, bias=None, splits=1, ldo=None):
        rec = self._begin_timer(("gemv_packed", epi), 2.0 * M * N * K, v.stream)
        _lib.call("tw_gemv_packed", A.data_ptr(), int(a_packed), K, Wp.data_ptr(), M, N, K, epi, out.data_ptr(),
                  ldo if ldo is not None else N, _lib.ptr(bias), splits, v.stream.cuda_stream)
        self._end_timer(rec, v.stream)

    def _resid_ln_p(self, R, nparts, bias, g, b, v: DecView):
        """xd += bias + sum(parts[:nparts]); hp = LayerNorm(xd) as a packed activation."""
        _lib.call("tw_resid_layernorm_packed", v.xd.data_ptr(), v.parts.data_ptr() if nparts else None, nparts,
                  _lib.ptr(bias), _lib.ptr(g), _lib.ptr(b), R, self.d.d_model, LN_EPS, v.hp.data_ptr(),
                  v.stream.cuda_stream)

    def set_suppress_tokens(self, tokens: Sequence[int]) -> None:
        """SuppressTokensLogitsProcessor's list as a device bitmask (in place: captured graphs stay valid)."""
        V = self.d.vocab
        bits = np.zeros((V + 31) // 32, np.uint32)
        for t in tokens:
            if 0 <= t < V:
                bits[t >> 5] |= np.uint32(1 << (t & 31))
        self.suppress_bits.copy_(torch.from_numpy(bits.view(np.int32)))
        self.gen.suppress_tokens = list(tokens)

    # ------------------------------------------------------------------ helpers
    @property
    def _s(self) -> int:
        return self.stream.cuda_stream

    _enc_cur = None  # the stream handle an encoder chunk's launches are issued under (_enc_chunk_ctx)

    def _on(self, st):
        """The context a torch.ops.tw call needs to launch on stream st (the ops use the current stream): nothing
        inside an encoder chunk already entered on st."""
        if self._enc_cur == st.cuda_stream or torch.cuda.current_stream(self.device).cuda_stream == st.cuda_stream:
            return contextlib.nullcontext()
        return torch.cuda.stream(st)

    @contextlib.contextmanager
    def _enc_chunk_ctx(self, st):
        """One encoder chunk's launches (between two yields of _encode_chunks) under one stream context."""
        with torch.cuda.stream(st):
            self._enc_cur = st.cuda_stream
            try:
                yield
            finally:
                self._enc_cur = None

    @staticmethod
    def _rows(t, M):
        return t if t.shape[0] == M else t[:M]

    def _gemm(self, A, W, M, N, K, epi, out, bias=None, aux=None, aux_rows=0, kv_geom=None, stream=None):
        """torch.ops.tw.gemm_bf16_out on A[:M] (K columns) x W^T (N rows) into out[:M] (CROSSKV: the head-major
        cross-K/V block, kv_geom = (S, B, D, H))."""
        st = stream or self.stream
        rec = self._begin_timer(("gemm_skinny" if M <= 32 else "gemm_big", epi), 2.0 * M * N * K, st)
        assert A.shape[1] == K and W.shape[0] == N and W.shape[1] == K
        if self.enc_via_ops:
            with self._on(st):
                self.ops.gemm_bf16_out(self._rows(A, M), W, epi, out if epi == _lib.TW_EPI_CROSSKV else
                                       self._rows(out, M), bias, aux, aux_rows,
                                       list(kv_geom) if kv_geom is not None else None)
        else:
            _lib.call("tw_gemm_bf16", A.data_ptr(), W.data_ptr(), M, N, K, K, K, epi, out.data_ptr(), N,
                      _lib.ptr(bias), _lib.ptr(aux), aux_rows,
                      None if kv_geom is None else (ctypes.c_int * 4)(*kv_geom), st.cuda_stream)
        self._end_timer(rec, st)

    # per-launch HIP-event timing of kernel families (bench roofline; off by default). timer_families: the
    # family names (key[0]) to time, None = all.
    timers: Optional[dict] = None
    timer_families: Optional[set] = None

    def _begin_timer(self, key, work, stream=None):
        """HIP events on the stream the kernel is launched on (none inside a graph capture: a captured launch's
        events would time the capture, not the replay)."""
        if self.timers is None or (self.timer_families is not None and key[0] not in self.timer_families):
            return None
        if torch.cuda.is_current_stream_capturing():
            return None
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream or self.stream)
        return (key, work, a, b)

    def _end_timer(self, rec, stream=None):
        if rec is None:
            return
        key, work, a, b = rec
        b.record(stream or self.stream)
        self.timers.setdefault(key, []).append((work, a, b))

    def timer_summary(self) -> dict:
        """{family: (launches, total_work, total_ms)} after a synchronize."""
        torch.cuda.synchronize(self.device)
        out = {}
        for k, lst in (self.timers or {}).items():
            out[k] = (len(lst), sum(w for w, _, _ in lst), sum(a.elapsed_time(b) for _, a, b in lst))
        return out

    def _ln(self, x, g, b, M, out, stream=None):
        if not self.enc_via_ops:
            _lib.call("tw_layernorm", x.data_ptr(), g.data_ptr(), b.data_ptr(), M, self.d.d_model, LN_EPS,
                      out.data_ptr(), (stream or self.stream).cuda_stream)
            return
        with self._on(stream or self.stream):
            self.ops.layernorm_out(self._rows(x, M), g, b, LN_EPS, self._rows(out, M))

    # ------------------------------------------------------------------ streams / slots
    def _pump_drain(self) -> None:
        if self._pump is not None:
            self._pump.drain()

    def _enc_begin(self, sync: bool):
        """Front-end/encoder work goes to enc_stream. sync: it is ordered after everything already queued on the
        decoder stream (host writes of wave/row_map/seek made there), and _enc_end makes the decoder stream wait
        for it; async (pipelined prefetch): independent of the decoder stream."""
        if sync:
            self.enc_stream.wait_stream(self.stream)
        return self.enc_stream

    def _enc_end(self, sync: bool, slot: int):
        self._enc_ev[slot].record(self.enc_stream)
        if sync:
            self.stream.wait_stream(self.enc_stream)

    def _view(self, r0: int = 0, n: Optional[int] = None, stream=None, parts=None) -> DecView:
        n = self.max_rows - r0 if n is None else n
        if stream is None and parts is None:  # the default views are cached: graphs capture their buffers
            key = ("view", r0, n)
            if key not in self._chain_cache:
                self._chain_cache[key] = self._view(r0, n, self.stream, self.parts)
            return self._chain_cache[key]
        sl = slice(r0, r0 + n)
        if n > VIEW_ROWS:
            raise ValueError(f"decoder views hold <= {VIEW_ROWS} rows (packed GEMV), got {n}")
        # per-view packed scratch (rows 0..n-1 of the view; pad rows zero)
        # (fp32 path: the row-major f32 LayerNorm / fc1 outputs)
        adt = torch.float32 if self.F32 else torch.bfloat16
        hp = torch.zeros(VIEW_ROWS * self.d.d_model, dtype=adt, device=self.device)
        fp = torch.zeros(VIEW_ROWS * self.d.ffn, dtype=adt, device=self.device)
        fsync = (torch.zeros(int(_lib.load().tw_dec_fused_sync_bytes()) // 4, dtype=torch.int32, device=self.device)
                 if self._fused_dims else None)
        return DecView(r0, n, stream or self.stream, self.xd[sl], self.qkvd[sl], self.qd[sl], self.attd[sl],
                       self.logits[sl], self.parts if parts is None else parts, self.sel_ws[sl], self.state[sl],
                       self.tokens[sl], self.ids[sl], self.pos[sl], hp, fp, fsync)

    @on_engine_streams
    def set_long_input(self, wave: Optional[torch.Tensor]) -> int:
        """Long-form source (generate() over one input longer than 30 s, the ASR pipeline without chunk_length_s):
        the log-mel of the whole input (tw_logmel_long: one STFT, the max - 8 clamp over the whole input, as the
        feature extractor with truncation=False / padding="longest") becomes the encoder's feature row 0 until
        set_long_input(None). Returns its frame count T (generate()'s total_input_frames = max_frames)."""
        if wave is None:
            self._long = None
            return 0
        wave = wave.to(self.device, torch.float32).contiguous()
        n = int(wave.numel())
        T = n // 160
        ld = max(T, N_FRAMES)
        feats = torch.zeros(self.d.n_mels, ld, dtype=torch.float32, device=self.device)
        key = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.call("tw_logmel_long", wave.data_ptr(), n, self.basis_cos.data_ptr(), self.basis_sin.data_ptr(),
                  self.mel_fb.data_ptr(), self.d.n_mels, feats.data_ptr(), ld, key.data_ptr(),
                  torch.cuda.current_stream(self.device).cuda_stream)
        mf = torch.tensor([T], dtype=torch.int32, device=self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.enc_stream.wait_stream(torch.cuda.current_stream(self.device))
        self._long = {"feats": feats, "ld": ld, "max_frames": mf, "T": T, "wave": wave}
        return T

    def use_slot(self, slot: int) -> None:
        """Point the decoder at the cross-K/V (and feature) buffers of pipeline slot `slot`."""
        self._slot = slot
        self.cross_kv = self.cross_kv_buf[slot]
        self.feats = self.feats_buf[slot]

    # ------------------------------------------------------------------ front end
    @on_engine_streams
    def logmel(self, n: int, slot: Optional[int] = None, sync: bool = True) -> None:
        """feats[slot][:n] = log-mel of wave[:n] (each row one 30-s window, zero padded)."""
        slot = self._slot if slot is None else slot
        st = self._enc_begin(sync)
        with self._on(st):
            self.ops.logmel_out(self.wave[:n], self.basis_cos, self.basis_sin, self.mel_fb, self.d.n_mels,
                                self.feats_buf[slot][:n], self.maxkeys)
        self._enc_end(sync, slot)

    # ------------------------------------------------------------------ encoder
    @on_engine_streams
    def encode(self, R: int, row_map=True, seek=True, slot: Optional[int] = None, sync: bool = True,
               alone: bool = True) -> None:
        """Encoder over R windows: slot r reads feats[slot][row_map[r]][:, seek[r]:] (zero padded to 3000), then
        projects every decoder layer's cross-attention K/V into cross_kv_buf[slot] (batch stride R). Runs on
        enc_stream (see _enc_begin for `sync`)."""
        self._pump_drain()  # a paced prefetch shares the encoder's activation buffers: queue all of it first
        for _ in self._encode_steps(R, row_map, seek, slot, sync, alone=alone):
            pass

    # large-M GEMM kernel of an encoder chunk that runs alone (tw_gemm_set_variant): 6 = the persistent k_gemm_8pp (the
    # next tile's first K-tile DMA'd under the epilogue: encoder layer 1404 -> 1332 us at 24 windows,
    # profiles/r05v_gemm_variant_ab.txt), 5 = k_gemm_8p
    gemm_alone = 6
    # beside a decode: k_gemm_big (1: 184 VGPRs, so a decoder wave fits on every SIMD of every CU), or the persistent
    # kernel on gemm_beside_cus CUs (6: the other CUs left to the decoder's kernels)
    gemm_beside = 1
    gemm_beside_cus = 224
    # MX fp8 GEMM kernel (tw_gemm_mx_set_variant) of config 5's encoder chunks alone / beside a decode: 0 = the
    # library's shape rule (k_gemm_mx for q/k/v, k_gemm_8p_mx for the rest: 180.7 vs 183.2 ms per step,
    # profiles/r05bb_mx_shape_rule_ab.txt), 8 = k_gemm_8p_mx everywhere (256 VGPRs), 1 = k_gemm_mx everywhere (182
    # VGPRs, so a decoder wave fits beside it — which does not pay: 188.6 vs 183.4 ms, profiles/r05ba_mx_beside_ab.txt)
    mx_alone = 0
    mx_beside = 0

    def _set_gemm_context(self, alone: bool) -> None:
        """Encoder kernels for the chunk about to be queued (see __init__): large-M GEMM gemm_alone alone, 1 beside a decode;
        the encoder attention capped at one workgroup per CU beside a decode (tw_attn_set_lds_pad: the decoder's
        kernels then find free wave slots; measured decoder GEMV 21.9 -> 5.6 us per launch beside it, bench step
        112.1 -> 108.5 ms), uncapped alone (the cap costs the attention itself 22 %)."""
        _lib.call("tw_gemm_set_variant", self.gemm_alone if alone else self.gemm_beside)
        _lib.call("tw_gemm_set_persistent_grid", 0 if alone else self.gemm_beside_cus)
        _lib.call("tw_attn_set_variant", self.attn_kernel[0 if alone else 1])
        _lib.call("tw_attn_set_lds_pad", self.attn_pad[0 if alone else 1])
        _lib.call("tw_layernorm_set_lds_pad", self.ln_pad[0 if alone else 1])
        if self.enc_fp8:
            _lib.call("tw_gemm_mx_set_variant", self.mx_alone if alone else self.mx_beside)

    def _encode_steps(self, R: int, row_map=True, seek=True, slot: Optional[int] = None, sync: bool = True,
                      alone: bool = True):
        """encode() as a generator that yields after the conv stem and after every layer, so a pipelined prefetch
        can queue the encoder a layer at a time (run_batches' _EncoderPump). Every launch names enc_stream.
        alone: no decode runs beside this encoder (picks the large-M GEMM kernel, re-applied after every yield)."""
        chunks = self._encode_chunks(R, row_map, seek, slot, sync)
        while True:
            self._set_gemm_context(alone)  # before each chunk is queued: the decode loop runs between chunks
            try:
                next(chunks)
            except StopIteration:
                break
            yield
        self._set_gemm_context(True)

    def _encode_chunks(self, R: int, row_map=True, seek=True, slot: Optional[int] = None, sync: bool = True):
        d, w = self.d, self.w
        slot = self._slot if slot is None else slot
        D, F, H = d.d_model, d.ffn, d.heads
        M3, M15 = R * N_FRAMES, R * S_ENC
        st = self._enc_begin(sync)
        s = st.cuda_stream
        # (one stream context per chunk, never across a yield: the caller runs there)
        with self._enc_chunk_ctx(st):
            if self._long is not None:  # a long-form input's features (set_long_input): one row of T frames
                lf = self._long
                _lib.call("tw_im2col_conv1_long", lf["feats"].data_ptr(), d.n_mels, lf["ld"],
                          lf["max_frames"].data_ptr(), self.row_map.data_ptr() if row_map else None,
                          self.seek.data_ptr(), R, w.kpad1, self.a1.data_ptr(), s)
            else:
                _lib.call("tw_im2col_conv1", self.feats_buf[slot].data_ptr(), d.n_mels,
                          self.row_map.data_ptr() if row_map else None, self.seek.data_ptr() if seek else None, R,
                          w.kpad1, self.a1.data_ptr(), s)
            self._gemm(self.a1, w.conv1_w, M3, D, w.kpad1, _lib.TW_EPI_GELU_BF16, self.h1, bias=w.conv1_b, stream=st)
            if self._conv2_im2col:
                _lib.call("tw_im2col_conv2", self.h1.data_ptr(), R, D, self.a2.data_ptr(), s)
                self._gemm(self.a2, w.conv2_w, M15, D, 3 * D, _lib.TW_EPI_GELU_POS_F32, self.x, bias=w.conv2_b,
                           aux=w.pos_enc, aux_rows=S_ENC, stream=st)
            else:
                rec = self._begin_timer(("gemm_big", _lib.TW_EPI_GELU_POS_F32), 2.0 * M15 * D * 3 * D, st)
                _lib.call("tw_conv2_gemm", self.h1.data_ptr(), R, D, w.conv2_w.data_ptr(), w.conv2_b.data_ptr(),
                          w.pos_enc.data_ptr(), self.x.data_ptr(), s)
                self._end_timer(rec, st)
        yield
        if self.enc_fp8:
            yield from self._encode_layers_mx(R, st)
        for L in ([] if self.enc_fp8 else w.enc):
            with self._enc_chunk_ctx(st):
                self._ln(self.x, L.ln1_g, L.ln1_b, M15, self.hln, stream=st)
                self._gemm(self.hln, L.wqkv, M15, 3 * D, D, _lib.TW_EPI_BF16, self.qkv, bias=L.bqkv, stream=st)
                rec = self._begin_timer(("attn_encoder", 0), 4.0 * S_ENC * S_ENC * 64 * H * R, st)
                if self.enc_via_ops:
                    with self._on(st):
                        self.ops.attn_encoder_out(self._rows(self.qkv, M15), R, H, self._rows(self.att, M15))
                else:
                    _lib.call("tw_attn_encoder", self.qkv.data_ptr(), R, S_ENC, H, self.att.data_ptr(), s)
                self._end_timer(rec, st)
                self._gemm(self.att, L.wo, M15, D, D, _lib.TW_EPI_RESID_F32, self.x, bias=L.bo, stream=st)
                self._ln(self.x, L.ln2_g, L.ln2_b, M15, self.hln, stream=st)
                self._gemm(self.hln, L.w1, M15, F, D, _lib.TW_EPI_GELU_BF16, self.ffn, bias=L.b1, stream=st)
                self._gemm(self.ffn, L.w2, M15, D, F, _lib.TW_EPI_RESID_F32, self.x, bias=L.b2, stream=st)
            yield
        with self._enc_chunk_ctx(st):
            self._ln(self.x, w.enc_ln_g, w.enc_ln_b, M15, self.hln, stream=st)  # encoder last_hidden_state (bf16)
            geom = (S_ENC, R, D, H)
            self._gemm(self.hln, w.wkv_x, M15, d.decoder_layers * 2 * D, D, _lib.TW_EPI_CROSSKV,
                       self.cross_kv_buf[slot], bias=w.bkv_x, kv_geom=geom, stream=st)
        self._enc_end(sync, slot)

    def _encode_layers_mx(self, R: int, st):
        """The 32 encoder layers of config 5: LayerNorms emit MX fp8 (tw_layernorm_mx), q/k/v/o and fc1/fc2 run on
        tw_gemm_mx, the attention core stays bf16 and stores its output as MX fp8 (tw_attn_encoder_mx), fc1's GELU
        output is quantised in its epilogue."""
        d, w = self.d, self.w
        D, F, H = d.d_model, d.ffn, d.heads
        M15, s = R * S_ENC, st.cuda_stream
        for L, Q in zip(w.enc, self.enc_mx):
            _lib.call("tw_layernorm_mx", self.x.data_ptr(), L.ln1_g.data_ptr(), L.ln1_b.data_ptr(), M15, D, LN_EPS,
                      self.hq.data_ptr(), self.hq_s.data_ptr(), self.m15p, s)
            self._gemm_mx(self.hq, self.hq_s, Q["wqkv"], M15, 3 * D, D, _lib.TW_EPI_BF16, self.qkv, bias=L.bqkv,
                          stream=st)
            rec = self._begin_timer(("attn_encoder", 0), 4.0 * S_ENC * S_ENC * 64 * H * R, st)
            _lib.call("tw_attn_encoder_mx", self.qkv.data_ptr(), R, S_ENC, H, self.attq.data_ptr(),
                      self.attq_s.data_ptr(), self.m15p, s)
            self._end_timer(rec, st)
            self._gemm_mx(self.attq, self.attq_s, Q["wo"], M15, D, D, _lib.TW_EPI_RESID_F32, self.x, bias=L.bo,
                          stream=st)
            _lib.call("tw_layernorm_mx", self.x.data_ptr(), L.ln2_g.data_ptr(), L.ln2_b.data_ptr(), M15, D, LN_EPS,
                      self.hq.data_ptr(), self.hq_s.data_ptr(), self.m15p, s)
            self._gemm_mx(self.hq, self.hq_s, Q["w1"], M15, F, D, _lib.TW_EPI_GELU_MX, self.ffnq, bias=L.b1,
                          sout=self.ffnq_s, stream=st)
            self._gemm_mx(self.ffnq, self.ffnq_s, Q["w2"], M15, D, F, _lib.TW_EPI_RESID_F32, self.x, bias=L.b2,
                          stream=st)
            yield

    def encoder_output(self, R: int) -> torch.Tensor:
        """Encoder last_hidden_state of the last encode() (bf16 view [R][1500][D])."""
        return self.hln[: R * S_ENC].view(R, S_ENC, self.d.d_model)

    # ------------------------------------------------------------------ decoder
    @on_engine_streams
    def decoder_step(self, R: int, with_logits: bool = True, v: Optional[DecView] = None, r_enc: Optional[int] = None,
                     pre_embedded: bool = False) -> None:
        """One token per row of view v (default: rows 0..R-1): ids[b] at position pos[b] -> logits[b] (f32).
        r_enc: the batch size the current cross-K/V was encoded with (its batch stride; default R).
        pre_embedded: the view's xd and first-layer LayerNorm output already hold this step's input (written by the
        previous step's fused select, _select(embed_next=True)); the step starts at layer 0's q/k/v projection.

        WhisperDecoder.forward / WhisperDecoderLayer.forward ($TF/models/whisper/modeling_whisper.py:690-795, 448-505)
        on the packed-GEMV path: the residual stream xd stays f32; LayerNorm outputs and fc1's GELU output are packed
        activations (the GEMVs' A operand), attention outputs stay row-major; every d_model-wide projection (self /
        cross out_proj, fc2) is a split-K partial product whose sum, bias and residual add are folded into the next
        LayerNorm launch."""
        if v is None and R > VIEW_ROWS:  # the packed decoder GEMVs take <= VIEW_ROWS rows: one view per VIEW_ROWS
            r_enc = R if r_enc is None else r_enc
            for r0 in range(0, R, VIEW_ROWS):
                n = min(VIEW_ROWS, R - r0)
                self.decoder_step(n, with_logits, self._view(r0, n), r_enc, pre_embedded)
            return
        v = v or self._view(0, R)
        r_enc = R if r_enc is None else r_enc
        d, w = self.d, self.w
        D, F, H, T = d.d_model, d.ffn, d.heads, d.max_target_positions
        st = v.stream
        s = st.cuda_stream
        if not pre_embedded:
            _lib.call("tw_embed_decoder", w.emb.data_ptr(), w.pos_dec.data_ptr(), v.ids.data_ptr(), v.pos.data_ptr(), R,
                      D, v.xd.data_ptr(), s)
        if self._fused_ok(R):  # the layers as one persistent launch (it recomputes layer 0's LayerNorm itself)
            self._fused_layers(R, r_enc, v)
            if with_logits:
                self._gemv(v.hp, True, self.emb_p, R, d.vocab, D, _lib.TW_EPI_F32, v.logits, v)
            return
        xkv_stride = 2 * r_enc * H * S_ENC * 64
        nparts, pbias = 0, None
        PART, K4 = _lib.TW_EPI_PARTIAL_F32, DEC_SPLITS
        # (the attention blocks with their LayerNorm / projection launches folded in, tw_attn_decode_self_q /
        # tw_attn_decode_cross_q, 31 launches per token, measured slower and archived: DESIGN §4, round 4)
        for li, L in enumerate(w.dec):
            P = self.dec_p[li]
            kc, vc = self.kcache[li, v.r0:].data_ptr(), self.vcache[li, v.r0:].data_ptr()
            if li or not pre_embedded:
                self._resid_ln_p(R, nparts, pbias, L.ln1_g, L.ln1_b, v)
            self._gemv(v.hp, True, P["wqkv"], R, 3 * D, D, _lib.TW_EPI_BF16, v.qkvd, v, bias=L.bqkv)
            ks = self._kv_start[v.r0:].data_ptr() if self._masked else None  # left-padded prompts (prefill)
            if self._kv_tab is not None:  # beam pass: histories through the position table
                if ks is not None:
                    _lib.call("tw_attn_decode_self_tab_masked", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc,
                              self._kv_tab.data_ptr(), v.r0, ks, v.attd.data_ptr(), s)
                else:
                    _lib.call("tw_attn_decode_self_tab", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc,
                              self._kv_tab.data_ptr(), v.r0, v.attd.data_ptr(), s)
            elif ks is not None:
                _lib.call("tw_attn_decode_self_masked", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc, ks,
                          v.attd.data_ptr(), s)
            else:
                _lib.call("tw_attn_decode_self", v.qkvd.data_ptr(), R, H, T, v.pos.data_ptr(), kc, vc,
                          v.attd.data_ptr(), s)
            self._gemv(v.attd, False, P["wo"], R, D, D, PART, v.parts, v, splits=K4)
            self._resid_ln_p(R, K4, L.bo, L.ln2_g, L.ln2_b, v)
            self._gemv(v.hp, True, P["wq_x"], R, D, D, _lib.TW_EPI_BF16, v.qd, v, bias=L.bq_x)
            ckv, rmap = self._cross_ptrs(li, xkv_stride, v)
            rec = self._begin_timer(("attn_decode_cross", 0), 2.0 * R * H * S_ENC * 64 * 2, st)  # K+V bytes read
            self._cross_attend(li, R, r_enc, rmap, ckv, v)
            self._end_timer(rec, st)
            self._gemv(v.attd, False, P["wo_x"], R, D, D, PART, v.parts, v, splits=K4)
            self._resid_ln_p(R, K4, L.bo_x, L.ln3_g, L.ln3_b, v)
            self._gemv(v.hp, True, P["w1"], R, F, D, _lib.TW_EPI_GELU_PACKED, v.fp, v, bias=L.b1)
            self._gemv(v.fp, True, P["w2"], R, D, F, PART, v.parts, v, splits=K4)
            nparts, pbias = K4, L.b2
        if with_logits:
            self._resid_ln_p(R, nparts, pbias, w.dec_ln_g, w.dec_ln_b, v)
            self._gemv(v.hp, True, self.emb_p, R, d.vocab, D, _lib.TW_EPI_F32, v.logits, v)

    def _cross_attend(self, li: int, R: int, r_enc: int, rmap, ckv, v: DecView) -> None:
        """Cross-attention of the view's rows; with token-level timestamps requested (self._align) the alignment
        heads of this layer also write their attention probabilities."""
        H, s = self.d.heads, v.stream.cuda_stream
        al = self._align
        if al is not None and li in al["layers"]:
            mask, slot0 = al["layers"][li]
            row_stride = al["n_steps"] * al["n_slots"] * S_ENC * 4
            _lib.call("tw_attn_decode_cross_probs", v.qd.data_ptr(), R, H, S_ENC, r_enc, rmap, ckv, v.attd.data_ptr(),
                      al["buf"].data_ptr() + v.r0 * row_stride, mask, slot0, al["n_slots"], v.pos.data_ptr(),
                      al["pos0"], al["n_steps"], s)
        elif self._row_group > 1 and rmap is not None:  # beam rows: one K/V read per window's beams
            g = self._row_group
            if self._xws is None:  # per-row key-slice states, rows at their global index (views never overlap)
                nbytes = int(_lib.load().tw_attn_decode_cross_grouped_ws_bytes(self.max_rows, H))
                self._xws = torch.empty(nbytes // 4, dtype=torch.float32, device=self.device)
            row_bytes = self._xws.numel() * 4 // self.max_rows
            _lib.call("tw_attn_decode_cross_grouped", v.qd.data_ptr(), R, H, S_ENC, r_enc, rmap, g, (g - v.r0 % g) % g,
                      ckv, self._xws.data_ptr() + v.r0 * row_bytes, v.attd.data_ptr(), s)
        else:
            _lib.call("tw_attn_decode_cross", v.qd.data_ptr(), R, H, S_ENC, r_enc, rmap, ckv, v.attd.data_ptr(), s)

    def _align_setup(self, R: int, pos0: int, n_steps: int) -> None:
        heads = self.gen.alignment_heads
        if not heads:
            raise ValueError("token-level timestamps need generation alignment_heads")
        layers: Dict[int, tuple] = {}
        slot = 0
        for li in sorted({l for l, _ in heads}):
            hs = sorted({h for l, h in heads if l == li})
            layers[li] = (sum(1 << h for h in hs), slot)
            slot += len(hs)
        order = [(l, h) for l in sorted(layers) for h in sorted({hh for ll, hh in heads if ll == l})]
        shape = (self.max_rows, n_steps, slot, S_ENC)
        buf = self._align_buf if getattr(self, "_align_buf", None) is not None else None
        if buf is None or buf.numel() < int(np.prod(shape)):
            buf = torch.empty(int(np.prod(shape)), dtype=torch.float32, device=self.device)
            self._align_buf = buf
        # slot order inside the buffer -> the order of generation_config.alignment_heads
        perm = [order.index((l, h)) for l, h in heads]
        self._align = {"layers": layers, "n_slots": slot, "pos0": pos0, "n_steps": n_steps, "buf": buf, "perm": perm}

    def _align_weights(self, R: int, n_rows: int) -> np.ndarray:
        """f32 [R][alignment heads][n_rows][S] of the generated tokens fed so far (steps 0 .. n_rows-1)."""
        al = self._align
        b = al["buf"][: R * al["n_steps"] * al["n_slots"] * S_ENC].view(R, al["n_steps"], al["n_slots"], S_ENC)
        w = b[:, :n_rows].permute(0, 2, 1, 3)[:, al["perm"]].float().cpu().numpy()
        return w

    def _cross_ptrs(self, li: int, xkv_stride: int, v: DecView):
        """This layer's [k|v][r_enc][H][S][64] block and the row map for the view's rows: identity rows start at
        the view's first row; with beam search every row reads its window's slot through dec_row_map."""
        H, esz = self.d.heads, self.cross_kv.element_size()
        base = self.cross_kv.data_ptr() + li * xkv_stride * esz
        if self._use_dec_row_map:
            return base, self.dec_row_map.data_ptr() + 4 * v.r0
        return base + v.r0 * H * S_ENC * 64 * esz, None

    def _select_params(self, mode: int, max_new: int, use_timestamps: bool = True) -> _lib.TwSelectParams:
        st, g = self.gen.special, self.gen
        p = _lib.TwSelectParams()
        p.V, p.eos, p.pad = self.d.vocab, st.eot, st.eot
        p.ts_begin, p.no_timestamps = st.timestamp_begin, st.notimestamps
        p.max_initial_ts = -1 if g.max_initial_timestamp_index is None else g.max_initial_timestamp_index
        p.use_timestamps = int(use_timestamps)
        p.max_new, p.mode = max_new, mode
        p.lo, p.hi = st.lang_begin, st.lang_end
        bs = list(g.begin_suppress_tokens or [])
        p.n_begin_suppress = len(bs)
        for i, t in enumerate(bs):
            p.begin_suppress[i] = t
        return p

    def _select(self, R: int, params: _lib.TwSelectParams, tokens: bool = True, v: Optional[DecView] = None,
                embed_next: bool = False) -> None:
        """Processors + greedy selection for the view's rows; embed_next: also the head of the next step (the chosen
        token's embedding into xd and layer 0's self_attn_layer_norm into the view's LN buffer, one fused launch)."""
        if v is None and R > VIEW_ROWS:  # per-row selection over the views decoder_step(R) ran (beam rows)
            for r0 in range(0, R, VIEW_ROWS):
                self._select(min(VIEW_ROWS, R - r0), params, tokens, self._view(r0, min(VIEW_ROWS, R - r0)), embed_next)
            return
        v = v or self._view(0, R)
        if embed_next:
            L0 = self.w.dec[0]
            _lib.call("tw_logits_select_embed", v.logits.data_ptr(), R, self.d.vocab, self.suppress_bits.data_ptr(),
                      ctypes.byref(params), v.state.data_ptr(), v.tokens.data_ptr() if tokens else None,
                      v.tokens.shape[1], v.ids.data_ptr(), v.pos.data_ptr(), v.sel_ws.data_ptr(),
                      self.w.emb.data_ptr(), self.w.pos_dec.data_ptr(), self.d.d_model, self.d.max_target_positions,
                      v.xd.data_ptr(), L0.ln1_g.data_ptr(), L0.ln1_b.data_ptr(), LN_EPS,
                      v.hp.data_ptr(), 1, v.stream.cuda_stream)
            return
        _lib.call("tw_logits_select", v.logits.data_ptr(), R, self.d.vocab, self.suppress_bits.data_ptr(),
                  ctypes.byref(params), v.state.data_ptr(), v.tokens.data_ptr() if tokens else None,
                  v.tokens.shape[1], v.ids.data_ptr(), v.pos.data_ptr(), v.sel_ws.data_ptr(), v.stream.cuda_stream)

    # Teacher-forcing hook of decode_pass (parity harness, tests/test_gpu_turbo.py and bench.py's parity leg):
    # hook(k, view) runs on the host after the step that produced generated position k (view None: the prompt's last
    # step, all rows), with that step's logits in place and the stream idle; it may overwrite `ids` of the view's rows
    # and re-run the head of the next step (embed_head) so the next replay of the captured step consumes the forced
    # token instead of the one the selection chose. None in normal decoding.
    step_hook = None
    # measurement: a list to which decode_pass appends (start event, end event, steps) of its generation loop, and the
    # host seconds of each graph replay of the passes measured (an instance list, started with the first such pass;
    # the caller clears it with pass_events)
    pass_events: Optional[list] = None
    replay_host: Optional[list] = None

    def embed_head(self, v: Optional[DecView] = None, R: Optional[int] = None) -> None:
        """The next step's head (embedding of ids at pos + layer 0's LayerNorm) for view v, or for rows [0, R) when
        v is None, as the fused selection would have written it."""
        if v is not None:
            self._embed_head(v)
            return
        for r0 in range(0, R, VIEW_ROWS):
            self._embed_head(self._view(r0, min(VIEW_ROWS, R - r0)))

    def _embed_head(self, v: DecView) -> None:
        """The head of a decoder step alone (embedding + layer 0's self_attn_layer_norm) for view v: primes a chain
        whose captured steps run pre_embedded."""
        L0 = self.w.dec[0]
        _lib.call("tw_embed_decoder", self.w.emb.data_ptr(), self.w.pos_dec.data_ptr(), v.ids.data_ptr(),
                  v.pos.data_ptr(), v.n, self.d.d_model, v.xd.data_ptr(), v.stream.cuda_stream)
        self._resid_ln_p(v.n, 0, None, L0.ln1_g, L0.ln1_b, v)

    def _gen_step(self, R: int, params, v: Optional[DecView] = None, r_enc: Optional[int] = None,
                  fused: bool = False) -> None:
        """One generated token. fused: the step starts pre-embedded and ends by embedding its token for the next
        step (tw_logits_select_embed); only for a view whose previous step did the same or that was primed."""
        self.decoder_step(R, v=v, r_enc=r_enc, pre_embedded=fused)
        self._select(R, params, v=v, embed_next=fused)

    # K-slices of the vocabulary-wide proj_out for a decode pass with no encoder beside it (the pipeline's last batch, a
    # single-batch call, beam passes of the as-shipped call, long-form). 1 by default: 4 slices make the launch itself
    # faster alone (22.7 vs 33 us) but the captured step slower (444.4 vs 439.6 us at 24 rows, bench 99.6 vs 98.9 ms,
    # profiles/r04n_ab.txt).
    dec_alone_wide_kw = 1
    # (the same beside an encoder chunk: 1)
    dec_beside_wide_kw = 1

    # The layer GEMVs' kernel (tw_gemv_set_variant) for a decode pass alone: k_gemv_q (1: one column group per wave, the
    # whole K-slice in flight; the library keeps k_gemv_pc at <= 16 rows and above 32) — captured step 393.5 -> 384.8
    # us at 24 rows (profiles/r05i_decode_chain.txt; at 64 rows 682.6 -> 651.1 in the captured step, but config 5's
    # bench 201.7-202.5 vs 198.8-198.9 ms with k_gemv_pc, profiles/r05aa_c5_gemv_ab.txt); beside an encoder chunk
    # k_gemv_pc (0): 87.86 vs 88.45 ms per bench step (profiles/r05i_gemv_ab.txt).
    dec_alone_gemv = 1
    dec_beside_gemv = 0

    # The decoder's layers for a decode pass alone as ONE persistent launch (tw_dec_fused, csrc/decfused.hip) instead
    # of the 45-launch chain, for passes of at most dec_fused_max_rows rows (greedy / sampled, without beams, prompt
    # masks or alignment heads). Measured per step alone (scripts/decode_step_time.py --fused 0 1,
    # profiles/r06o_fused_small_rows.txt): 1 row 238 vs 276 us, 2: 243 vs 280, 4: 259 vs 283, 8: 303 vs 293,
    # 15: 362 vs 324, 24: 407 vs 385 — the single-upload calls of the reference's API (a few windows) gain, the
    # engine batches do not. Opt-in (False by default): its rows round differently from the chain's, so
    # with it a call's transcript depends on how many windows share its decode pass, and a window-sharded call
    # (twamd.dist: ranks of <= 4 windows) would no longer equal the single-process call bit for bit
    # (tests/test_gpu_c3_c4.py). Beside an encoder chunk the chain stays (a persistent grid would hold every CU the
    # encoder GEMM needs).
    dec_fused_alone = False
    dec_fused_max_rows = 4

    @property
    def _wide_kw(self) -> int:
        return self._dec_ctx[0]

    def _dec_context(self) -> tuple:
        """Set the decoder-step kernel choices for a pass starting now (the proj_out K-slice count and the layer GEMV
        kernel): alone unless run_batches' encoder pump is queued beside it. Graph keys carry the returned value (a
        captured step bakes the launches it recorded)."""
        beside = self._pump is not None
        ctx = ((self.dec_beside_wide_kw, self.dec_beside_gemv, False) if beside
               else (self.dec_alone_wide_kw, self.dec_alone_gemv, bool(self.dec_fused_alone and self._fused_dims)))
        if ctx[:2] != self._dec_ctx[:2]:
            _lib.call("tw_gemv_set_wide_slices", ctx[0])
            _lib.call("tw_gemv_set_variant", ctx[1])
        self._dec_ctx = ctx
        return ctx

    def _fused_ok(self, R: int) -> bool:
        """The current step runs as tw_dec_fused (see dec_fused_alone)."""
        return (self._dec_ctx[2] and R <= min(32, self.dec_fused_max_rows) and self._kv_tab is None
                and not self._masked and self._align is None and not self._use_dec_row_map)

    def _fused_layers(self, R: int, r_enc: int, v: DecView) -> None:
        """tw_dec_fused for the view's rows: xd (the embedded token) -> the last layer's output, the self K/V caches
        appended, hp = the final LayerNorm (proj_out's packed operand)."""
        d, w = self.d, self.w
        H, T = d.heads, d.max_target_positions
        esz = self.cross_kv.element_size()
        xkv = self.cross_kv.data_ptr() + v.r0 * H * S_ENC * 64 * esz
        _lib.call("tw_dec_fused", self._fused_tab.data_ptr(), d.decoder_layers, R, v.pos.data_ptr(), v.xd.data_ptr(),
                  self.kcache[0, v.r0].data_ptr(), self.vcache[0, v.r0].data_ptr(), self.kcache.stride(0), T, xkv,
                  2 * r_enc * H * S_ENC * 64, r_enc * H * S_ENC * 64, S_ENC, v.qd.data_ptr(), v.attd.data_ptr(),
                  v.fp.data_ptr(), v.parts.data_ptr(), self._fused_xpart.data_ptr(), w.dec_ln_g.data_ptr(),
                  w.dec_ln_b.data_ptr(), v.hp.data_ptr(),
                  LN_EPS, v.fsync.data_ptr(), self._fused_err.data_ptr(), v.stream.cuda_stream)

    def _fused_table(self) -> torch.Tensor:
        """tw_dec_fused's layer table: per decoder layer the TwDecLayerW pointers (packed weights, f32 biases and
        LayerNorm parameters), int64 [layers][18] on the device."""
        names_w = ("wqkv", "wo", "wq_x", "wo_x", "w1", "w2")
        names_f = ("bqkv", "bo", "bq_x", "bo_x", "b1", "b2", "ln1_g", "ln1_b", "ln2_g", "ln2_b", "ln3_g", "ln3_b")
        rows = []
        for L, P in zip(self.w.dec, self.dec_p):
            for k in names_f:
                t = getattr(L, k)
                if t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError(f"tw_dec_fused: decoder {k} must be contiguous f32")
            rows.append([P[k].data_ptr() for k in names_w] + [getattr(L, k).data_ptr() for k in names_f])
        return torch.tensor(rows, dtype=torch.int64, device=self.device)

    def check_fused(self) -> None:
        """Raise if a tw_dec_fused launch since the last check timed out in a phase wait (its outputs are void)."""
        e = int(self._fused_err[0].item())
        if e:
            self._fused_err.zero_()
            raise _lib.TwError(f"tw_dec_fused: a phase wait timed out (code {e:#x}); the decode pass is void")

    def _prompt_len(self, tail: Sequence[int], prefix=None) -> int:
        """decoder_input_ids' length: [prefix] + SOT (+ language) + tail (num_input_ids of the token timestamps)."""
        L = len(prefix[0][0]) if prefix is not None and prefix[0] else 0
        return L + 1 + (1 if self.gen.special.is_multilingual else 0) + len(tail)

    def _token_ts(self, R: int, P: int, res: PassResult, num_frames: Optional[Sequence[int]]) -> None:
        """res.token_ts from the alignment heads' probabilities of a greedy / sampled pass (self._align): the pass's
        rows standardised over its padded length (max generated - 1 fed tokens), as _extract_token_timestamps does
        over the batch (generation_whisper.py:241-381); prompt positions 0."""
        st = self.gen.special
        real = [(t.index(st.eot) + 1) if st.eot in t else len(t) for t in res.tokens]
        rows = max(real) - 1 if real else 0
        w = self._align_weights(R, rows) if rows > 0 else None
        res.token_ts = []
        for r in range(R):
            nf = None if num_frames is None else int(num_frames[r])
            ts = (alignment.token_timestamps(w[r], 0, nf, self.gen.median_filter_width) if w is not None
                  else np.zeros(1, np.float32))
            res.token_ts.append(np.concatenate([np.zeros(P, np.float32), ts]))

    def _prefill(self, R: int, prefix, r_enc: Optional[int] = None) -> int:
        """condition_on_prev_tokens: feed a pass's left-padded prefix (per row [<|startofprev|>] + the previous
        segments' tokens, generation_whisper.py:1853-1918) at positions 0 .. L-1 ahead of the init tokens; returns L.
        prefix = (rows [R][L], pads [R]). The pad positions are fed too (transformers' cache positions count them) and
        masked out of every later query (kv_start, tw_attn_decode_self_masked); the caller ends the pass with
        _masked = False."""
        if prefix is None:
            return 0
        rows, pads = prefix
        L = len(rows[0]) if rows else 0
        if L == 0:
            return 0
        if len(rows) != R or any(len(r) != L for r in rows):
            raise ValueError("prefix: one left-padded row of equal length per decoder row")
        dev = self.device
        cols = torch.as_tensor(rows, dtype=torch.int32, device=dev)
        self._kv_start[:R] = torch.as_tensor(list(pads), dtype=torch.int32, device=dev)
        self._masked = True
        for k in range(L):
            self.ids[:R] = cols[:, k]
            self.pos[:R] = k
            self.decoder_step(R, with_logits=False, r_enc=r_enc)
        return L

    @on_engine_streams
    def _detect_languages(self, R: int) -> List[int]:
        """detect_language (generation_whisper.py:1455-1520) for the R rows encoded into the current slot: one decoder
        step on [SOT] at position 0 and the language argmax (the mode-1 selection), with no prompt in front — what
        generate() does before its seek loop. Positions it writes are rewritten by the pass that follows."""
        st = self.gen.special
        self._dec_context()
        self.stream.wait_event(self._enc_ev[self._slot])
        with torch.cuda.stream(self.stream):
            self.state[:R].zero_()
            self.state[:R, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
            self.pos[:R] = 0
            self.ids[:R] = st.sot
            self.decoder_step(R)
            self._select(R, self._select_params(1, 1), tokens=False)  # ids <- lang
            out = self.ids[:R].tolist()
        return [int(x) for x in out]

    @on_engine_streams
    def decode_pass(self, R: int, tail: Sequence[int], lang_ids: Optional[Sequence[int]], max_new: int,
                    check_every: int = 8, use_timestamps: bool = True, align: bool = False,
                    num_frames: Optional[Sequence[int]] = None, prefix=None) -> PassResult:
        """Greedy decode of R rows from the prompt [SOT, (lang), *tail] (the init tokens of
        _retrieve_init_tokens; the language is detected from the SOT step when lang_ids is None on a
        multilingual model). Returns the generated tokens of every row; with align, also every row's token-level
        timestamps (alignment-head cross-attention of the fed tokens -> DTW; num_frames: the rows' valid frames
        minus their seek, as generate() passes them)."""
        if align:
            P = self._prompt_len(tail, prefix)
            self._align_setup(R, P, max_new)
            try:
                res = self.decode_pass(R, tail, lang_ids, max_new, check_every, use_timestamps, prefix=prefix)
                self._token_ts(R, P, res, num_frames)
                return res
            finally:
                self._align = None
        st = self.gen.special
        dev = self.device
        self._dec_context()
        self.stream.wait_event(self._enc_ev[self._slot])  # the cross-K/V of this slot is written
        detect = st.is_multilingual and lang_ids is None
        params = self._select_params(0, max_new, use_timestamps)
        base = self._prefill(R, prefix)  # (condition_on_prev_tokens: the init tokens start at position base)

        def prompt() -> None:
            """State reset, the prompt steps [SOT, (lang), *tail] and the first generated token (one token per
            step; the language detected from the SOT step's logits by the mode-1 selection when lang_ids is None)."""
            self.state[:R].zero_()
            self.state[:R, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
            self.pos[:R] = base
            self.ids[:R] = st.sot
            prompt_rest: List = []  # per-position token ids after SOT (int, or per-row list)
            if st.is_multilingual:
                prompt_rest.append(None if lang_ids is None else list(lang_ids))
            prompt_rest.extend(int(t) for t in tail)
            for k, tok in enumerate(prompt_rest):
                if k == 0 and detect:
                    self.decoder_step(R)
                    self._select(R, self._select_params(1, max_new), tokens=False)  # ids <- lang, pos += 1
                    continue
                self.decoder_step(R, with_logits=False)
                if isinstance(tok, list):
                    self.ids[:R] = torch.as_tensor(tok, dtype=torch.int32, device=dev)
                else:
                    self.ids[:R] = tok
                self.pos[:R] = base + k + 1
            self._gen_step(R, params)  # last prompt token -> first generated token

        # the prompt phase as one captured graph (its ~140 launches replayed instead of issued one by one from the
        # host while the next batch's encoder keeps the GPU busy); per-row language ids given by the caller stay eager
        # (their host-to-device copy is not capturable)
        if self.use_graphs and self.prompt_graph and (detect or not st.is_multilingual) and not base:
            al = self._align  # (keyed like _graph_for: an alignment pass captures the probability-recording kernel)
            key = ("prompt", R, tuple(int(t) for t in tail), max_new, use_timestamps, self._slot,
                   None if al is None else (al["pos0"], al["n_steps"], al["buf"].data_ptr()), self._dec_ctx)
            g = self._graphs.get(key)
            if g is None:
                g = torch.cuda.CUDAGraph()
                with _capture(g, self.stream):  # records, does not execute
                    prompt()
                self._graphs[key] = g
            g.replay()
        else:
            prompt()
        steps = 1
        # generation loop: the rows split into chains on their own high-priority streams, each replaying its
        # captured decode step; the chains' latency-bound kernels run concurrently
        chains = self._chains(R)
        fused = self.fused_select
        graphs = ([self._graph_for(R, params, i, c, fused) for i, c in enumerate(chains)] if self.use_graphs
                  else None)
        hook = self.step_hook
        if hook is not None:  # teacher forcing (parity harness): logits of generated position 0 are in place
            self.stream.synchronize()
            with torch.cuda.stream(self.stream):
                hook(0, None)
        for c in chains:
            c.stream.wait_stream(self.stream)
            if fused and max_new > 1:
                with torch.cuda.stream(c.stream):
                    self._embed_head(c)
        pump, inflight = self._pump, []
        # steps per graph replay: several captured back to back when no encoder chunk is pumped between steps and no
        # teacher-forcing hook runs after each (one host replay per graph_steps tokens)
        gs = 1 if (hook is not None or graphs is None) else (
            self.graph_steps_beside if pump is not None else self.graph_steps_alone)
        if gs > 1 and max_new - steps >= gs:  # (captured before the loop, like the one-step graphs)
            for i, c in enumerate(chains):
                self._graph_for(R, params, i, c, fused, gs)
        ev0 = None
        if self.pass_events is not None:  # (measurement: HIP events around the generation loop)
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(chains[0].stream)
            th0 = time.perf_counter()
            if self.replay_host is None:
                self.replay_host = []
        while steps < max_new:
            n = min(check_every if hook is None else 1, max_new - steps)
            done = 0
            while done < n:
                k = gs if n - done >= gs else 1
                done += k
                for i, c in enumerate(chains):
                    if graphs is not None:
                        g = graphs[i] if k == 1 else self._graph_for(R, params, i, c, fused, k)
                        if ev0 is not None:
                            tr = time.perf_counter()
                        with torch.cuda.stream(c.stream):
                            g.replay()
                        if ev0 is not None:
                            self.replay_host.append(time.perf_counter() - tr)
                    else:
                        self._gen_step(c.n, params, v=c, r_enc=R, fused=fused)
                if hook is not None:
                    for i, c in enumerate(chains):
                        c.stream.synchronize()
                        with torch.cuda.stream(c.stream):
                            hook(steps, c)
                if pump is not None:  # keep both queues shallow: <= dec_ahead steps, <= pump.ahead encoder chunks
                    ev = torch.cuda.Event()
                    ev.record(chains[-1].stream)
                    inflight.append(ev)
                    while len(inflight) > self.dec_ahead:
                        if inflight[0].query():
                            inflight.pop(0)
                        elif not pump():
                            _wait(inflight.pop(0))
            steps += n
            # the finished check on the chains' own stream: a wait of the engine stream on the chain stream here, with
            # the steps still queued, slowed every queued step by ~50 us (438 vs 389 us at 24 rows,
            # scripts/decode_chain_costs.py --passlike); the engine stream joins once the host has synchronised
            cs = chains[0].stream
            for c in chains[1:]:
                if c.stream is not cs:
                    cs.wait_stream(c.stream)
            with torch.cuda.stream(cs):
                done_all = bool(self.state[:R, _lib.TW_ST_FINISHED].all().item())
            if done_all:
                break
        for c in chains:
            self.stream.wait_stream(c.stream)
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(self.stream)
            self.pass_events.append((ev0, ev1, steps - 1, time.perf_counter() - th0))
        ngen = self.state[:R, _lib.TW_ST_NGEN].tolist()
        toks = self.tokens[:R].tolist()
        if self._dec_ctx[2]:
            self.check_fused()
        detected = self.state[:R, _lib.TW_ST_LANG].tolist() if detect else None  # (mode-1 selection only writes it)
        return PassResult([toks[r][: ngen[r]] for r in range(R)], detected if lang_ids is None else list(lang_ids))

    @on_engine_streams
    def sample_pass(self, R: int, tail: Sequence[int], lang_ids: Optional[Sequence[int]], max_new: int,
                    temperature: float = 0.0, top_k: int = 50, seed: int = 0, row_keys: Optional[Sequence[int]] = None,
                    use_timestamps: bool = True, enc_rows: Optional[Sequence[int]] = None, r_enc: Optional[int] = None,
                    no_speech_token: Optional[int] = None, check_every: int = 8, prefix=None, align: bool = False,
                    num_frames: Optional[Sequence[int]] = None) -> PassResult:
        """One decode pass of the temperature-fallback loop (WhisperGenerationMixin.generate_with_fallback,
        generation_whisper.py:970-1116), eager, one tw_logits_sample per token: greedy when temperature == 0
        (the tokens of decode_pass), else a draw from softmax(processed / T) over the top_k scores. Per row it also
        returns the sum of the chosen tokens' log-probabilities (the avg_logprob criterion's numerator) and, with
        no_speech_token, WhisperNoSpeechDetection's probability of it at the SOT position. enc_rows: the encoder
        rows (of the r_enc-row encoded batch in this slot) the R decoder rows read (default 0..R-1). align: also the
        rows' token-level timestamps (as decode_pass)."""
        if align:
            P = self._prompt_len(tail, prefix)
            self._align_setup(R, P, max_new)
            try:
                res = self.sample_pass(R, tail, lang_ids, max_new, temperature, top_k, seed, row_keys, use_timestamps,
                                       enc_rows, r_enc, no_speech_token, check_every, prefix)
                self._token_ts(R, P, res, num_frames)
                return res
            finally:
                self._align = None
        st = self.gen.special
        dev = self.device
        r_enc = R if r_enc is None else r_enc
        self._dec_context()
        self.stream.wait_event(self._enc_ev[self._slot])
        detect = st.is_multilingual and lang_ids is None
        params = self._select_params(0, max_new, use_timestamps)
        keys = torch.as_tensor(list(row_keys) if row_keys is not None else list(range(R)), dtype=torch.int32,
                               device=dev)
        V = self.d.vocab
        s = self.stream.cuda_stream
        if enc_rows is not None:
            self.dec_row_map[:R] = torch.as_tensor(list(enc_rows), dtype=torch.int32, device=dev)
            self._use_dec_row_map = True
            self._row_group = 1
        try:
            base = self._prefill(R, prefix, r_enc)
            self.state[:R].zero_()
            self.state[:R, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
            self.pos[:R] = base
            self.ids[:R] = st.sot
            prompt_rest: List = []
            if st.is_multilingual:
                prompt_rest.append(None if lang_ids is None else list(lang_ids))
            prompt_rest.extend(int(t) for t in tail)

            def no_speech() -> None:  # the logits of the step that fed <|startoftranscript|>
                if no_speech_token is not None:
                    _lib.call("tw_token_prob", self.logits.data_ptr(), R, V, V, int(no_speech_token),
                              self.state.data_ptr(), s)

            for k, tok in enumerate(prompt_rest):
                want = k == 0 and (detect or no_speech_token is not None)
                self.decoder_step(R, with_logits=want, r_enc=r_enc)
                if k == 0:
                    no_speech()
                if k == 0 and detect:
                    self._select(R, self._select_params(1, max_new), tokens=False)  # ids <- lang, pos += 1
                    continue
                if isinstance(tok, list):
                    self.ids[:R] = torch.as_tensor(tok, dtype=torch.int32, device=dev)
                else:
                    self.ids[:R] = tok
                self.pos[:R] = base + k + 1
            steps = 0
            while steps < max_new:
                self.decoder_step(R, r_enc=r_enc)
                if steps == 0 and not prompt_rest:
                    no_speech()
                _lib.call("tw_logits_sample", self.logits.data_ptr(), R, V, self.suppress_bits.data_ptr(),
                          ctypes.byref(params), float(temperature), int(top_k), int(seed) & 0xFFFFFFFFFFFFFFFF,
                          keys.data_ptr(), self.state.data_ptr(), self.tokens.data_ptr(), self.tokens.shape[1],
                          self.ids.data_ptr(), self.pos.data_ptr(), s)
                steps += 1
                if steps % check_every == 0 and bool(self.state[:R, _lib.TW_ST_FINISHED].all().item()):
                    break
            stt = self.state[:R].cpu()
        finally:
            self._use_dec_row_map = False
            self._row_group = 1
        ngen = stt[:, _lib.TW_ST_NGEN].tolist()
        toks = self.tokens[:R].tolist()
        if self._dec_ctx[2]:
            self.check_fused()
        f32 = stt.view(torch.float32)
        return PassResult([toks[r][: ngen[r]] for r in range(R)],
                          stt[:, _lib.TW_ST_LANG].tolist() if detect else list(lang_ids) if lang_ids is not None else None,
                          sum_logprob=f32[:, _lib.TW_ST_SUMLP].tolist(),
                          no_speech_prob=f32[:, _lib.TW_ST_NOSPEECH].tolist() if no_speech_token is not None else None)

    def _beam_buffers(self, R: int) -> dict:
        if self._beam is None or self._beam["rows"] < R:
            dev, d = self.device, self.d
            T = d.max_target_positions
            ws_bytes = int(_lib.load().tw_beam_workspace_bytes(self.max_rows))
            self._beam = {
                "rows": self.max_rows,
                "run_score": torch.zeros(self.max_rows, dtype=torch.float32, device=dev),
                "fin_score": torch.zeros(self.max_rows, dtype=torch.float32, device=dev),
                "fin_flag": torch.zeros(self.max_rows, dtype=torch.int32, device=dev),
                "fin_len": torch.zeros(self.max_rows, dtype=torch.int32, device=dev),
                "fin_tokens": torch.zeros(self.max_rows, T, dtype=torch.int32, device=dev),
                "win": torch.zeros(self.max_batch, 4, dtype=torch.int32, device=dev),
                "src_rows": torch.zeros(self.max_rows, dtype=torch.int32, device=dev),
                "ws": torch.empty(ws_bytes, dtype=torch.uint8, device=dev),
                "kv_tab": torch.empty(self.max_rows, T, dtype=torch.int32, device=dev),
                "fin_tab": torch.zeros(self.max_rows, T, dtype=torch.int32, device=dev),
                "run_lp": torch.zeros(self.max_rows, dtype=torch.float32, device=dev),
                "fin_lp": torch.zeros(self.max_rows, dtype=torch.float32, device=dev),
            }
        return self._beam

    @on_engine_streams
    def beam_pass(self, W: int, num_beams: int, tail: Sequence[int], lang_ids: Optional[Sequence[int]], max_new: int,
                  use_timestamps: bool = True, check_every: int = 8, length_penalty: float = 1.0,
                  enc_row0: int = 0, r_enc: Optional[int] = None, prefix=None, align: bool = False,
                  num_frames: Optional[Sequence[int]] = None, enc_rows: Optional[Sequence[int]] = None,
                  criteria: bool = False, no_speech_token: Optional[int] = None) -> PassResult:
        """Beam-search decode (GenerationMixin._beam_search, $TF/generation/utils.py:3208-3512) of W windows with
        num_beams rows each (row = w * num_beams + j, all reading window w's cross-K/V): the prompt as
        decode_pass (language detected from the SOT step when lang_ids is None), then per token one decoder step
        over all rows and tw_beam_step (which also repoints the self-attention K/V position table). Returns the best finished hypothesis of
        every window (with its EOS when it ended on one). enc_row0 / r_enc: the windows' first row and the batch
        the cross-K/V slot was encoded with (default 0 / W). align: also every window's token-level timestamps, from
        the alignment heads' cross-attention of the rows that fed its best hypothesis (the kernel's fin_tab: generate's
        beam_indices, generation_whisper.py:265-300; past a hypothesis' end, row 0's, as index -1 -> 0 there).
        enc_rows: each window's encoder row (instead of enc_row0 + w: a fallback round's subset). criteria: also each
        best hypothesis' sum of log-probabilities renormalised over the allowed tokens (the fallback's average
        log-probability numerator, tw_beam_step's fin_lp) and, with no_speech_token, WhisperNoSpeechDetection's
        probability at the <|startoftranscript|> step (PassResult.sum_logprob / no_speech_prob)."""
        if align:
            P = self._prompt_len(tail, prefix)
            self._align_setup(W * num_beams, P, max_new)
            try:
                res = self.beam_pass(W, num_beams, tail, lang_ids, max_new, use_timestamps, check_every, length_penalty,
                                     enc_row0, r_enc, prefix, enc_rows=enc_rows, criteria=criteria,
                                     no_speech_token=no_speech_token)
                bb = self._beam
                nb, st = num_beams, self.gen.special
                lens = [len(t) for t in res.tokens]  # generated tokens, EOS included (beam_indices' entries)
                rows = max(lens) - 1 if lens else 0
                res.token_ts = []
                if rows > 0:
                    al = self._align
                    b = al["buf"][: W * nb * al["n_steps"] * al["n_slots"] * S_ENC].view(
                        W * nb, al["n_steps"], al["n_slots"], S_ENC)
                    ftab = bb["fin_tab"][: W * nb: nb, P: P + rows].long()  # rows that fed positions P .. P+rows-1
                    i = torch.arange(rows, device=self.device)
                    ftab = torch.where(i[None, :] + 1 < torch.tensor(lens, device=self.device)[:, None], ftab, 0)
                    w = b[ftab, i[None, :]].permute(0, 2, 1, 3)[:, al["perm"]].float().cpu().numpy()
                for k in range(W):
                    nf = None if num_frames is None else int(num_frames[k])
                    ts = (alignment.token_timestamps(w[k], 0, nf, self.gen.median_filter_width) if rows > 0
                          else np.zeros(1, np.float32))
                    res.token_ts.append(np.concatenate([np.zeros(P, np.float32), ts]))
                return res
            finally:
                self._align = None
        nb, R = num_beams, W * num_beams
        r_enc = W if r_enc is None else r_enc
        if R > self.max_rows:
            raise ValueError(f"{W} windows x {nb} beams > {self.max_rows} decoder rows (construct with max_beams)")
        st = self.gen.special
        dev = self.device
        T = self.d.max_target_positions
        bb = self._beam_buffers(R)
        self._dec_context()
        self.stream.wait_event(self._enc_ev[self._slot])
        if enc_rows is not None:
            self.dec_row_map[:R] = torch.as_tensor([int(enc_rows[w]) for w in range(W) for _ in range(nb)],
                                                   dtype=torch.int32, device=dev)
        else:
            self.dec_row_map[:R] = enc_row0 + torch.arange(R, dtype=torch.int32, device=dev) // nb
        self._use_dec_row_map = True
        self._row_group = nb  # rows w * nb + j share window w's cross K/V
        # self-attention K/V position table: every row starts on its own history; tw_beam_step points a continuing
        # beam at its source's rows (no K/V copy: the reorder moved ~550 MB per step at 60 rows)
        bb["kv_tab"][:R] = torch.arange(R, dtype=torch.int32, device=dev)[:, None]
        self._kv_tab = bb["kv_tab"]
        try:
            # (a window's prefix on each of its beam rows)
            base = self._prefill(R, None if prefix is None else
                                 ([prefix[0][w] for w in range(W) for _ in range(nb)],
                                  [prefix[1][w] for w in range(W) for _ in range(nb)]), r_enc)
            self.state[:R].zero_()
            self.state[:R, _lib.TW_ST_LAST:_lib.TW_ST_LASTTS + 1] = -1
            self.pos[:R] = base
            self.ids[:R] = st.sot
            detected = None
            prompt_rest: List = []
            if st.is_multilingual:
                prompt_rest.append(None if lang_ids is None else [int(x) for x in lang_ids for _ in range(nb)])
            prompt_rest.extend(int(t) for t in tail)
            V = self.d.vocab

            def no_speech() -> None:  # the logits of the step that fed <|startoftranscript|>
                if no_speech_token is not None:
                    _lib.call("tw_token_prob", self.logits.data_ptr(), R, V, V, int(no_speech_token),
                              self.state.data_ptr(), self.stream.cuda_stream)

            for k, tok in enumerate(prompt_rest):
                if k == 0 and st.is_multilingual and lang_ids is None:
                    self.decoder_step(R, r_enc=r_enc)
                    no_speech()
                    self._select(R, self._select_params(1, max_new), tokens=False)  # ids <- lang, pos += 1
                    detected = self.state[:R:nb, _lib.TW_ST_LANG].tolist()
                    continue
                self.decoder_step(R, with_logits=k == 0 and no_speech_token is not None, r_enc=r_enc)
                if k == 0:
                    no_speech()
                if isinstance(tok, list):
                    self.ids[:R] = torch.as_tensor(tok, dtype=torch.int32, device=dev)
                else:
                    self.ids[:R] = tok
                self.pos[:R] = base + k + 1
            bb["run_score"][:R].view(W, nb).fill_(-1e9)
            bb["run_score"][:R].view(W, nb)[:, 0] = 0.0
            bb["fin_score"][:R] = -1e9
            bb["fin_flag"][:R] = 0
            bb["fin_len"][:R] = 0
            if criteria:
                bb["run_lp"][:R] = 0.0
                bb["fin_lp"][:R] = 0.0
            bb["win"][:W] = torch.tensor([1, 0, 0, 0], dtype=torch.int32, device=dev)
            self.state[:R, _lib.TW_ST_NGEN] = 0
            sel = self._select_params(0, max_new, use_timestamps)
            bp = _lib.TwBeamParams(nb, max_new, float(length_penalty), T)
            bst = _lib.TwBeamState(bb["run_score"].data_ptr(), bb["fin_score"].data_ptr(), bb["fin_flag"].data_ptr(),
                                   bb["fin_len"].data_ptr(), bb["fin_tokens"].data_ptr(), bb["win"].data_ptr(),
                                   bb["src_rows"].data_ptr(), bb["kv_tab"].data_ptr(),
                                   bb["fin_tab"].data_ptr() if self._align is not None else None,
                                   bb["run_lp"].data_ptr() if criteria else None,
                                   bb["fin_lp"].data_ptr() if criteria else None)
            s = self.stream.cuda_stream

            def step() -> None:
                self.decoder_step(R, r_enc=r_enc)
                _lib.call("tw_beam_step", self.logits.data_ptr(), W, self.d.vocab, self.suppress_bits.data_ptr(),
                          ctypes.byref(sel), ctypes.byref(bp), ctypes.byref(bst), self.state.data_ptr(),
                          self.tokens.data_ptr(), self.ids.data_ptr(), self.pos.data_ptr(), bb["ws"].data_ptr(), s)

            # one beam step (decoder step over every row, tw_beam_step with its K/V table update) as one captured graph: the
            # step reads its position, scores and histories from device memory, so the same graph serves every step
            # (eager, each of its ~100 launches would be issued from the host every token)
            g = None
            if self.use_graphs:
                al = self._align
                key = ("beam", R, nb, max_new, bool(use_timestamps), float(length_penalty), self._slot, r_enc,
                       self._masked, None if al is None else (al["pos0"], al["n_steps"], al["buf"].data_ptr()),
                       bool(criteria), self._dec_ctx)
                g = self._graphs.get(key)
                if g is None:
                    g = torch.cuda.CUDAGraph()
                    with _capture(g, self.stream):  # records, does not execute
                        step()
                    self._graphs[key] = g
            steps = 0
            while steps < max_new:
                if steps == 0 and not prompt_rest and no_speech_token is not None:
                    # (a bare <|startoftranscript|> prompt: its step is the first beam step, eager with the probability)
                    self.decoder_step(R, r_enc=r_enc)
                    no_speech()
                    _lib.call("tw_beam_step", self.logits.data_ptr(), W, V, self.suppress_bits.data_ptr(),
                              ctypes.byref(sel), ctypes.byref(bp), ctypes.byref(bst), self.state.data_ptr(),
                              self.tokens.data_ptr(), self.ids.data_ptr(), self.pos.data_ptr(), bb["ws"].data_ptr(), s)
                elif g is not None:
                    g.replay()
                else:
                    step()
                steps += 1
                if steps % check_every == 0 or steps >= max_new:
                    if bool(bb["win"][:W, 1].all().item()):
                        break
            flen = bb["fin_len"][:R:nb].tolist()
            ftok = bb["fin_tokens"][:R:nb].tolist()
            sum_lp = bb["fin_lp"][:R:nb].tolist() if criteria else None
            nsp = (self.state[:R:nb, _lib.TW_ST_NOSPEECH].contiguous().view(torch.float32).tolist()
                   if no_speech_token is not None else None)
        finally:
            self._use_dec_row_map = False
            self._row_group = 1
            self._kv_tab = None
        return PassResult([ftok[w][: flen[w]] for w in range(W)], detected if lang_ids is None else list(lang_ids),
                          sum_logprob=sum_lp, no_speech_prob=nsp)

    def _chains(self, R: int) -> List[DecView]:
        """Contiguous row ranges of [0, R), one per decode chain (each with its own partial-sum buffer)."""
        key = ("chains", R)
        if key not in self._chain_cache:
            k = max(1, min(self.n_chains, R // 4))
            k = max(k, (R + VIEW_ROWS - 1) // VIEW_ROWS)  # <= VIEW_ROWS rows per chain (packed GEMV limit)
            while len(self._chain_streams) < k:
                self._chain_streams.append(self._chain_streams[0])  # one stream: the chains run in turn
            views = []
            for i in range(k):
                r0, r1 = i * R // k, (i + 1) * R // k
                parts = torch.empty(DEC_SPLITS, r1 - r0, self.d.d_model, dtype=torch.float32, device=self.device)
                views.append(self._view(r0, r1 - r0, self._chain_streams[i], parts))
            self._chain_cache[key] = views
        return self._chain_cache[key]

    def _graph_for(self, R: int, params, i: int, v: DecView, fused: bool = False,
                   n_steps: int = 1) -> Optional[torch.cuda.CUDAGraph]:
        """The captured decode step of chain i (n_steps > 1: that many steps back to back in one graph)."""
        al = self._align
        key = (R, params.max_new, params.use_timestamps, self._slot, i, fused,
               None if al is None else (al["pos0"], al["n_steps"], al["buf"].data_ptr()), self._masked, self._dec_ctx,
               n_steps)
        g = self._graphs.get(key)
        if g is not None:
            return g
        g = torch.cuda.CUDAGraph()
        v.stream.wait_stream(self.stream)
        with torch.cuda.stream(v.stream):
            with _capture(g, v.stream):  # records, does not execute
                for _ in range(n_steps):
                    self._gen_step(v.n, params, v=v, r_enc=R, fused=fused)
        self.stream.wait_stream(v.stream)
        self._graphs[key] = g
        return g

    # ------------------------------------------------------------------ seek loop
    def prompt_tail(self, task: Optional[str], return_timestamps: bool, language_given: bool = False) -> List[int]:
        """Init tokens after SOT/lang (_retrieve_init_tokens, generation_whisper.py:1455-1608)."""
        st = self.gen.special
        tail: List[int] = []
        if task is not None:
            if not st.is_multilingual:
                raise ValueError("Cannot specify `task` or `language` for an English-only model.")
            if task not in ("transcribe", "translate"):
                raise ValueError(f"The `{task}` task is not supported. The task should be one of "
                                 "`['translate', 'transcribe']`")
            tail.append(st.transcribe if task == "transcribe" else st.translate)
        elif st.is_multilingual and language_given:
            tail.append(st.transcribe)  # language given without a task: transcribe
        if not return_timestamps:
            tail.append(st.notimestamps)
        return tail

    def max_new_for(self, prompt_len: int, max_new_tokens: Optional[int] = None) -> int:
        """_set_max_new_tokens_and_length (generation_whisper.py:1920-1950) for one seek pass."""
        g, T = self.gen, self.d.max_target_positions
        mnt = max_new_tokens if max_new_tokens is not None else g.max_new_tokens
        if mnt is not None:
            if mnt + prompt_len > T:
                raise ValueError(f"prompt length {prompt_len} + max_new_tokens {mnt} exceeds {T}")
            return mnt
        return min(g.max_length + prompt_len, T) - prompt_len

    @on_engine_streams
    def generate(self, n_chunks: int, task: Optional[str] = "transcribe", lang_ids: Optional[Sequence[int]] = None,
                 max_new_tokens: Optional[int] = None, return_timestamps: bool = True,
                 max_passes: Optional[int] = None, slot: Optional[int] = None,
                 pre_encoded: bool = False, num_beams: int = 1, word_timestamps: bool = False,
                 num_frames: Optional[Sequence[int]] = None, fallback: Optional[FallbackConfig] = None,
                 window_offset: int = 0, condition_on_prev_tokens: bool = False,
                 prompt_ids: Optional[Sequence[int]] = None,
                 prompt_condition_type: Optional[str] = None) -> List[List[int]]:
        """Whisper short-form generate() over feats[slot][:n_chunks] (each 3000 frames): language
        detection, the seek loop and segment extraction, returning for every chunk the concatenated
        segment tokens (what generate() returns before padding).

        pre_encoded: the first seek pass (all chunks, seek 0, n_chunks <= max_batch) was already encoded into
        this slot by encode(n_chunks, row_map=False, seek=False, slot=slot, sync=False) (pipelined prefetch).
        fallback: generate()'s temperature / compression_ratio_threshold / logprob_threshold / no_speech_threshold;
        when it asks for more than greedy decoding every pass runs generate_with_fallback's loop (sample_pass).
        window_offset: the global index of chunk 0 (run_batches' batch offset): the sampler's per-row keys are built
        from global window indices, so windows of different batches draw independent noise.
        condition_on_prev_tokens: every pass after a chunk's first is prompted with <|startofprev|> + the chunk's
        previous segments (_prepare_decoder_input_ids, generation_whisper.py:1853-1918), left padded over the batch.
        prompt_ids / prompt_condition_type: generate()'s initial prompt (<|startofprev|> + text tokens). Unconditioned,
        every pass is prompted with it (:1909-1912); conditioned, "first-segment" makes it the chunks' first segment
        (:1119-1124: behind <|startofprev|>, cut with the rest to the last 223 tokens) and "all-segments" puts it in
        front of the previous segments of every pass after the first (:1887-1888). The language is detected from the
        SOT step alone, before any prompt (detect_language); the prompt is not part of the returned tokens."""
        if slot is not None:
            self.use_slot(slot)
        if pre_encoded and n_chunks > self.max_batch:
            raise ValueError("pre_encoded needs n_chunks <= max_batch")
        st = self.gen.special
        tail = self.prompt_tail(task, return_timestamps, language_given=lang_ids is not None)
        prompt_len = 1 + (1 if st.is_multilingual else 0) + len(tail)
        max_new = self.max_new_for(prompt_len, max_new_tokens)
        seek = [0] * n_chunks
        segs: List[List[int]] = [[] for _ in range(n_chunks)]
        passes_raw: List[List[List[int]]] = [[] for _ in range(n_chunks)]  # every seek pass's raw tokens
        # language: given, or detected on the first pass (seek == 0, the whole 30-s window) as
        # _retrieve_init_tokens -> detect_language does before the seek loop
        langs: List[Optional[int]] = list(lang_ids)[:n_chunks] if lang_ids is not None else [None] * n_chunks
        fb = fallback if fallback is not None and fallback.active else None
        # word timestamps: per chunk the segments' token times (segment token_timestamps of generate(), i.e. the
        # pass's DTW times of the kept tokens + seek * 0.01 s); num_frames: the chunks' valid feature frames
        tts: List[List[float]] = [[] for _ in range(n_chunks)]
        # condition_on_prev_tokens: every chunk's segments so far (current_segments' "tokens") and the per-position
        # flags of generate_with_fallback (written at the row's position in the pass's batch, read by chunk index:
        # transformers' indexing, :1089-1093 / :1885)
        seg_lists: List[List[List[int]]] = [[] for _ in range(n_chunks)]
        do_cond = [bool(condition_on_prev_tokens)] * n_chunks
        prev_sot = self.gen.prev_sot_token_id
        if prev_sot is None and len(self.gen.suppress_tokens) >= 2:
            prev_sot = self.gen.suppress_tokens[-2]  # (:1876-1881)
        prompt = None
        if prompt_ids is not None:
            prompt = [int(t) for t in prompt_ids]
            ptype = prompt_condition_type or "first-segment"  # (_set_prompt_condition_type, :1732-1748)
            if ptype not in ("first-segment", "all-segments"):
                raise ValueError(f"`prompt_condition_type={ptype} does not exist. Make sure to set "
                                 "`prompt_condition_type` to one of first-segment, all-segments")
            if ptype == "all-segments" and not condition_on_prev_tokens:
                raise ValueError("Make sure to set `condition_on_prev_tokens=True` when setting "
                                 "`prompt_condition_type='all-segments'`.")
            if ptype == "first-segment":  # the prompt is every chunk's first segment (_prepare_segments, :1119-1124)
                first = prompt[1:] if prompt and prompt[0] == self.gen.prev_sot_token_id else prompt
                seg_lists = [[list(first)] for _ in range(n_chunks)]
            prompt = {"ids": prompt, "all": ptype == "all-segments"}
        # max_frames (_retrieve_max_frames_and_seek): 3000 per 30-s window; a long-form input's total frames
        if self._long is not None:
            if n_chunks != 1 or pre_encoded:
                raise ValueError("a long-form input is one chunk (set_long_input), encoded per seek pass")
            maxf = [self._long["T"]]
        else:
            maxf = [N_FRAMES] * n_chunks
        passes = 0
        self.last_pass_prefixes: List[list] = [[] for _ in range(n_chunks)]
        try:
            return self._seek_loop(n_chunks, tail, prompt_len, max_new_tokens, max_new, seek, segs, passes_raw, langs,
                                   tts, maxf, seg_lists, do_cond, prev_sot, condition_on_prev_tokens, max_passes,
                                   pre_encoded, num_beams, word_timestamps, num_frames, fb, return_timestamps,
                                   window_offset, prompt)
        finally:
            self._masked = False

    def _seek_loop(self, n_chunks, tail, prompt_len, max_new_tokens, max_new, seek, segs, passes_raw, langs, tts, maxf,
                   seg_lists, do_cond, prev_sot, condition, max_passes, pre_encoded, num_beams, word_timestamps,
                   num_frames, fb, return_timestamps, window_offset, prompt=None):
        st = self.gen.special
        passes = 0
        while any(seek[i] < maxf[i] for i in range(n_chunks)):
            rows = [i for i in range(n_chunks) if seek[i] < maxf[i]]
            per = self.max_batch if num_beams == 1 else min(self.max_batch, self.max_rows // num_beams)
            if per < 1:
                raise ValueError(f"num_beams={num_beams} > the engine's {self.max_rows} decoder rows")
            prefix = None
            if condition and any(do_cond) and len(seg_lists[0]) > 0:
                if len(rows) > per:
                    raise NotImplementedError(f"condition_on_prev_tokens over more than {per} rows in one pass")
                bos = prompt["ids"] if prompt is not None and prompt["all"] else prev_sot
                prefix = condition_prefixes([seg_lists[i] if do_cond[i] else None for i in rows], bos, st.eot,
                                            st.timestamp_begin, self.d.max_target_positions // 2 - 1)
            elif prompt is not None:  # every pass prompted, no padding (:1909-1912)
                prefix = ([list(prompt["ids"]) for _ in rows], [0] * len(rows))
            L = len(prefix[0][0]) if prefix is not None and prefix[0] else 0
            mnew = self.max_new_for(prompt_len + L, max_new_tokens) if L else max_new
            if (prefix is not None and pre_encoded and passes == 0 and st.is_multilingual
                    and any(langs[i] is None for i in rows)):
                # (a pre-encoded first pass holds every chunk in the slot: detect them all before it is split)
                det = self._detect_languages(len(rows))
                for j, i in enumerate(rows):
                    langs[i] = det[j] if langs[i] is None else langs[i]
            for b0 in range(0, len(rows), per):
                part = rows[b0: b0 + per]
                R = len(part)
                pfx = None if prefix is None else (prefix[0][b0: b0 + per], prefix[1][b0: b0 + per])
                for j, i in enumerate(part):  # (diagnostics: the prompt prefix each pass was fed)
                    self.last_pass_prefixes[i].append(None if pfx is None else (pfx[0][j], pfx[1][j]))
                if not (pre_encoded and passes == 0):
                    self.row_map[:R] = torch.as_tensor(part, dtype=torch.int32, device=self.device)
                    self.seek[:R] = torch.as_tensor([seek[i] for i in part], dtype=torch.int32, device=self.device)
                    self.encode(R)
                part_langs = [langs[i] for i in part]
                known = all(lg is not None for lg in part_langs) or not st.is_multilingual
                if not known and pfx is not None:  # detect_language sees [SOT] alone, never the prompt
                    det = self._detect_languages(R)
                    part_langs = [lg if lg is not None else d for lg, d in zip(part_langs, det)]
                    for j, i in enumerate(part):  # (kept for the later passes and last_langs)
                        langs[i] = part_langs[j]
                    known = True
                given = part_langs if (known and st.is_multilingual) else None
                nf_part = None if num_frames is None else [int(num_frames[i]) - seek[i] for i in part]
                if fb is not None:
                    pre = pre_encoded and passes == 0
                    toks_f, skip_f, lang_f, temp_f, nb_left, ts_f = self._fallback_pass(
                        R, tail, given, mnew, return_timestamps, fb, [window_offset + i for i in part], passes,
                        enc_row0=b0 if pre else 0, r_enc=n_chunks if pre else R, prefix=pfx, num_beams=num_beams,
                        align=word_timestamps, num_frames=nf_part)
                    num_beams = nb_left  # (a sampling round left generation_config.num_beams = 1)
                    for j in range(R):  # (by position in the pass's batch, as transformers writes it)
                        do_cond[j] = bool(condition) and (temp_f[j] is None or temp_f[j] < 0.5)
                    for j, i in enumerate(part):
                        if not known:
                            langs[i] = lang_f[j]
                        passes_raw[i].append(list(toks_f[j]))
                        snf = min(maxf[i] - seek[i], N_FRAMES)  # seek_num_frames
                        if skip_f[j]:  # generate(): seek += seek_num_frames, nothing kept
                            seek[i] += snf
                            continue
                        seg_tokens, offset = retrieve_segment(toks_f[j], seek[i], snf, st.timestamp_begin)
                        segs[i].extend(seg_tokens)
                        seg_lists[i].extend(segment_slices(toks_f[j], st.timestamp_begin))
                        if word_timestamps:
                            self._add_times(tts[i], ts_f[j], prompt_len + L, len(seg_tokens), seek[i])
                        seek[i] += offset
                    continue
                if num_beams > 1:  # pre-encoded first pass: this part's windows sit at encoder rows b0..
                    pre = pre_encoded and passes == 0
                    res = self.beam_pass(R, num_beams, tail, given, mnew, use_timestamps=return_timestamps,
                                         enc_row0=b0 if pre else 0, r_enc=n_chunks if pre else R, prefix=pfx,
                                         align=word_timestamps, num_frames=nf_part)
                else:
                    res = self.decode_pass(R, tail, given, mnew, use_timestamps=return_timestamps,
                                           align=word_timestamps, num_frames=nf_part, prefix=pfx)
                self._masked = False
                for j in range(R):
                    do_cond[j] = bool(condition)
                for j, i in enumerate(part):
                    if not known:
                        langs[i] = res.lang_ids[j]
                    passes_raw[i].append(list(res.tokens[j]))
                    seq = strip_generated(res.tokens[j], st.eot)
                    seg_tokens, offset = retrieve_segment(seq, seek[i], min(maxf[i] - seek[i], N_FRAMES),
                                                          st.timestamp_begin)
                    segs[i].extend(seg_tokens)
                    seg_lists[i].extend(segment_slices(seq, st.timestamp_begin))
                    if word_timestamps:
                        self._add_times(tts[i], res.token_ts[j], prompt_len + L, len(seg_tokens), seek[i])
                    seek[i] += offset
            passes += 1
            if max_passes is not None and passes >= max_passes:
                break
            if passes >= 4 * N_FRAMES:  # a zero seek advance would loop forever (as generate() would)
                raise RuntimeError("seek loop made no progress")
        self.last_langs = langs
        self.last_passes = passes_raw
        self.last_token_timestamps = tts if word_timestamps else None
        return segs

    @staticmethod
    def _add_times(out: List[float], token_ts: np.ndarray, P: int, n: int, seek: int) -> None:
        """A segment's token_timestamps (_retrieve_segment, :2034-2037): the pass's times of its n kept tokens (after the
        P prompt positions) + time_offset = seek * time_precision / input_stride."""
        off = np.float32(seek * 0.02 / 2)
        out.extend(float(np.float32(x) + off) for x in token_ts[P: P + n])

    def _fallback_pass(self, R: int, tail, given, max_new: int, return_timestamps: bool, fb: FallbackConfig,
                       windows: Sequence[int], pass_no: int, enc_row0: int = 0, r_enc: Optional[int] = None,
                       prefix=None, num_beams: int = 1, align: bool = False,
                       num_frames: Optional[Sequence[int]] = None):
        """generate_with_fallback (generation_whisper.py:970-1116) for one seek pass of R encoded rows: decode at
        the first temperature, re-decode the rows whose criteria fail at the next one, until none does or the
        temperatures run out. Returns per row the kept sequence (EOS removed), should_skip, the language ids, each
        row's last temperature, the beam count left for the rest of the generate() call and (align) each row's token
        times from the round that decided it (its round's batch: _postprocess_outputs per round, :1051).
        Bug-compatible with transformers: needs_fallback / should_skip are written at the row's position in the
        CURRENT (shrinking) subset, and the main loop reads should_skip by batch position (:1074-1088, :879); the
        no-speech probability of a retry round is read by subset position from the whole pass's (the processor's
        inputs are the pass's full batch, :999-1000, logits_process.py WhisperNoSpeechDetection); with num_beams > 1 a
        round at temperature <= 0 is a beam search (its average log-probability from the hypothesis' renormalised
        scores, beam_pass(criteria=True)), and a sampling round sets num_beams = 1 for the rest of the call
        (generation_config.num_beams, :1004-1005, never restored)."""
        st = self.gen.special
        V = self.d.vocab
        idx = list(range(R))
        seqs: List[Optional[List[int]]] = [None] * R
        skip = [False] * R
        langs = list(given) if given is not None else None
        ns_tok = st.notimestamps - 1 if fb.no_speech_threshold is not None else None  # no_timestamps_token_id - 1
        temps = list(fb.temperatures) or [None]
        final_t: List[Optional[float]] = [None] * R  # the temperature of each row's last round
        nb = num_beams
        ns_pass: Optional[List[float]] = None  # the first round's no-speech probabilities (the whole pass's rows)
        row_ts: List[Optional[np.ndarray]] = [None] * R
        for fi, t in enumerate(temps):
            do_sample = t is not None and t > 0.0
            if do_sample:
                nb = 1
            sub_lang = None if langs is None else [langs[i] for i in idx]
            sub_pfx = None if prefix is None else ([prefix[0][i] for i in idx], [prefix[1][i] for i in idx])
            sub_nf = None if num_frames is None else [num_frames[i] for i in idx]
            if nb > 1:
                res = self.beam_pass(len(idx), nb, tail, sub_lang, max_new, use_timestamps=return_timestamps,
                                     enc_rows=[enc_row0 + i for i in idx], r_enc=r_enc, prefix=sub_pfx,
                                     criteria=True, no_speech_token=ns_tok, align=align, num_frames=sub_nf)
            else:
                res = self.sample_pass(len(idx), tail, sub_lang, max_new,
                                       temperature=float(t) if do_sample else 0.0, top_k=fb.top_k, seed=fb.seed,
                                       row_keys=[fallback_row_key(windows[i], pass_no, fi) for i in idx],
                                       use_timestamps=return_timestamps, enc_rows=[enc_row0 + i for i in idx],
                                       r_enc=r_enc, no_speech_token=ns_tok, prefix=sub_pfx, align=align,
                                       num_frames=sub_nf)
            self._masked = False
            if align:
                for j, i in enumerate(idx):
                    row_ts[i] = res.token_ts[j]
            if ns_pass is None and res.no_speech_prob is not None:
                ns_pass = list(res.no_speech_prob)
            for i in idx:
                final_t[i] = t
            if langs is None and res.lang_ids is not None:  # detected on the first round (all rows)
                langs = list(res.lang_ids)
            new_idx = []
            for j, toks in enumerate(res.tokens):
                seq = fallback_sequence(toks, st.eot, st.eot)
                needs, sk = need_fallback(seq, res.sum_logprob[j], None if ns_pass is None else ns_pass[j], V, fb)
                skip[j] = sk
                if seq and seq[-1] == st.eot:
                    seq = seq[:-1]
                seqs[idx[j]] = seq
                if needs:
                    new_idx.append(idx[j])
            idx = new_idx
            if not idx or fi == len(temps) - 1:
                break
        return seqs, skip, langs if langs is not None else [None] * R, final_t, nb, (row_ts if align else None)

    @on_engine_streams
    def run_batches(self, sizes: Sequence[int], load=None, batch_kwargs: Optional[Sequence[dict]] = None,
                    **gen_kwargs) -> List[List[List[int]]]:
        """generate() over consecutive window batches with a two-slot software pipeline: while batch k decodes on
        the decoder stream, batch k+1's log-mel + encoder + cross-K/V run on enc_stream into the other slot.
        sizes[k] = windows in batch k (<= max_batch); load(k) fills wave[:sizes[k]] for batch k (queued on
        enc_stream; None = the waveforms are already resident). Returns generate()'s output per batch."""
        if any(n < 1 or n > self.max_batch for n in sizes):
            raise ValueError(f"batch sizes must be in [1, {self.max_batch}]")

        def prefetch(k, alone=True):
            with torch.cuda.stream(self.enc_stream):
                if load is not None:
                    load(k)
                self.logmel(sizes[k], slot=k % 2, sync=False)
                self.encode(sizes[k], row_map=False, seek=False, slot=k % 2, sync=False, alone=alone)

        def prefetch_steps(k):  # the same work as prefetch(k), queued chunk by chunk by an _EncoderPump
            with torch.cuda.stream(self.enc_stream):
                if load is not None:
                    load(k)
                self.logmel(sizes[k], slot=k % 2, sync=False)
            yield
            yield from self._encode_steps(sizes[k], row_map=False, seek=False, slot=k % 2, sync=False, alone=False)

        # the first prefetch is ordered after whatever the caller queued on the decoder stream
        self.enc_stream.wait_stream(self.stream)
        out = []
        self.batch_langs = []
        self.batch_passes = []
        self.batch_token_timestamps = []
        self.batch_prefixes = []
        overlap = self.overlap  # False: encoder and decoder strictly in turn
        if sizes:
            prefetch(0)
        for k, n in enumerate(sizes):
            if not overlap and k > 0:
                self.enc_stream.wait_stream(self.stream)
                prefetch(k)
            if overlap and k + 1 < len(sizes):  # runs beside the decode of batch k, queued between its decode steps
                self._pump = _EncoderPump(self, prefetch_steps(k + 1), ahead=self.pump_ahead)
                self._pump()
            kw = dict(gen_kwargs, **(batch_kwargs[k] if batch_kwargs else {}))
            kw["window_offset"] = kw.get("window_offset", 0) + sum(sizes[:k])
            try:
                out.append(self.generate(n, slot=k % 2, pre_encoded=True, **kw))
            finally:
                self._pump_drain()
                self._pump = None
            self.batch_langs.append(self.last_langs)
            self.batch_passes.append(self.last_passes)
            self.batch_token_timestamps.append(self.last_token_timestamps)
            self.batch_prefixes.append(self.last_pass_prefixes)
        self.use_slot(0)
        return out
