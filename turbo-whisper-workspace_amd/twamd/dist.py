"""Chunk data parallelism: one process per GPU, 30-s windows sharded over ranks, one all-gather.

The reference has no multi-GPU path (it hard-codes cuda:0, /root/reference/vocalis/core/audio_pipeline.py:191);
SURVEY.md §8e adds exactly one strategy for it. Windows are independent until `_decode_asr` stitches them
($TF/models/whisper/tokenization_whisper.py:901-1150), so:

  * `shard_range`      contiguous, order-preserving ranges: rank r takes windows [r*n/W, (r+1)*n/W)
  * each rank runs its windows through its own engine (weights replicated; no data-path collective)
  * `gather_tokens`    ONE all_gather_into_tensor of an int32 [n_local_max, 2 + T] array per rank
                       (col 0 = number of tokens, col 1 = language id or -1, then the tokens, pad -1);
                       T = the longest sequence over all ranks (one tiny MAX all-reduce agrees on it: a window
                       that ran several seek passes can return more than max_target_positions tokens)
  * rank order = window order, so the gathered rows are already the global window list for stitching.

Failures are collective: the same MAX all-reduce carries an error flag, so when one rank's engine raises, every
rank raises (the failing rank its own exception, the others `PeerError`) instead of the healthy ranks blocking in
the all-gather; a rank-0 input decode failure travels the same way through `broadcast_waveform`.

With the nccl backend (= RCCL on ROCm) the gather runs over xGMI from device tensors; with gloo (CPU tests)
from host tensors. Messages are tiny (1 h of audio = 120 windows x 450 x 4 B = 216 KB): latency-bound.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

MAX_TOKENS = 448  # max_target_positions: the longest sequence ONE decode pass can return


class PeerError(RuntimeError):
    """Raised on the ranks whose own work succeeded when another rank failed the same collective call."""


def world() -> Tuple[int, int]:
    """(rank, world_size) of the default group, (0, 1) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


# force_collective: run the collectives even in a world of one (an nccl = RCCL group of size 1 exercises the device-
# tensor all-gather / broadcast on a one-GPU box; the results must equal the host path's). TW_FORCE_COLLECTIVE=1 sets
# the default for every call.
FORCE_COLLECTIVE = os.environ.get("TW_FORCE_COLLECTIVE", "0") == "1"


def collective_path(force_collective: Optional[bool] = None) -> bool:
    """Whether the sharded path (broadcast, shard, all-gather) runs: more than one rank, or forced in an initialised
    world of one."""
    _, ws = world()
    forced = FORCE_COLLECTIVE if force_collective is None else bool(force_collective)
    return ws > 1 or (forced and dist.is_available() and dist.is_initialized())


def shard_range(n: int, world_size: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of the windows rank `rank` processes (r*n/W .. (r+1)*n/W)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world {world_size}")
    return rank * n // world_size, (rank + 1) * n // world_size


def shard_sizes(n: int, world_size: int) -> List[int]:
    return [shard_range(n, world_size, r)[1] - shard_range(n, world_size, r)[0] for r in range(world_size)]


def _coll_device(device: Optional[torch.device], group) -> torch.device:
    """Where a collective's buffers live: cuda for nccl (= RCCL), cpu for gloo."""
    if device is not None:
        return device
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
        else torch.device("cpu")


def agree(failed: bool, width: int, device: Optional[torch.device] = None, group=None) -> Tuple[bool, int]:
    """One MAX all-reduce of (error flag, sequence width): (did any rank fail, the widest sequence anywhere)."""
    t = torch.tensor([int(bool(failed)), int(width)], dtype=torch.int64, device=_coll_device(device, group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    f, w = t.cpu().tolist()
    return bool(f), int(w)


def pack_tokens(seqs: Sequence[Sequence[int]], langs: Optional[Sequence[Optional[int]]], rows: int,
                width: int = MAX_TOKENS) -> np.ndarray:
    """int32 [rows, 2 + width]: (len, lang, tokens..., -1 pad). rows >= len(seqs)."""
    if len(seqs) > rows:
        raise ValueError(f"{len(seqs)} sequences do not fit {rows} rows")
    out = np.full((rows, 2 + width), -1, np.int32)
    for i, s in enumerate(seqs):
        if len(s) > width:
            raise ValueError(f"window {i}: {len(s)} tokens > {width}")
        out[i, 0] = len(s)
        lg = None if langs is None else langs[i]
        out[i, 1] = -1 if lg is None else int(lg)
        out[i, 2: 2 + len(s)] = np.asarray(s, np.int32)
    return out


def unpack_tokens(arr: np.ndarray, n: int) -> Tuple[List[List[int]], List[Optional[int]]]:
    seqs, langs = [], []
    for i in range(n):
        k = int(arr[i, 0])
        seqs.append([int(t) for t in arr[i, 2: 2 + k]])
        langs.append(None if arr[i, 1] < 0 else int(arr[i, 1]))
    return seqs, langs


def gather_tokens(local_seqs: Sequence[Sequence[int]], local_langs: Optional[Sequence[Optional[int]]], n_total: int,
                  device: Optional[torch.device] = None, group=None, width: Optional[int] = None,
                  force_collective: Optional[bool] = None) -> Tuple[List[List[int]], List[Optional[int]]]:
    """All-gather every rank's window results; returns all n_total windows in global order (on every rank).

    `device`: where the collective's buffers live (a cuda device for RCCL, cpu for gloo; default: cuda when
    the default backend is nccl). `width`: a minimum number of token columns per row; the columns used are the max
    over ranks of it and of the longest local sequence, agreed with one MAX all-reduce that also reports a
    shard-size mismatch, so no rank is left waiting in the gather. force_collective: see FORCE_COLLECTIVE."""
    rank, ws = world()
    if not collective_path(force_collective):
        return [list(s) for s in local_seqs], list(local_langs) if local_langs is not None else [None] * len(
            local_seqs)
    sizes = shard_sizes(n_total, ws)
    bad = len(local_seqs) != sizes[rank]
    # always one collective agreement first: a shard-size mismatch on any rank is reported on every rank
    # before the gather, also when the caller fixed the width; the width is the max over ranks and the caller's
    failed, agreed = agree(bad, max([len(s) for s in local_seqs] + [int(width or 0)], default=0), device, group)
    if bad:
        raise ValueError(f"rank {rank} holds {len(local_seqs)} windows, its shard has {sizes[rank]}")
    if failed:
        raise PeerError("another rank's window shard did not match its range")
    width = max(agreed, 1)
    rows = max(max(sizes), 1)
    device = _coll_device(device, group)
    loc = torch.from_numpy(pack_tokens(local_seqs, local_langs, rows, width)).to(device)
    allt = torch.empty(ws * rows, 2 + width, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(allt, loc, group=group)
    arr = allt.cpu().numpy()
    seqs: List[List[int]] = []
    langs: List[Optional[int]] = []
    for r in range(ws):
        s, lg = unpack_tokens(arr[r * rows:], sizes[r])
        seqs.extend(s)
        langs.extend(lg)
    return seqs, langs


def broadcast_waveform(wav: Optional[np.ndarray], device: Optional[torch.device] = None, src: int = 0,
                       group=None, failed: bool = False, as_tensor: bool = False,
                       force_collective: Optional[bool] = None):
    """Rank `src` holds the decoded 16 kHz waveform; every rank returns a copy (length first, then samples):
    a host array, or with as_tensor the collective's own buffer (device memory under RCCL: no host round trip).

    `failed` (meaningful on `src`): decoding the input raised there. The length slot then carries -1: `src` gets
    None back (and re-raises its own error), every other rank raises PeerError, so no rank waits for samples."""
    rank, ws = world()
    if not collective_path(force_collective):
        return wav
    device = _coll_device(device, group)
    n = torch.tensor([-1 if (rank == src and failed) else (0 if wav is None else len(wav))], dtype=torch.int64,
                     device=device)
    dist.broadcast(n, src=src, group=group)
    if int(n.item()) < 0:
        if rank == src:
            return None
        raise PeerError(f"rank {src} failed to decode the input")
    buf = torch.empty(int(n.item()), dtype=torch.float32, device=device)
    if rank == src:
        buf.copy_(torch.from_numpy(np.ascontiguousarray(wav, np.float32)))
    dist.broadcast(buf, src=src, group=group)
    return buf if as_tensor else buf.cpu().numpy()


def transcribe_sharded(run_windows, wav: np.ndarray, windows: Sequence, device: Optional[torch.device] = None,
                       group=None, timed: bool = False, force_collective: Optional[bool] = None) -> List:
    """Every rank calls this with the same `windows` (chunk_iter windows over `wav`); each rank runs
    `run_windows(wav, windows[lo:hi]) -> List[List[int]]` on its own shard, then the results are all-gathered
    into the global window order. `timed`: run_windows returns (tokens, per-token times) pairs (word
    timestamps); the times are gathered too and the pairs are returned."""
    rank, ws = world()
    lo, hi = shard_range(len(windows), ws, rank)
    err: Optional[BaseException] = None
    toks: List = []
    bits: List = []
    try:
        local = run_windows(wav, list(windows[lo:hi])) if hi > lo else []
        if len(local) != hi - lo:
            raise ValueError(f"rank {rank}: {len(local)} results for {hi - lo} windows")
        # (inside the try: a malformed result must reach agree() too)
        toks = [list(t) for t, _ in local] if timed else [list(t) for t in local]
        bits = [np.asarray(ts, dtype=np.float32).view(np.int32).tolist() for _, ts in local] if timed else []
    except Exception as e:  # made collective below: every rank learns of it before anyone enters the gather
        err, toks, bits = e, [], []
    failed, width = agree(err is not None, max((len(t) for t in list(toks) + bits), default=0), device, group)
    if failed:
        if err is not None:
            raise err
        raise PeerError("transcription failed on another rank")
    seqs, _ = gather_tokens(toks, None, len(windows), device=device, group=group, width=width,
                            force_collective=force_collective)
    if not timed:
        return seqs
    # word timestamps: (tokens, per-token float32 times); the times travel as their int32 bit patterns
    tsb, _ = gather_tokens(bits, None, len(windows), device=device, group=group, width=width,
                           force_collective=force_collective)
    return [(s, np.asarray(b, dtype=np.int32).view(np.float32).tolist()) for s, b in zip(seqs, tsb)]


# ---- sharded _decode_asr -------------------------------------------------------------------------------------------
# $TF/models/whisper/tokenization_whisper.py:901-1150 walks the windows in order and carries a state from one window
# to the next (twamd.tokenizer.AsrStitcher.state). Each rank stitches its own shard of windows from the state it
# expects to come in — clean (every segment closed), with the exact last language and time offset of the windows
# before it, both computable from those windows' tokens and strides alone — and the closed chunks of all shards are
# gathered. The merge walks the shards in order: where a shard's assumed incoming state is the previous shard's
# final state, its chunks are taken as they are; otherwise (a segment left open across the shard boundary) that
# shard is stitched again from the true state. The result equals the serial _decode_asr by construction.

def _language_of(vocab, tokens) -> Optional[str]:
    """The last language token's name in one window's tokens (as AsrStitcher.feed reads them), or None."""
    from .tokenizer import LANGUAGE_NAMES
    st = vocab.special
    ids = list(tokens)
    if ids and ids[0] == st.startofprev:
        ids = ids[ids.index(st.sot):] if st.sot in ids else []
    special = vocab.all_special_ids
    for t in reversed(ids):
        if t in special:
            lang = LANGUAGE_NAMES.get(vocab.id_to_token[t][2:-2])
            if lang is not None:
                return lang
    return None


def assumed_state(vocab, outputs: Sequence[dict], lo: int) -> dict:
    """The incoming state a shard starting at window `lo` assumes: clean, last language and time offset exact."""
    from .tokenizer import AsrStitcher
    lang = None
    for o in reversed(outputs[:lo]):
        lang = _language_of(vocab, o["tokens"])
        if lang is not None:
            break
    t = 0.0
    for o in outputs[:lo]:  # the same float operations, in the same order, as AsrStitcher.feed
        if "stride" in o:
            chunk_len, stride_left, stride_right = o["stride"]
            t -= stride_left
            t += chunk_len - stride_right
    return AsrStitcher.initial_state(lang, t)


def shard_piece(vocab, outputs: Sequence[dict], lo: int, hi: int, **kw) -> tuple:
    """One shard's stitching: (assumed incoming state, its closed chunks, its final state)."""
    from .tokenizer import AsrStitcher
    st0 = assumed_state(vocab, outputs, lo)
    sti = AsrStitcher(vocab, state=st0, **kw)
    for o in outputs[lo:hi]:
        sti.feed(o)
    return st0, sti.chunks, sti.state()


def merge_pieces(vocab, outputs: Sequence[dict], pieces: Sequence[tuple], bounds: Sequence[Tuple[int, int]],
                 **kw) -> Tuple[str, dict]:
    """The serial _decode_asr result from the shards' pieces (see above); returns (text, optional)."""
    from .tokenizer import AsrStitcher
    chunks: List[dict] = []
    true = AsrStitcher.initial_state()
    restitched = 0
    for (assumed, ch, final), (lo, hi) in zip(pieces, bounds):
        if assumed == true:
            chunks.extend(ch)
            true = final
        else:  # a segment open across the boundary (or a skip in flight): this shard again, from the true state
            sti = AsrStitcher(vocab, state=true, **kw)
            for o in outputs[lo:hi]:
                sti.feed(o)
            chunks.extend(sti.chunks)
            true = sti.state()
            restitched += 1
    end = AsrStitcher(vocab, state=true, **kw)
    end.chunks = chunks
    merge_pieces.last_restitched = restitched
    return end.finish()


merge_pieces.last_restitched = 0


def stitch_sharded(vocab, outputs: Sequence[dict], group=None, force_collective: Optional[bool] = None,
                   **kw) -> Tuple[str, dict]:
    """decode_asr over every window (`outputs` in global order, identical on every rank), with the work split over
    the ranks: each stitches its own window shard, one all_gather_object brings the pieces to every rank, and every
    rank merges them (merge_pieces). kw: decode_asr's return_timestamps, return_language, time_precision,
    segment_size."""
    from .tokenizer import decode_asr
    rank, ws = world()
    # without timestamps no window closes its chunk (the text accumulates until the end), so every shard after the
    # first would be re-stitched by the merge: the plain serial pass is less work
    if not collective_path(force_collective) or not kw.get("return_timestamps"):
        return decode_asr(vocab, outputs, **kw)
    bounds = [shard_range(len(outputs), ws, r) for r in range(ws)]
    piece = shard_piece(vocab, outputs, *bounds[rank], **kw)
    pieces: List = [None] * ws
    dist.all_gather_object(pieces, piece, group=group)
    return merge_pieces(vocab, outputs, pieces, bounds, **kw)


class RankZeroFrontend:
    """Serving on N GPUs: rank 0 owns the request surface (AudioProcessingPipeline / POST /api/transcribe) and
    calls this like the single-GPU callable; the other ranks sit in `follow()`. Each call broadcasts the call's
    keyword arguments, then every rank enters the SPMD TurboTranscriber.__call__ (rank 0 decodes the input and
    broadcasts the waveform, windows are sharded, token arrays all-gathered)."""

    def __init__(self, transcriber, group=None):
        self.transcriber = transcriber
        self.group = group

    def __call__(self, inputs, **kwargs):
        dist.broadcast_object_list([kwargs], src=0, group=self.group)
        return self.transcriber(inputs, **kwargs)

    def close(self) -> None:
        dist.broadcast_object_list([None], src=0, group=self.group)

    def follow(self) -> int:
        """Loop of ranks != 0 until rank 0 calls close(); returns the number of calls served. A call that fails
        (collectively: rank 0 could not decode its input, or some rank's engine raised) is skipped here; rank 0
        raises it to its caller, which maps it to the reference's error convention."""
        n = 0
        while True:
            box = [None]
            dist.broadcast_object_list(box, src=0, group=self.group)
            if box[0] is None:
                return n
            try:
                self.transcriber(None, **box[0])
            except Exception as e:  # every rank saw the same failure; keep serving
                print(f"rank {dist.get_rank(self.group)}: call skipped: {e!r}")
                continue
            n += 1
