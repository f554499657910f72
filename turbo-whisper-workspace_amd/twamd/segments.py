"""Host bookkeeping of Whisper's seek loop (integer token work, runs after each decode pass).

Restates, on plain int lists:
  * the pad / EOS stripping of WhisperGenerationMixin.generate_with_fallback
    ($TF/models/whisper/generation_whisper.py:1051-1071),
  * _retrieve_segment (:1977-2074) reduced to what the pipeline consumes: the tokens the pass
    contributes to the final sequence (segment slices are contiguous from 0, so their
    concatenation is a prefix of the sequence) and the seek advance in mel frames,
  * the final right padding of _pad_to_max_length (:125-232),
  * the temperature-fallback criteria of _need_fallback (:1243-1287): compression ratio
    (_retrieve_compression_ratio, :1949-1956), average log-probability (_retrieve_avg_logprobs, :1958-1975, from
    the device's per-row sum) and the no-speech skip.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

INPUT_STRIDE = 2  # conv1.stride * conv2.stride: mel frames per encoder position


def strip_generated(seq: Sequence[int], eos: int) -> List[int]:
    """Drop trailing pad tokens (pad == eos for Whisper) and then one EOS."""
    seq = list(seq)
    if seq and seq[-1] == eos:
        n_pad = sum(1 for t in seq if t == eos) - 1  # pad_token_id == eos_token_id keeps one EOS
        if n_pad:
            seq = seq[:-n_pad]
    if seq and seq[-1] == eos:
        seq = seq[:-1]
    return seq


def retrieve_segment(seq: Sequence[int], seek: int, seek_num_frames: int, timestamp_begin: int
                     ) -> Tuple[List[int], int]:
    """Tokens kept from this pass and the seek offset (frames) for one row."""
    ts = [t >= timestamp_begin for t in seq]
    single_ending = ts[-2:] == [False, True]
    pair_idx = [i + 1 for i in range(len(seq) - 1) if ts[i] and ts[i + 1]]
    if pair_idx:
        if single_ending:
            return list(seq), seek_num_frames
        end = pair_idx[-1] + 1          # the last pair's closing timestamp is kept
        last_ts_pos = seq[end - 2] - timestamp_begin
        return list(seq[:end]), last_ts_pos * INPUT_STRIDE
    return list(seq), seek_num_frames


def segment_slices(seq: Sequence[int], timestamp_begin: int) -> List[List[int]]:
    """The "tokens" of the segments _retrieve_segment (:1991-2072) cuts one pass into: at every pair of consecutive
    timestamps, the last slice ending after the closing timestamp (or at the end on a single timestamp ending);
    no pair: one segment of the whole sequence. Their concatenation is retrieve_segment's tokens."""
    seq = list(seq)
    ts = [t >= timestamp_begin for t in seq]
    pair_idx = [i + 1 for i in range(len(seq) - 1) if ts[i] and ts[i + 1]]
    if not pair_idx:
        return [seq]
    cuts = list(pair_idx)
    if ts[-2:] == [False, True]:
        cuts.append(len(seq))
    else:
        cuts[-1] += 1
    out, last = [], 0
    for c in cuts:
        out.append(seq[last:c])
        last = c
    return out


def condition_prefixes(segments: Sequence[Optional[Sequence[Sequence[int]]]], prev_sot, pad: int,
                       timestamp_begin: int, cut_off_length: int) -> Tuple[List[List[int]], List[int]]:
    """_prepare_decoder_input_ids' previous-token prompts (generation_whisper.py:1883-1906 via _pad_to_max_length with
    padding_side="left", skip_ending_double_timestamps=True, :126-232): per active row its segments' tokens (a segment
    ending in two timestamps loses the last one; None = the row is not conditioned), the last cut_off_length of them
    behind <|startofprev|>, left padded with `pad` to the longest. Returns (rows, pad counts).
    prev_sot: the token in front (an int), or a token list (prompt_condition_type="all-segments": the prompt_ids,
    generate()'s bos_token_tensor = prompt_ids, :1887-1888), or None."""
    bos = [] if prev_sot is None else [int(t) for t in prev_sot] if isinstance(prev_sot, (list, tuple)) else [prev_sot]
    seqs = []
    for segs in segments:
        if segs is not None and len(segs) > 0:
            toks: List[int] = []
            for d in segs:
                toks.extend(d[:-1] if len(d) > 2 and d[-2] >= timestamp_begin else d)
            toks = toks[-cut_off_length:] if cut_off_length else toks
            seqs.append(bos + toks)
        else:
            seqs.append(list(bos))
    L = max((len(x) for x in seqs), default=0)
    return [[pad] * (L - len(x)) + x for x in seqs], [L - len(x) for x in seqs]


def pad_right(seqs: Sequence[Sequence[int]], pad: int) -> List[List[int]]:
    n = max((len(s) for s in seqs), default=0)
    return [list(s) + [pad] * (n - len(s)) for s in seqs]


def fallback_sequence(seq: Sequence[int], pad: int, eos: int) -> List[int]:
    """generate_with_fallback's per-row cut (:1058-1066): every pad token removed from a sequence that ends on one,
    except one when pad == eos (the EOS counts in the average log-probability)."""
    seq = list(seq)
    if seq and seq[-1] == pad:
        n = sum(1 for t in seq if t == pad) - (1 if pad == eos else 0)
        if n:
            seq = seq[:-n]
    return seq


def compression_ratio(tokens: Sequence[int], vocab_size: int) -> float:
    """_retrieve_compression_ratio: raw little-endian token bytes over their zlib-compressed length."""
    length = int(math.log2(vocab_size) / 8) + 1
    raw = b"".join(int(t).to_bytes(length, "little") for t in tokens)
    return len(raw) / len(zlib.compress(raw))


@dataclass
class FallbackConfig:
    """The generate() kwargs of the temperature fallback (generation_whisper.py:398-401, 483-512)."""
    temperatures: Tuple[Optional[float], ...] = (None,)
    compression_ratio_threshold: Optional[float] = None
    logprob_threshold: Optional[float] = None
    no_speech_threshold: Optional[float] = None
    top_k: int = 50          # GenerationConfig's default, applied when sampling (TopKLogitsWarper)
    seed: int = 0

    @property
    def active(self) -> bool:
        """Anything beyond plain greedy decoding: sampling, or a criterion (which may skip a segment)."""
        return (any(t is not None and t > 0.0 for t in self.temperatures) or self.compression_ratio_threshold is not None
                or self.logprob_threshold is not None or self.no_speech_threshold is not None)


def need_fallback(seq: Sequence[int], sum_logprob: float, no_speech_prob: Optional[float], vocab_size: int,
                  cfg: FallbackConfig) -> Tuple[bool, bool]:
    """_need_fallback for one row: (needs_fallback, should_skip). seq is fallback_sequence's cut (EOS kept);
    sum_logprob the device's sum of log_softmax(scores)[token] over it."""
    needs, skip = False, False
    if cfg.compression_ratio_threshold is not None:
        if compression_ratio(seq, vocab_size) > cfg.compression_ratio_threshold:
            needs = True
    logprob = None
    if cfg.logprob_threshold is not None:
        logprob = sum_logprob / len(seq) if seq else float("-inf")
        if logprob < cfg.logprob_threshold:
            needs = True
    if cfg.no_speech_threshold is not None:
        if logprob is None:  # transformers reads an unset local here (UnboundLocalError)
            raise ValueError("no_speech_threshold needs logprob_threshold (generation_whisper.py:1275-1283)")
        if logprob < cfg.logprob_threshold and no_speech_prob > cfg.no_speech_threshold:
            needs, skip = False, True
    return needs, skip
