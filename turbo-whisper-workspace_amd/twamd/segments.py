"""Host bookkeeping of Whisper's seek loop (integer token work, runs after each decode pass).

Restates, on plain int lists:
  * the pad / EOS stripping of WhisperGenerationMixin.generate_with_fallback
    ($TF/models/whisper/generation_whisper.py:1051-1071),
  * _retrieve_segment (:1977-2074) reduced to what the pipeline consumes: the tokens the pass
    contributes to the final sequence (segment slices are contiguous from 0, so their
    concatenation is a prefix of the sequence) and the seek advance in mel frames,
  * the final right padding of _pad_to_max_length (:125-232).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

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


def pad_right(seqs: Sequence[Sequence[int]], pad: int) -> List[List[int]]:
    n = max((len(s) for s in seqs), default=0)
    return [list(s) + [pad] * (n - len(s)) for s in seqs]
