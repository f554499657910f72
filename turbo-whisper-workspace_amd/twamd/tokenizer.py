"""Whisper token decoding and the ASR pipeline's chunk stitching (host CPU, after the GPU passes).

* `WhisperVocab`: byte-level BPE id -> text (GPT-2 byte<->unicode table; the tokenizer's
  `decoders.ByteLevel()`, $TF/models/whisper/tokenization_whisper.py:239-251), built from a local
  checkpoint's vocab.json / added tokens or from the deterministic synthetic vocabulary.
* `decode_asr` restates `_decode_asr` ($TF/models/whisper/tokenization_whisper.py:901-1150) for
  return_timestamps in {False, True} and `_find_longest_common_sequence` (:1153-1270), driven by
  AutomaticSpeechRecognitionPipeline.postprocess (:600-710 of automatic_speech_recognition.py:
  stride samples -> seconds, time_precision = 30 / max_source_positions).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .config import LANGUAGE_CODES, SpecialTokens

# Whisper's LANGUAGES code -> name table (only the codes are needed to recognise language tokens;
# names are what _decode_asr stores in chunk["language"])
LANGUAGE_NAMES = {
    "en": "english", "zh": "chinese", "de": "german", "es": "spanish", "ru": "russian", "ko": "korean",
    "fr": "french", "ja": "japanese", "pt": "portuguese", "tr": "turkish", "pl": "polish", "ca": "catalan",
    "nl": "dutch", "ar": "arabic", "sv": "swedish", "it": "italian", "id": "indonesian", "hi": "hindi",
    "fi": "finnish", "vi": "vietnamese", "he": "hebrew", "uk": "ukrainian", "el": "greek", "ms": "malay",
    "cs": "czech", "ro": "romanian", "da": "danish", "hu": "hungarian", "ta": "tamil", "no": "norwegian",
    "th": "thai", "ur": "urdu", "hr": "croatian", "bg": "bulgarian", "lt": "lithuanian", "la": "latin",
    "mi": "maori", "ml": "malayalam", "cy": "welsh", "sk": "slovak", "te": "telugu", "fa": "persian",
    "lv": "latvian", "bn": "bengali", "sr": "serbian", "az": "azerbaijani", "sl": "slovenian", "kn": "kannada",
    "et": "estonian", "mk": "macedonian", "br": "breton", "eu": "basque", "is": "icelandic", "hy": "armenian",
    "ne": "nepali", "mn": "mongolian", "bs": "bosnian", "kk": "kazakh", "sq": "albanian", "sw": "swahili",
    "gl": "galician", "mr": "marathi", "pa": "punjabi", "si": "sinhala", "km": "khmer", "sn": "shona",
    "yo": "yoruba", "so": "somali", "af": "afrikaans", "oc": "occitan", "ka": "georgian", "be": "belarusian",
    "tg": "tajik", "sd": "sindhi", "gu": "gujarati", "am": "amharic", "yi": "yiddish", "lo": "lao",
    "uz": "uzbek", "fo": "faroese", "ht": "haitian creole", "ps": "pashto", "tk": "turkmen", "nn": "nynorsk",
    "mt": "maltese", "sa": "sanskrit", "lb": "luxembourgish", "my": "myanmar", "bo": "tibetan", "tl": "tagalog",
    "mg": "malagasy", "as": "assamese", "tt": "tatar", "haw": "hawaiian", "ln": "lingala", "ha": "hausa",
    "ba": "bashkir", "jw": "javanese", "su": "sundanese", "yue": "cantonese",
}


def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2 reversible byte <-> printable-unicode table."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def special_token_strings(st: SpecialTokens) -> Dict[int, str]:
    out = {st.eot: "<|endoftext|>", st.sot: "<|startoftranscript|>"}
    for i, code in enumerate(LANGUAGE_CODES[: st.n_languages]):
        out[st.lang_begin + i] = f"<|{code}|>"
    out.update({st.translate: "<|translate|>", st.transcribe: "<|transcribe|>", st.startoflm: "<|startoflm|>",
                st.startofprev: "<|startofprev|>", st.nospeech: "<|nospeech|>" if st.vocab == 51866 else "<|nocaptions|>",
                st.notimestamps: "<|notimestamps|>"})
    for i in range(1501):
        out[st.timestamp_begin + i] = f"<|{i * 0.02:.2f}|>"
    return out


def synthetic_vocab(st: SpecialTokens) -> List[str]:
    """Deterministic byte-level vocabulary of size st.vocab: ids < 256 are the 256 byte symbols, text ids
    up to eot are unique letter strings (even ids carry the 'Ġ' = space prefix), then the specials."""
    b2u = bytes_to_unicode()
    base = [b2u[b] for b in sorted(b2u, key=lambda x: list(b2u).index(x))]
    toks: List[str] = list(base)
    letters = "abcdefghijklmnopqrstuvwxyz"
    for i in range(256, st.eot):
        n, s = i, ""
        while n:
            s += letters[n % 26]
            n //= 26
        toks.append(("Ġ" + s) if i % 2 == 0 else s)
    spec = special_token_strings(st)
    for i in range(st.eot, st.vocab):
        toks.append(spec[i])
    return toks


class WhisperVocab:
    """id -> token string table plus byte-level decoding."""

    def __init__(self, id_to_token: Sequence[str], special: SpecialTokens):
        self.id_to_token = list(id_to_token)
        self.special = special
        self.byte_decoder = {v: k for k, v in bytes_to_unicode().items()}
        self.all_special_ids = set(special.special_ids())
        # per token: its bytes when every character is in the byte-level table (None otherwise), so decode() of
        # byte-level runs is one join + one UTF-8 decode (rank 0 stitches every window of a sharded hour on the host)
        bd = self.byte_decoder
        self._token_bytes = [bytes(bd[c] for c in t) if all(c in bd for c in t) else None for t in self.id_to_token]

    @staticmethod
    def synthetic(special: SpecialTokens) -> "WhisperVocab":
        return WhisperVocab(synthetic_vocab(special), special)

    @staticmethod
    def from_checkpoint(path: str, special: SpecialTokens) -> "WhisperVocab":
        with open(os.path.join(path, "vocab.json"), encoding="utf-8") as f:
            vocab = json.load(f)
        toks = [""] * special.vocab
        for t, i in vocab.items():
            if i < special.vocab:
                toks[i] = t
        added = os.path.join(path, "added_tokens.json")
        if os.path.exists(added):
            with open(added, encoding="utf-8") as f:
                for t, i in json.load(f).items():
                    if i < special.vocab:
                        toks[i] = t
        for i, t in special_token_strings(special).items():
            if not toks[i]:
                toks[i] = t
        return WhisperVocab(toks, special)

    def decode(self, ids: Sequence[int]) -> str:
        """tokenizer.decode(ids) for text tokens (specials render as their strings)."""
        tb = self._token_bytes
        try:
            return b"".join(tb[i] for i in ids).decode("utf-8", errors="replace")
        except TypeError:  # a token with characters outside the byte table: the general path below
            pass
        text = "".join(self.id_to_token[i] for i in ids)
        data = bytearray()
        out = []
        for ch in text:
            b = self.byte_decoder.get(ch)
            if b is None:  # special-token characters outside the byte table
                if data:
                    out.append(data.decode("utf-8", errors="replace"))
                    data = bytearray()
                out.append(ch)
            else:
                data.append(b)
        if data:
            out.append(data.decode("utf-8", errors="replace"))
        return "".join(out)


def find_longest_common_sequence(sequences: List[List[int]], token_timestamp_sequences=None):
    """Greedy overlap merge of consecutive token runs (the pipeline's stride stitching,
    $TF/models/whisper/tokenization_whisper.py:1153-1270). With token_timestamp_sequences (word timestamps) a match
    also needs the left token's (start, end) <= the right one's, the timestamps are split the same way, and the
    result is (tokens, timestamps)."""
    left = sequences[0]
    left_len = len(left)
    total: List[int] = []
    with_ts = bool(token_timestamp_sequences)
    if with_ts:
        left_ts = token_timestamp_sequences[0]
        total_ts: list = []
    for seq_idx, right in enumerate(sequences[1:]):
        best = 0.0
        best_idx = (left_len, left_len, 0, 0)
        right_len = len(right)
        if with_ts:
            for i in range(1, left_len + right_len):
                eps = i / 10000.0
                ls, le = max(0, left_len - i), min(left_len, left_len + right_len - i)
                rs, re_ = max(0, i - left_len), min(right_len, i)
                rts = token_timestamp_sequences[seq_idx + 1]
                matches = sum(1 for k in range(le - ls)
                              if left[ls + k] == right[rs + k] and tuple(left_ts[ls + k]) <= tuple(rts[rs + k]))
                matching = matches / i + eps
                if matches > 1 and matching > best:
                    best = matching
                    best_idx = (ls, le, rs, re_)
        elif left_len and right_len:
            # the same scan, vectorised: offset i aligns left[a] with right[b] where b - a = i - left_len, so the
            # matches at every offset are the diagonal sums of the equality matrix; the first offset with the
            # largest matches / i + i / 10000 (matches > 1) wins, as the strict '>' of the sequential scan picks it
            a, b = np.nonzero(np.asarray(left)[:, None] == np.asarray(right)[None, :])
            n = left_len + right_len
            matches = np.bincount(b - a + left_len, minlength=n)[1:n]
            i = np.arange(1, n)
            matching = matches / i + i / 10000.0
            ok = matches > 1
            if ok.any():
                k = int(np.argmax(np.where(ok, matching, -np.inf)))
                i_best = k + 1
                best_idx = (max(0, left_len - i_best), min(left_len, left_len + right_len - i_best),
                            max(0, i_best - left_len), min(right_len, i_best))
        ls, le, rs, re_ = best_idx
        lmid = (le + ls) // 2
        rmid = (re_ + rs) // 2
        total.extend(left[:lmid])
        left = right[rmid:]
        left_len = len(left)
        if with_ts:
            total_ts.extend(left_ts[:lmid])
            left_ts = token_timestamp_sequences[seq_idx + 1][rmid:]
    total.extend(left)
    if token_timestamp_sequences is None:
        return total
    if with_ts:
        total_ts.extend(left_ts)
        return total, total_ts
    return total, []


_PUNCT = "!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~"


def _split_tokens_on_unicode(vocab: "WhisperVocab", tokens: List[int]):
    """tokenization_whisper.py:1315-1344: cut wherever the decoded prefix is complete unicode."""
    decoded_full = vocab.decode(tokens)
    rep = "\ufffd"
    words, word_tokens, token_indices = [], [], []
    cur, cur_idx = [], []
    offset = 0
    for k, tok in enumerate(tokens):
        cur.append(tok)
        cur_idx.append(k)
        dec = vocab.decode(cur)
        if rep not in dec or offset + dec.index(rep) >= len(decoded_full) or decoded_full[offset + dec.index(rep)] == rep:
            words.append(dec)
            word_tokens.append(cur)
            token_indices.append(cur_idx)
            cur, cur_idx = [], []
            offset += len(dec)
    return words, word_tokens, token_indices


def _split_tokens_on_spaces(vocab: "WhisperVocab", tokens: List[int]):
    """:1347-1368: subwords start a new word on a leading space, a punctuation mark or a special token."""
    subwords, sub_tokens, sub_idx = _split_tokens_on_unicode(vocab, tokens)
    words, word_tokens, token_indices = [], [], []
    for sw, stoks, sidx in zip(subwords, sub_tokens, sub_idx):
        special = stoks[0] >= vocab.special.eot
        if special or sw.startswith(" ") or sw.strip() in _PUNCT or not words:
            words.append(sw)
            word_tokens.append(list(stoks))
            token_indices.append(list(sidx))
        else:
            words[-1] = words[-1] + sw
            word_tokens[-1].extend(stoks)
            token_indices[-1].extend(sidx)
    return words, word_tokens, token_indices


def _merge_punctuations(words, tokens, indices, prepended="\"'“¡¿([{-", appended="\"'.。,，!！?？:：”)]}、"):
    """:1371-1404."""
    i, j = len(words) - 2, len(words) - 1
    while i >= 0:
        if words[i].startswith(" ") and words[i].strip() in prepended:
            words[j] = words[i] + words[j]
            tokens[j] = tokens[i] + tokens[j]
            indices[j] = indices[i] + indices[j]
            words[i], tokens[i], indices[i] = "", [], []
        else:
            j = i
        i -= 1
    i, j = 0, 1
    while j < len(words):
        if not words[i].endswith(" ") and words[j] in appended:
            words[i] += words[j]
            tokens[i] += tokens[j]
            indices[i] += indices[j]
            words[j], tokens[j], indices[j] = "", [], []
        else:
            i = j
        j += 1
    words[:] = [w for w in words if w]
    tokens[:] = [t for t in tokens if t]
    indices[:] = [x for x in indices if x]


def collate_word_timestamps(vocab: "WhisperVocab", tokens: List[int], token_timestamps, language: Optional[str],
                            return_language: bool) -> List[dict]:
    """_collate_word_timestamps + _combine_tokens_into_words (:1273-1312)."""
    language = language or "english"
    if language in {"chinese", "japanese", "thai", "lao", "myanmar", "cantonese"}:
        words, wtoks, idx = _split_tokens_on_unicode(vocab, tokens)
    else:
        words, wtoks, idx = _split_tokens_on_spaces(vocab, tokens)
    _merge_punctuations(words, wtoks, idx)
    extra = {"language": language} if return_language else {}
    return [{"text": w, "timestamp": (token_timestamps[ix[0]][0], token_timestamps[ix[-1]][1]), **extra}
            for w, ix in zip(words, idx)]


class AsrStitcher:
    """`_decode_asr` as a resumable state machine: feed() the pipeline's model outputs in window order, finish() for
    (text, optional). Everything carried from one window to the next is `state()` — the open chunk, the token runs
    still waiting for their closing timestamp (and their word times), the skip flag, the last language and the time
    offset — so a shard of windows can be stitched from a given incoming state and its closed chunks concatenated
    with the other shards' (twamd.dist.stitch_sharded)."""

    def __init__(self, vocab: WhisperVocab, return_timestamps, return_language: bool = False,
                 time_precision: float = 0.02, segment_size: int = 1500, state: Optional[dict] = None):
        self.vocab, self.return_timestamps, self.return_language = vocab, return_timestamps, return_language
        self.time_precision, self.segment_size = time_precision, segment_size
        self.word = return_timestamps == "word"
        self.chunks: List[dict] = []  # closed chunks, in order
        st = state or self.initial_state()
        self.chunk = {"language": st["chunk"]["language"], "timestamp": list(st["chunk"]["timestamp"]),
                      "text": st["chunk"]["text"]}
        self.previous_tokens = [list(t) for t in st["previous_tokens"]]
        self.previous_token_timestamps = [list(t) for t in st["previous_token_timestamps"]]
        self.skip, self.last_language, self.time_offset = st["skip"], st["last_language"], st["time_offset"]

    @staticmethod
    def initial_state(last_language: Optional[str] = None, time_offset: float = 0.0) -> dict:
        """A clean state: no open chunk, nothing pending (what decode_asr starts from, and what holds after every
        window whose last segment closed)."""
        return {"chunk": {"language": last_language, "timestamp": [None, None], "text": ""}, "previous_tokens": [],
                "previous_token_timestamps": [], "skip": False, "last_language": last_language,
                "time_offset": time_offset}

    def state(self) -> dict:
        return {"chunk": {"language": self.chunk["language"], "timestamp": list(self.chunk["timestamp"]),
                          "text": self.chunk["text"]},
                "previous_tokens": [list(t) for t in self.previous_tokens],
                "previous_token_timestamps": [[tuple(x) for x in t] for t in self.previous_token_timestamps],
                "skip": self.skip, "last_language": self.last_language, "time_offset": self.time_offset}

    def _new_chunk(self) -> dict:
        return {"language": self.last_language, "timestamp": [None, None], "text": ""}

    def feed(self, output: dict) -> None:
        vocab, st, word = self.vocab, self.vocab.special, self.word
        time_precision, segment_size = self.time_precision, self.segment_size
        timestamp_begin = st.timestamp_begin
        special_ids = vocab.all_special_ids
        token_ids = list(output["tokens"])
        # _strip_prompt: a leading <|startofprev|> prompt is cut up to <|startoftranscript|>
        if token_ids and token_ids[0] == st.startofprev:
            token_ids = token_ids[token_ids.index(st.sot):] if st.sot in token_ids else []
        token_timestamps = list(output["token_timestamps"]) if word else None
        last_timestamp = None
        first_timestamp = timestamp_begin
        cur_max_timestamp = 0.0
        prev_segments_len = 0.0
        penultimate_timestamp = 0.0
        if "stride" in output:
            chunk_len, stride_left, stride_right = output["stride"]
            self.time_offset -= stride_left
            right_stride_start = chunk_len - stride_right
            if stride_left:
                first_timestamp = stride_left / time_precision + timestamp_begin
            if stride_right:
                for token in reversed(token_ids):
                    if token >= timestamp_begin:
                        if last_timestamp is not None and (token - timestamp_begin) * time_precision < right_stride_start:
                            break
                        last_timestamp = token
        current_tokens: List[int] = []
        current_token_timestamps: list = []
        chunk = self.chunk
        for i, token in enumerate(token_ids):
            if token in special_ids:
                text = vocab.id_to_token[token][2:-2]
                language = LANGUAGE_NAMES.get(text)
                if language is not None:
                    if self.last_language and language != self.last_language and not self.return_timestamps:
                        self.previous_tokens.append(current_tokens)
                        resolved = find_longest_common_sequence(self.previous_tokens)
                        chunk["text"] = vocab.decode(resolved)
                        self.chunks.append(chunk)
                        self.previous_tokens = []
                        current_tokens = []
                        chunk = self._new_chunk()
                    chunk["language"] = language
                    self.last_language = language
            elif token >= timestamp_begin:
                timestamp = float((token - timestamp_begin) * time_precision)
                if timestamp < cur_max_timestamp:
                    last_was_single_ending = i >= 2 and not (
                        token_ids[i - 1] >= timestamp_begin and token_ids[i - 2] >= timestamp_begin)
                    if last_was_single_ending:
                        prev_segments_len += time_precision * segment_size
                    else:
                        cur_max_timestamp = penultimate_timestamp
                        prev_segments_len += penultimate_timestamp
                penultimate_timestamp = cur_max_timestamp
                cur_max_timestamp = timestamp
                time = (token - timestamp_begin) * time_precision + self.time_offset + prev_segments_len
                time = round(time, 2)
                if last_timestamp and token >= last_timestamp:
                    self.skip = True
                elif self.skip or (self.previous_tokens and token < first_timestamp):
                    self.skip = False
                elif chunk["timestamp"][0] is None:
                    chunk["timestamp"][0] = time
                else:
                    if time == chunk["timestamp"][0]:
                        pass
                    else:
                        chunk["timestamp"][1] = time
                        self.previous_tokens.append(current_tokens)
                        if word:
                            self.previous_token_timestamps.append(current_token_timestamps)
                        resolved, resolved_ts = find_longest_common_sequence(self.previous_tokens,
                                                                             self.previous_token_timestamps)
                        chunk["text"] = vocab.decode(resolved)
                        if word:
                            chunk["words"] = collate_word_timestamps(vocab, resolved, resolved_ts, self.last_language,
                                                                     self.return_language)
                        self.chunks.append(chunk)
                        self.previous_tokens = []
                        current_tokens = []
                        self.previous_token_timestamps = []
                        current_token_timestamps = []
                        chunk = self._new_chunk()
            else:
                current_tokens.append(token)
                if word:
                    start = (round(0.0 + self.time_offset, 2) if i == 0
                             else round(token_timestamps[i - 1] + self.time_offset, 2))
                    current_token_timestamps.append((start, round(token_timestamps[i] + self.time_offset, 2)))
        if "stride" in output:
            self.time_offset += chunk_len - stride_right
        if current_tokens:
            self.previous_tokens.append(current_tokens)
            if word:
                self.previous_token_timestamps.append(current_token_timestamps)
        elif not any(p for p in self.previous_tokens):
            chunk = self._new_chunk()
            self.previous_tokens = []
            self.previous_token_timestamps = []
        self.chunk = chunk

    def finish(self) -> Tuple[str, dict]:
        chunks = list(self.chunks)
        if self.previous_tokens:
            chunk = self.chunk
            resolved, resolved_ts = find_longest_common_sequence(self.previous_tokens, self.previous_token_timestamps)
            chunk["text"] = self.vocab.decode(resolved)
            if self.word:
                chunk["words"] = collate_word_timestamps(self.vocab, resolved, resolved_ts, self.last_language,
                                                         self.return_language)
            chunks.append(chunk)
        return assemble_asr(chunks, self.return_timestamps, self.return_language)


def assemble_asr(chunks: List[dict], return_timestamps, return_language: bool) -> Tuple[str, dict]:
    """The tail of _decode_asr: the full text and the optional chunk / word list from the closed chunks."""
    word = return_timestamps == "word"
    full_text = "".join(c["text"] for c in chunks)
    if return_timestamps or return_language:
        for c in chunks:
            if not return_timestamps:
                c.pop("timestamp")
            else:
                c["timestamp"] = tuple(c["timestamp"])
            if not return_language:
                c.pop("language")
        if word:
            optional = {"chunks": [w for c in chunks for w in c["words"]]}
        else:
            optional = {"chunks": chunks}
    else:
        optional = {}
    return full_text, optional


def decode_asr(vocab: WhisperVocab, outputs: Sequence[dict], return_timestamps, return_language: bool = False,
               time_precision: float = 0.02, segment_size: int = 1500) -> Tuple[str, dict]:
    """outputs: [{"tokens": [ids...], "stride": (chunk_len_s, left_s, right_s) optional,
    "token_timestamps": [s...] (return_timestamps="word")}, ...] in chunk order."""
    stitcher = AsrStitcher(vocab, return_timestamps, return_language, time_precision, segment_size)
    for output in outputs:
        stitcher.feed(output)
    return stitcher.finish()
