"""Whisper tokenizer surface used by the host side (prompt encoding, word splitting, text).

faster-whisper wraps the HF `tokenizers` BPE of the checkpoint (tokenizer.json).  No vocabulary is reachable
offline, so two backends exist:
  * HFTokenizer: a real tokenizer.json (when a checkpoint directory provides one), via the `tokenizers` package;
  * SyntheticTokenizer: every id < eot decodes to " t<id>" — a deterministic stand-in so the whole pipeline
    (prompt ids, word grouping, text, LocalAgreement) runs end-to-end with synthetic weights.
Special-token ids follow openai-whisper tokenizer.py (large-v3 shifts everything after the languages by one).
"""
from __future__ import annotations

import os
import string

LANGUAGES = [
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it",
    "id", "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur",
    "hr", "bg", "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn",
    "et", "mk", "br", "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si",
    "km", "sn", "yo", "so", "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo",
    "ht", "ps", "tk", "nn", "mt", "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha",
    "ba", "jw", "su", "yue",
]

# openai-whisper tokenizer.non_speech_tokens for the multilingual GPT-2 vocabulary as shipped in the HF
# generation_config "suppress_tokens" (faster-whisper's suppress_tokens=[-1] expands to this set); only valid
# for the real multilingual vocabulary, not verifiable offline.
DEFAULT_SUPPRESS = [
    1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93, 359, 503, 522, 542, 873,
    893, 902, 918, 922, 931, 1350, 1853, 1982, 2460, 2627, 3246, 3253, 3268, 3536, 3846, 3961, 4183, 4667, 6585,
    6647, 7273, 9061, 9383, 10428, 10929, 11938, 12033, 12331, 12562, 13793, 14157, 14635, 15265, 15618, 16553,
    16604, 18362, 18956, 20075, 21675, 22520, 26130, 26161, 26435, 28279, 29464, 31650, 32302, 32470, 36865,
    42863, 47425, 49870, 50254,
]


def suppressed_tokens(sp, suppress_tokens=(-1,)):
    """faster-whisper 1.2.1 get_suppressed_tokens (openai decoding._get_suppress_tokens): -1 expands to the
    non-speech symbols; the task / sot / prev / lm control tokens are always suppressed, and so is no_speech
    (openai), so a sampled or beam-searched sequence can never emit a control token into the text or the prompt
    history."""
    toks = list(suppress_tokens or [])
    if -1 in toks:
        toks = [t for t in toks if t >= 0] + list(DEFAULT_SUPPRESS)
    toks += [sp.transcribe, sp.translate, sp.sot, sp.sot_prev, sp.sot_lm, sp.no_speech]
    return sorted(set(int(t) for t in toks))


class SpecialTokens:
    def __init__(self, n_vocab: int):
        self.n_langs = 100 if n_vocab >= 51866 else 99
        self.eot = 50257
        self.sot = 50258
        self.lang0 = 50259
        base = 50259 + self.n_langs
        self.translate, self.transcribe, self.sot_lm, self.sot_prev = base, base + 1, base + 2, base + 3
        self.no_speech, self.no_timestamps, self.timestamp_begin = base + 4, base + 5, base + 6

    def language_token(self, code: str) -> int:
        i = LANGUAGES.index(code)
        if i >= self.n_langs:
            raise ValueError(f"language {code} not in this vocabulary")
        return self.lang0 + i

    def language_code(self, token: int) -> str:
        return LANGUAGES[token - self.lang0]


class _Base:
    def __init__(self, n_vocab: int):
        self.sp = SpecialTokens(n_vocab)
        self.eot = self.sp.eot
        self.timestamp_begin = self.sp.timestamp_begin

    # --- openai tokenizer.split_to_word_tokens ---
    def split_to_word_tokens(self, tokens, language: str = "en"):
        if language in {"zh", "ja", "th", "lo", "my", "yue"}:
            return self.split_tokens_on_unicode(tokens)
        return self.split_tokens_on_spaces(tokens)

    def split_tokens_on_unicode(self, tokens):
        """openai / faster-whisper split_tokens_on_unicode, with the bounds guard transformers adds: a run that ends
        inside a cut multi-byte character (the replacement character lies past the full decode) closes a word
        instead of raising IndexError."""
        decoded_full = self.decode_with_timestamps(tokens)
        rc = "�"
        words, word_tokens, current, offset = [], [], [], 0
        for t in tokens:
            current.append(t)
            dec = self.decode_with_timestamps(current)
            if (rc not in dec or offset + dec.index(rc) >= len(decoded_full)
                    or decoded_full[offset + dec.index(rc)] == rc):
                words.append(dec)
                word_tokens.append(current)
                current = []
                offset += len(dec)
        return words, word_tokens

    def split_tokens_on_spaces(self, tokens):
        subwords, subword_tokens = self.split_tokens_on_unicode(tokens)
        words, word_tokens = [], []
        for sw, st in zip(subwords, subword_tokens):
            special = st[0] >= self.eot
            with_space = sw.startswith(" ")
            punct = sw.strip() in string.punctuation
            if special or with_space or punct or not words:
                words.append(sw)
                word_tokens.append(list(st))
            else:
                words[-1] = words[-1] + sw
                word_tokens[-1].extend(st)
        return words, word_tokens

    def decode(self, tokens):
        return self.decode_with_timestamps([t for t in tokens if t < self.eot])


class SyntheticTokenizer(_Base):
    """Deterministic stand-in vocabulary: id -> " t<id>", words are single tokens."""

    def encode(self, text: str):
        out = []
        for w in text.split():
            if w.startswith("t") and w[1:].isdigit() and int(w[1:]) < self.eot:
                out.append(int(w[1:]))
            else:  # map arbitrary words into the vocabulary deterministically
                out.append(sum(ord(c) * 31 ** i for i, c in enumerate(w)) % 50000 + 256)
        return out

    def decode_with_timestamps(self, tokens):
        parts = []
        for t in tokens:
            if t >= self.timestamp_begin:
                parts.append(f"<|{(t - self.timestamp_begin) * 0.02:.2f}|>")
            elif t >= self.eot:
                parts.append("<|endoftext|>" if t == self.eot else f"<|special{t}|>")
            else:
                parts.append(f" t{t}")
        return "".join(parts)


class HFTokenizer(_Base):
    """tokenizer.json of a real checkpoint (faster-whisper loads the same file)."""

    def __init__(self, path: str, n_vocab: int):
        super().__init__(n_vocab)
        from tokenizers import Tokenizer
        self.tk = Tokenizer.from_file(path)

    def encode(self, text: str):
        return self.tk.encode(text, add_special_tokens=False).ids

    def decode_with_timestamps(self, tokens):
        out, run = [], []
        for t in tokens:
            if t >= self.timestamp_begin:
                if run:
                    out.append(self.tk.decode(run))
                    run = []
                out.append(f"<|{(t - self.timestamp_begin) * 0.02:.2f}|>")
            else:
                run.append(t)
        if run:
            out.append(self.tk.decode(run, skip_special_tokens=False))
        return "".join(out)


def load_tokenizer(model_dir: str | None, n_vocab: int):
    if model_dir:
        p = os.path.join(model_dir, "tokenizer.json")
        if os.path.exists(p):
            return HFTokenizer(p, n_vocab)
    return SyntheticTokenizer(n_vocab)
