"""Word splitting and punctuation merging (SURVEY §8f-2 and the host half of a9) pinned to transformers.

faster-whisper 1.2.1 groups the aligned tokens into words with openai's tokenizer.split_to_word_tokens
(split_tokens_on_spaces / split_tokens_on_unicode) and merges punctuation with timing.merge_punctuations before it
builds Segment.words (which the reference's ts_words reads, asr_components.py:291-297).  faster-whisper is not
installed here; transformers 5.x carries the same algorithm as module functions of
transformers/models/whisper/tokenization_whisper.py: _split_tokens_on_unicode, _split_tokens_on_spaces,
_merge_punctuations and _combine_tokens_into_words (same punctuation sets as faster-whisper's defaults).

Both sides run on one byte-level BPE vocabulary trained here with `tokenizers` (English, punctuation, CJK), decoded by
the same `tokenizers` decoder; the transformers functions see it through a minimal adapter (decode with timestamps
rendered <|x.xx|> like WhisperTokenizer._decode_with_timestamps, eos_token_id = <|endoftext|>).  Compared on 40
sequences: encoded sentences with punctuation / quotes / brackets / CJK, and raw random id runs (which cut multi-byte
characters): the split words and token groups, the merged words, and the grouping that words_from_jumps and
add_word_timestamps build (empty merged-away entries dropped, as transformers drops them).
"""
import numpy as np
import pytest

from wmx.tokenizer import HFTokenizer
from wmx.transcribe import APPEND_PUNCT, PREPEND_PUNCT, merge_punctuations, words_from_jumps

tw = pytest.importorskip("transformers.models.whisper.tokenization_whisper")

V = 51866
LANG_NAME = {"en": "english", "zh": "chinese", "ja": "japanese", "de": "german"}


@pytest.fixture(scope="module")
def tok(tmp_path_factory):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=600, initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = ["hello world, this is a tiny whisper tokenizer test.", "the quick brown fox jumps over the lazy dog!",
              "\"quoted\" words (in brackets) and [more] {braces}: yes; no? 'single' - dash",
              "你好世界，语音识别。今天天气很好！", "日本語のテキスト、です。", "Grüße aus Köln — schön!"] * 20
    tk.train_from_iterator(corpus, tr)
    d = tmp_path_factory.mktemp("tok")
    tk.save(str(d / "tokenizer.json"))
    return HFTokenizer(str(d / "tokenizer.json"), V)


class _HFView:
    """What transformers' word functions need from a WhisperTokenizer."""

    def __init__(self, t: HFTokenizer):
        self.t = t
        self.eos_token_id = t.eot
        self.language = None

    def decode(self, tokens, decode_with_timestamps=False):
        tb = self.t.timestamp_begin
        out, run = [], []
        for x in tokens:
            if x >= tb:
                if run:
                    out.append(self.t.tk.decode(run, skip_special_tokens=False))
                    run = []
                out.append("<|%.2f|>" % ((x - tb) * 0.02))
            else:
                run.append(x)
        if run:
            out.append(self.t.tk.decode(run, skip_special_tokens=False))
        return "".join(out)


SENTENCES = [
    " hello world, this is a test.", " the quick brown fox jumps over the lazy dog!",
    " \"quoted\" words (in brackets) and [more] {braces}: yes; no?", " 'single' - dash, \"double\".",
    " 你好世界，语音识别。", " 今天天气很好！你好？", " 日本語のテキスト、です。", " Grüße aus Köln — schön!",
    " hello, world! (yes) [no] {maybe}.", " a-b c.d e,f g!h", " ¿qué? ¡sí! «non»", " 你好 world, 世界!",
    " “curly” quotes… and dashes —", " numbers 1, 2, 3. and 4!", " end with space ", " ((nested)) !!",
    " 语音、识别：测试。", " x y z", " 。，！", " \"", " hello", " 你",
]


def _cases(tok):
    rng = np.random.default_rng(0)
    cases = [(tok.encode(s), "zh" if any("　" <= c <= "鿿" for c in s) else "en") for s in SENTENCES]
    vocab_n = tok.tk.get_vocab_size()
    for i in range(18):  # raw id runs: words may cut multi-byte characters
        n = int(rng.integers(1, 24))
        cases.append(([int(x) for x in rng.integers(0, vocab_n, size=n)], "zh" if i % 3 == 0 else "en"))
    return cases


def test_split_to_word_tokens_matches_transformers(tok):
    view = _HFView(tok)
    n = 0
    for ids, lang in _cases(tok):
        seq = ids + [tok.eot]
        words, wt = tok.split_to_word_tokens(seq, lang)
        if lang == "zh":
            rw, rt, _ = tw._split_tokens_on_unicode(view, seq)
        else:
            rw, rt, _ = tw._split_tokens_on_spaces(view, seq)
        assert words == rw, (ids, lang, words, rw)
        assert [list(t) for t in wt] == [list(t) for t in rt], (ids, lang)
        n += 1
    assert n >= 40


def test_merge_punctuations_matches_transformers(tok):
    view = _HFView(tok)
    for ids, lang in _cases(tok):
        seq = ids + [tok.eot]
        words, wt = tok.split_to_word_tokens(seq, lang)
        align = [dict(word=w, tokens=list(t)) for w, t in zip(words, wt)]
        merge_punctuations(align, PREPEND_PUNCT, APPEND_PUNCT)
        ours = [(a["word"], a["tokens"]) for a in align if a["word"]]
        rw, rt, _ = tw._combine_tokens_into_words(view, seq, LANG_NAME[lang], PREPEND_PUNCT, APPEND_PUNCT)
        assert ours == list(zip(rw, [list(t) for t in rt])), (ids, lang, ours, list(zip(rw, rt)))


def test_words_from_jumps_grouping_matches_transformers(tok):
    """The word list faster-whisper's find_alignment + add_word_timestamps builds from the text tokens (grouping by
    split_to_word_tokens, start / end from the jump times at the word boundaries, then the punctuation merge):
    the surviving words and their tokens equal transformers' _combine_tokens_into_words, and every word's time span
    runs from its first token's jump time to its last token's successor's."""
    view = _HFView(tok)
    for k, (ids, lang) in enumerate(_cases(tok)):
        if not ids:
            continue
        jt = np.cumsum(np.random.default_rng(k).uniform(0.0, 0.3, len(ids) + 1)).astype(np.float32)
        align = words_from_jumps(tok, ids, jt, np.full(len(ids), 0.5, np.float32), lang)
        words, wt = tok.split_to_word_tokens(ids + [tok.eot], lang)
        if len(wt) <= 1:
            assert align == []
            continue
        pos = 0
        for a in align:  # times before the merge: the jump times at the word's token boundaries
            assert a["start"] == pytest.approx(float(jt[pos])) and a["end"] == pytest.approx(float(jt[pos + len(a["tokens"])]))
            pos += len(a["tokens"])
        merge_punctuations(align, PREPEND_PUNCT, APPEND_PUNCT)
        ours = [(a["word"], a["tokens"]) for a in align if a["word"]]
        # faster-whisper's pipeline on transformers' primitives: split text + <|endoftext|>, keep every word but the
        # last (its word_tokens[:-1] boundaries), merge punctuation
        split = tw._split_tokens_on_unicode if lang == "zh" else tw._split_tokens_on_spaces
        rw, rt, ri = split(view, ids + [tok.eot])
        rw, rt, ri = rw[:-1], [list(t) for t in rt[:-1]], ri[:-1]
        tw._merge_punctuations(rw, rt, ri, PREPEND_PUNCT, APPEND_PUNCT)
        ref = [(w, list(t)) for w, t in zip(rw, rt)]
        assert ours == ref, (ids, lang, ours, ref)
