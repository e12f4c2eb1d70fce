"""CPU tests of the streaming caller (wmx.online) and the faster-whisper host post-processing (wmx.transcribe):
LocalAgreement-n, prompt building, segment trimming, VAD state machine, VAC gating, segment splitting by
timestamp tokens, word grouping and word-timestamp heuristics.  A fake ASR stands in for the GPU engine."""
import numpy as np
import pytest

from wmx import online as OL
from wmx.tokenizer import SpecialTokens, SyntheticTokenizer


class W:
    def __init__(self, s, e, w):
        self.start, self.end, self.word = s, e, w


class Seg:
    def __init__(self, words, end):
        self.words, self.end = words, end


class FakeASR:
    """Emits one word every 0.5 s of buffered audio; words are a deterministic function of absolute time, so
    successive transcriptions of a growing buffer agree on their common prefix (the LocalAgreement premise)."""
    sep = ""

    def __init__(self):
        self.calls = []

    def transcribe(self, audio, init_prompt=""):
        self.calls.append((len(audio), init_prompt))
        dur = len(audio) / 16000
        n = int(dur / 0.5)
        words = [W(i * 0.5, i * 0.5 + 0.4, f" w{i}") for i in range(n)]
        segs, cur = [], []
        for w in words:
            cur.append(w)
            if len(cur) == 4:
                segs.append(Seg(cur, cur[-1].end))
                cur = []
        if cur:
            segs.append(Seg(cur, cur[-1].end))
        return segs

    def ts_words(self, segments):
        return [(w.start, w.end, w.word) for s in segments for w in s.words]

    def segments_end_ts(self, segments):
        return [s.end for s in segments]


def test_hypothesis_buffer_local_agreement_2():
    hb = OL.HypothesisBuffer()
    hb.insert([(0.0, 0.4, " a"), (0.5, 0.9, " b")], 0)
    assert hb.flush() == []  # nothing to agree with yet
    hb.insert([(0.0, 0.4, " a"), (0.5, 0.9, " b"), (1.0, 1.4, " c")], 0)
    assert [w for _, _, w in hb.flush()] == [" a", " b"]
    assert hb.last_commited_time == 0.9
    # a re-transcription that repeats the committed tail drops the duplicate n-gram
    hb.insert([(0.5, 0.9, " b"), (1.0, 1.4, " c"), (1.5, 1.9, " d")], 0)
    assert [w for _, _, w in hb.new] == [" c", " d"]


def test_enhanced_buffer_local_agreement_3():
    hb = OL.EnhancedHypothesisBuffer(agreement_n=3)
    seq = [(0.0, 0.4, " a"), (0.5, 0.9, " b"), (1.0, 1.4, " c")]
    hb.insert(seq[:2], 0)
    assert hb.flush() == []
    hb.insert(seq, 0)
    assert hb.flush() == []
    hb.insert(seq + [(1.5, 1.9, " d")], 0)
    assert [w for _, _, w in hb.flush()] == [" a", " b"]


def test_online_processor_commits_and_trims():
    asr = FakeASR()
    p = OL.OnlineASRProcessor(asr, buffer_trimming=("segment", 3))
    committed = []
    rng = np.random.default_rng(0)
    for _ in range(20):
        p.insert_audio_chunk(rng.normal(0, 0.1, 8000).astype(np.float32))
        beg, end, text = p.process_iter()
        if text:
            committed.append(text)
    full = "".join(committed)
    assert full.startswith(" w0 w1")
    # trimming kept the buffer bounded
    assert len(p.audio_buffer) / 16000 <= 3 + 0.5 + 1e-6 or p.buffer_time_offset > 0
    assert p.buffer_time_offset > 0
    # later calls carry a prompt made of committed words scrolled out of the buffer
    assert any(pr for _, pr in asr.calls[-3:])


def test_enhanced_online_processor_prompt_limit_and_error_reset():
    asr = FakeASR()
    p = OL.EnhancedOnlineASRProcessor(asr, agreement_n=3)
    p.commited = [(i, i + 0.4, f" word{i:03d}") for i in range(100)]
    prompt, _ = p.prompt()
    assert len(prompt) <= 300 and prompt.endswith(" word099")

    class Boom(FakeASR):
        def transcribe(self, audio, init_prompt=""):
            raise RuntimeError("gpu error")

    q = OL.EnhancedOnlineASRProcessor(Boom(), agreement_n=2)
    q.insert_audio_chunk(np.zeros(16000, np.float32))
    assert q.process_iter() == (None, None, "")
    assert len(q.audio_buffer) == 0  # re-initialised


def test_dynamic_buffer_manager():
    m = OL.DynamicBufferManager(15, 5, 30)
    for _ in range(3):
        m.record_delay(5.0)
    assert m.adjust_trimming_sec() and m.get_trimming_sec() == 13
    m.recent_delays = [1.0]
    assert m.adjust_trimming_sec() and m.get_trimming_sec() == 15


def test_vad_iterator_rules():
    # windows of 512: speech from window 3 to 9, then silence
    probs = [0.1] * 3 + [0.9] * 7 + [0.1] * 30
    v = OL.VADIterator(OL.ScriptedVAD(probs), threshold=0.5, min_silence_duration_ms=100, speech_pad_ms=30)
    events = []
    for i in range(len(probs)):
        r = v(np.zeros(512, np.float32))
        if r:
            events.append((i, r))
    assert events[0] == (3, {"start": int(4 * 512 - 480 - 512)})
    end_i, end_ev = events[1]
    # silence starts at window 10 (temp_end = 11*512); end fires once 1600 samples of silence elapsed
    assert "end" in end_ev and end_ev["end"] == int(11 * 512 + 480 - 512)
    assert end_i == 10 + int(np.ceil(1600 / 512))


def test_dynamic_vad_silence_clamp():
    d = OL.DynamicVADIterator(OL.ScriptedVAD([]), initial_silence_ms=500, min_silence_ms=200, max_silence_ms=1000)
    assert d.set_silence_duration(5000) and d.vad.min_silence_samples == 16000
    assert not d.set_silence_duration(980)  # change <= 50 ms ignored
    assert d.set_silence_duration(100) and d.vad.min_silence_samples == 3200


def test_vac_processor_gates_asr_calls():
    asr = FakeASR()
    n = 80
    probs = [0.0] * 20 + [0.95] * 40 + [0.0] * (n - 60)
    vac = OL.VACOnlineASRProcessor(0.5, asr, vad=OL.FixedVADIterator(OL.ScriptedVAD(probs), min_silence_duration_ms=200))
    outs = []
    for _ in range(n * 512 // 640):
        vac.insert_audio_chunk(np.zeros(640, np.float32))
        outs.append(vac.process_iter())
    assert asr.calls, "voiced audio must reach the ASR"
    assert all(n_samples > 0 for n_samples, _ in asr.calls)
    assert any(o[2] for o in outs)


# ---------------- faster-whisper host logic ----------------
def test_split_segments_by_timestamps():
    from wmx.transcribe import split_segments_by_timestamps
    tb = 50364
    toks = [tb, 100, 101, tb + 50, tb + 50, 102, tb + 100]
    segs, seek, single = split_segments_by_timestamps(tb, toks, 0.0, 3000, 30.0, 0)
    assert single and seek == 3000
    assert [(s["start"], s["end"]) for s in segs] == [(0.0, 1.0), (1.0, 2.0)]
    toks2 = [tb, 100, tb + 40, tb + 40, 101]  # unfinished segment: seek to the last timestamp
    segs2, seek2, single2 = split_segments_by_timestamps(tb, toks2, 0.0, 3000, 30.0, 0)
    assert not single2 and seek2 == 40 * 2 and len(segs2) == 1
    segs3, seek3, _ = split_segments_by_timestamps(tb, [100, 101], 2.0, 500, 5.0, 100)
    assert segs3[0]["start"] == 2.0 and segs3[0]["end"] == 7.0 and seek3 == 600


def test_words_from_jumps_and_timestamps():
    from wmx.transcribe import add_word_timestamps, words_from_jumps
    tok = SyntheticTokenizer(51865)
    text = [10, 11, 12]
    jt = np.array([0.2, 0.6, 1.0, 1.3])
    al = words_from_jumps(tok, text, jt, np.array([0.9, 0.8, 0.7]), "en")
    assert [a["word"] for a in al] == [" t10", " t11", " t12"]
    assert [(a["start"], a["end"]) for a in al] == [(0.2, 0.6), (0.6, 1.0), (1.0, 1.3)]
    subs = [dict(seek=0, start=0.0, end=1.4, tokens=[50364] + text + [50364 + 70])]
    last = add_word_timestamps(subs, al, 0, 0.0)
    assert [w["word"] for w in subs[0]["words"]] == [" t10", " t11", " t12"]
    assert subs[0]["start"] == 0.2 and last == subs[0]["end"]


def test_merge_punctuations():
    from wmx.transcribe import merge_punctuations
    al = [dict(word=" (", tokens=[1]), dict(word=" hi", tokens=[2]), dict(word=",", tokens=[3])]
    merge_punctuations(al, "\"'“¿([{-", "\"'.。,，!！?？:：”)]}、")
    assert [a["word"] for a in al] == ["", " ( hi,", ""]


def test_special_token_layout():
    s2, s3 = SpecialTokens(51865), SpecialTokens(51866)
    assert (s2.transcribe, s2.timestamp_begin) == (50359, 50364)
    assert (s3.transcribe, s3.timestamp_begin, s3.language_token("yue")) == (50360, 50365, 50358)
    with pytest.raises(ValueError):
        s2.language_token("yue")
