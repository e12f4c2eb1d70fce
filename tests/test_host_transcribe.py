"""CPU tests of the faster-whisper host loop (wmx.transcribe.WhisperModel) over a fake decoding context:
language detected once and then fixed, the word-timestamp seek rule, the no-speech skip, control-token
suppression, keyword validation, and StreamBatcher's per-stream options and error handling.

Rules restated from faster-whisper 1.2.1 transcribe.py (not in the container):
  * generate_segments: `seek = round(last_word_end * frames_per_second)` when word_timestamps and the window does
    not end on a single timestamp; detect_language once before the loop; initial_prompt " " + prompt.strip();
  * get_suppressed_tokens: -1 -> non-speech set, + transcribe/translate/sot/sot_prev/sot_lm (+ no_speech, openai).
"""
import numpy as np
import pytest

from wmx import online as OL
from wmx import transcribe as TR
from wmx.engine import WindowResult
from wmx.tokenizer import DEFAULT_SUPPRESS, SpecialTokens, SyntheticTokenizer, suppressed_tokens

V = 51865
SP = SpecialTokens(V)
TB = SP.timestamp_begin


class FakeCtx:
    """Stands in for engine.Context: returns scripted windows and records what it was asked for."""

    def __init__(self, log, key, windows):
        self.log, self.key, self.windows = log, key, windows

    def transcribe(self, audios, prompts=None, seek=None):
        s = seek[0] if seek else 0
        self.log.append({"key": self.key, "seek": s, "prompt": list(prompts[0]) if prompts else [],
                         "n": len(audios)})
        return [self.windows(s, i) for i in range(len(audios))]

    def set_sample_seed(self, seed):
        self.log.append({"seed": (self.key, seed)})


def make_model(windows, max_batch=1):
    m = TR.WhisperModel.__new__(TR.WhisperModel)
    m.tokenizer = SyntheticTokenizer(V)
    m.name = "micro"
    m.max_batch = max_batch
    m.default_beam = 5
    m.max_new_tokens = 32
    m.suppress_tokens = [-1]
    m.use_graph = False
    m._ctx = {}
    m.log = []
    m.sample_seed, m._sample_calls = 1, 0

    def context(beam_size, language_token, task, word_timestamps, **kw):
        m.log.append({"context": (beam_size, language_token, task, word_timestamps, kw)})
        return FakeCtx(m.log, (beam_size, language_token, task), windows)

    m.context = context
    return m


def window(seek, i, lang=SP.lang0 + 1, no_speech=0.01, avg_lp=-0.3, single_ending=False):
    """Two timestamped segments: [0.00 t1 t2 1.00][1.00 t3 t4 2.00] (+ a trailing timestamp pair unless
    single_ending); DTW jump times put the last word's end at 1.87 s."""
    toks = [TB + 0, 101, 102, TB + 50, TB + 50, 103, 104, TB + 100]
    if not single_ending:
        toks += [TB + 100]
    jt = np.array([0.1, 0.5, 0.9, 1.3, 1.87], np.float32)
    return WindowResult(toks, lang, 0.9, -2.0, avg_lp, no_speech, seek, jt, np.full(4, 0.8, np.float32))


def test_language_detected_once_then_fixed():
    m = make_model(window)
    audio = np.zeros(16000 * 65, np.float32)  # 3 windows
    segs, info = m.transcribe(audio, language=None, word_timestamps=False)
    segs = list(segs)
    keys = [e["key"] for e in m.log if "key" in e]
    assert keys[0][1] is None  # first window: the engine detects
    assert all(k[1] == SP.lang0 + 1 for k in keys[1:])  # later windows: the detected language, fixed
    assert info.language == "zh" and len(keys) >= 3 and segs


def test_word_timestamp_seek_rule():
    m = make_model(window)
    audio = np.zeros(16000 * 40, np.float32)
    segs = list(m.transcribe(audio, word_timestamps=True)[0])
    seeks = [e["seek"] for e in m.log if "seek" in e]
    first_end = max(w.end for s in segs if s.seek == 0 for w in s.words)
    # not single-ending -> seek = round(last word end * 100), not the timestamp-token position (200)
    assert seeks[1] == round(first_end * 100) != 200
    # without word timestamps the timestamp rule applies: last consecutive pair ends at <|2.00|> -> 100 * 2 frames
    m2 = make_model(window)
    list(m2.transcribe(audio, word_timestamps=False)[0])
    assert [e["seek"] for e in m2.log if "seek" in e][1] == 200


def test_single_ending_window_advances_full_segment():
    m = make_model(lambda s, i: window(s, i, single_ending=True))
    list(m.transcribe(np.zeros(16000 * 40, np.float32), word_timestamps=True)[0])
    assert [e["seek"] for e in m.log if "seek" in e][:2] == [0, 3000]


def test_no_speech_skip_rule():
    # skipped: no_speech above threshold and avg_logprob not above log_prob_threshold
    m = make_model(lambda s, i: window(s, i, no_speech=0.9, avg_lp=-1.0))
    assert list(m.transcribe(np.zeros(16000 * 10, np.float32))[0]) == []
    # kept: a high enough log probability overrides the no-speech probability
    m = make_model(lambda s, i: window(s, i, no_speech=0.9, avg_lp=-0.5))
    assert list(m.transcribe(np.zeros(16000 * 10, np.float32))[0])


def test_initial_prompt_encoding_like_faster_whisper():
    m = make_model(window)
    list(m.transcribe(np.zeros(16000 * 5, np.float32), initial_prompt="  t12 t99 "))
    assert [e["prompt"] for e in m.log if "prompt" in e][0] == [12, 99]
    m = make_model(window)
    list(m.transcribe(np.zeros(16000 * 5, np.float32), initial_prompt=[5, 6, 7]))
    assert [e["prompt"] for e in m.log if "prompt" in e][0] == [5, 6, 7]


@pytest.mark.parametrize("kw,exc", [({"prefix": "so"}, NotImplementedError),
                                    ({"temperature": -0.2}, ValueError),
                                    ({"temperature": (0.0, float("nan"))}, ValueError),
                                    ({"hotwords": "abc"}, NotImplementedError),
                                    ({"no_such_option": 1}, TypeError)])
def test_unsupported_options_raise(kw, exc):
    m = make_model(window)
    with pytest.raises(exc):
        m.transcribe(np.zeros(16000, np.float32), **kw)


def test_supported_options_reach_the_context():
    m = make_model(window)
    list(m.transcribe(np.zeros(16000, np.float32), beam_size=3, patience=2.0, length_penalty=0.5,
                      vad_filter=False, temperature=[0.0], log_progress=True)[0])
    ctx = [e["context"] for e in m.log if "context" in e][0]
    assert ctx[0] == 3 and ctx[4]["patience"] == 2.0 and ctx[4]["length_penalty"] == 0.5


def test_suppressed_tokens_include_control_tokens():
    s = suppressed_tokens(SP, [-1])
    for t in (SP.transcribe, SP.translate, SP.sot, SP.sot_prev, SP.sot_lm, SP.no_speech):
        assert t in s
    assert set(DEFAULT_SUPPRESS) <= set(s)
    assert SP.eot not in s and TB not in s and SP.lang0 not in s
    s2 = suppressed_tokens(SP, [])
    assert set(s2) == {SP.transcribe, SP.translate, SP.sot, SP.sot_prev, SP.sot_lm, SP.no_speech}


class ASRView:
    sep = ""

    def __init__(self, lang=None, task=None):
        self.original_language = lang
        self.transcribe_kargs = {"beam_size": 5}
        if task:
            self.transcribe_kargs["task"] = task

    def ts_words(self, segments):
        return [(w.start, w.end, w.word) for s in segments for w in (s.words or [])]

    def segments_end_ts(self, segments):
        return [s.end for s in segments]


class BatchModel:
    def __init__(self, fail=()):
        self.calls, self.fail = [], set(fail)

    def transcribe_batch(self, audios, prompts, language=None, task="transcribe", beam_size=None, temperature=0.0,
                         best_of=5):
        self.calls.append({"n": len(audios), "language": language, "task": task, "beam": beam_size,
                           "temperature": temperature, "best_of": best_of})
        return [RuntimeError("boom") if i in self.fail else [] for i in range(len(audios))]


def _streams(n):
    out = []
    for _ in range(n):
        v = OL.VACOnlineASRProcessor(0.5, ASRView(), vad=OL.FixedVADIterator(OL.ScriptedVAD([0.9] * 400)))
        v.insert_audio_chunk(np.zeros(16000, np.float32))  # speech starts (padded start inside this chunk)
        v.insert_audio_chunk(np.zeros(16000, np.float32))  # voiced: the whole chunk reaches the processor
        assert v.wants_iter()
        out.append(v)
    return out


def test_stream_batcher_passes_language_and_task():
    bm = BatchModel()
    OL.StreamBatcher(bm, ASRView("zh", "translate")).step(_streams(3))
    assert bm.calls == [{"n": 3, "language": "zh", "task": "translate", "beam": 5, "temperature": 0.0, "best_of": 5}]


def test_stream_batcher_passes_the_adaptive_temperature():
    """speech_rate_audio_processor.py:217-218 raises temperature to 0.1 (beam 7) on fast speech; the batched path
    samples then instead of failing."""
    bm = BatchModel()
    view = ASRView()
    view.transcribe_kargs.update({"beam_size": 7, "temperature": 0.1})
    OL.StreamBatcher(bm, view).step(_streams(2))
    assert bm.calls[0]["temperature"] == 0.1 and bm.calls[0]["beam"] == 7


class StubAdaptive:
    """speech_rate_audio_processor.AdaptiveWhisperParams stand-in: the kwargs change between steps."""

    def __init__(self, seq):
        self.seq, self.i = list(seq), 0

    def get_transcribe_kwargs(self):
        kw = self.seq[min(self.i, len(self.seq) - 1)]
        self.i += 1
        return dict(kw)


def test_stream_batcher_merges_adaptive_params():
    """asr_components.py:270-275: adaptive_params.get_transcribe_kwargs() overrides transcribe_kargs on every call,
    on the batched path as on MI355XWhisperASR.transcribe."""
    bm = BatchModel()
    view = ASRView()
    view.adaptive_params = StubAdaptive([{"beam_size": 7, "temperature": 0.1}, {"beam_size": 3, "temperature": 0.0}])
    OL.StreamBatcher(bm, view).step(_streams(2))
    OL.StreamBatcher(bm, view).step(_streams(2))
    assert [(c["beam"], c["temperature"]) for c in bm.calls] == [(7, 0.1), (3, 0.0)]


@pytest.mark.parametrize("extra", [{"vad_filter": True}, {"patience": 2.0}, {"initial_prompt": "x"}])
def test_stream_batcher_rejects_unsupported_options(extra):
    bm = BatchModel()
    view = ASRView()
    view.transcribe_kargs.update(extra)
    with pytest.raises(NotImplementedError):
        OL.StreamBatcher(bm, view).step(_streams(1))
    view = ASRView()
    view.adaptive_params = StubAdaptive([extra])
    with pytest.raises(NotImplementedError):
        OL.StreamBatcher(bm, view).step(_streams(1))


def test_empty_prompt_same_on_both_batch_paths():
    """An empty-string prompt encodes " " on the multi-window path as on the one-window path (faster-whisper:
    initial_prompt is not None -> encode(" " + prompt.strip())); None encodes nothing."""
    class SpaceTok(SyntheticTokenizer):
        def encode(self, text):
            return [777] if text == " " else super().encode(text)

    for p, want in (("", [777]), (None, [])):
        m = make_model(window, max_batch=2)
        m.tokenizer = SpaceTok(V)
        m._sample_calls, m.sample_seed = 0, 1
        m.transcribe_batch([np.zeros(16000 * 40, np.float32), np.zeros(16000 * 5, np.float32)], [p, p])
        prompts = [e["prompt"] for e in m.log if "prompt" in e]
        # calls: the 40 s stream's first window (seek loop), its second window, then the 5 s stream (one batch)
        assert prompts[0] == want and prompts[-1] == want, (p, prompts)


def test_sampling_seed_differs_per_call_and_temperature():
    """Each T > 0 decode call draws with its own seed (fallback retries must not reuse one draw), and the
    same model seed replays the same sequence of seeds."""
    seeds = []

    class SeedCtx(FakeCtx):
        def set_sample_seed(self, s):
            seeds.append((self.key, s))

    def run():
        m = make_model(lambda s, i: window(s, i, avg_lp=-2.0))  # every attempt fails the log-prob check
        m.sample_seed, m._sample_calls = 7, 0
        m.context = lambda beam_size, language_token, task, word_timestamps, **kw: SeedCtx(
            m.log, (kw.get("temperature"),), lambda s, i: window(s, i, avg_lp=-2.0))
        list(m.transcribe(np.zeros(16000 * 40, np.float32), temperature=[0.0, 0.2, 0.4, 0.6])[0])
        return list(seeds)

    a = run()
    seeds.clear()
    b = run()
    assert a == b and len(a) >= 6  # 2 windows x 3 sampled temperatures
    assert len({s for _, s in a}) == len(a)
    assert TR.call_seed(7, 0, 1) != TR.call_seed(7, 0, 2) != TR.call_seed(7, 1, 1)


def test_stream_batcher_isolates_a_failing_stream():
    bm = BatchModel(fail={1})
    st = _streams(3)
    st[1].online.buffer_time_offset = 7.0
    outs = OL.StreamBatcher(bm, ASRView()).step(st)
    assert outs[1] == (None, None, "")
    assert st[1].online.buffer_time_offset == 7.0 and len(st[1].online.audio_buffer) == 0  # reset, offset kept
    assert len(st[0].online.audio_buffer) > 0  # the other streams are untouched


# ---- real-checkpoint host paths (SURVEY §8f-2 tokenizer, §8f-4 checkpoint config) ----
def _tiny_tokenizer_dir(tmp_path):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=400, initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = ["hello world, this is a tiny whisper tokenizer test.", "the quick brown fox jumps over the lazy dog!",
              "你好世界 speech recognition"] * 20
    tk.train_from_iterator(corpus, tr)
    tk.save(str(tmp_path / "tokenizer.json"))
    return str(tmp_path)


def test_hf_tokenizer_prompt_and_word_split(tmp_path):
    from wmx.tokenizer import HFTokenizer, load_tokenizer
    d = _tiny_tokenizer_dir(tmp_path)
    tok = load_tokenizer(d, V)
    assert isinstance(tok, HFTokenizer)
    text = " hello world, the quick fox!"
    ids = tok.encode(text)
    assert ids and all(0 <= t < tok.eot for t in ids)
    assert tok.decode(ids) == text
    # timestamps render like openai's decode_with_timestamps; decode() drops them
    assert tok.decode_with_timestamps([TB + 50] + ids[:2]).startswith("<|1.00|>")
    assert tok.decode(ids + [TB + 3]) == text
    # word grouping (split_tokens_on_spaces): words re-join to the text, punctuation is its own word
    words, wt = tok.split_to_word_tokens(ids + [tok.eot], "en")
    assert "".join(words[:-1]) == text
    assert [w.strip() for w in words[:-1]] == ["hello", "world", ",", "the", "quick", "fox", "!"]
    assert sum(len(t) for t in wt) == len(ids) + 1
    # unicode splitting (zh): every word decodes to whole characters
    zh = tok.encode("你好世界")
    zw, zt = tok.split_to_word_tokens(zh + [tok.eot], "zh")
    assert "".join(zw[:-1]) == "你好世界" and all("�" not in w for w in zw)
    # the prompt path of WhisperModel.transcribe: " " + prompt.strip()
    m = make_model(window)
    m.tokenizer = tok
    list(m.transcribe(np.zeros(16000 * 5, np.float32), initial_prompt="hello world ")[0])
    assert [e["prompt"] for e in m.log if "prompt" in e][0] == tok.encode(" hello world")


@pytest.mark.parametrize("cfg,name", [
    ({"d_model": 1280, "num_mel_bins": 128, "decoder_layers": 32, "encoder_layers": 32}, "large-v3"),
    ({"d_model": 1280, "num_mel_bins": 80, "decoder_layers": 32, "encoder_layers": 32}, "large-v2"),
    ({"d_model": 1280, "num_mel_bins": 128, "decoder_layers": 4, "encoder_layers": 32}, "large-v3-turbo"),
    ({"d_model": 384, "num_mel_bins": 80, "decoder_layers": 4, "encoder_layers": 4}, "tiny"),
    ({"d_model": 512, "num_mel_bins": 80, "decoder_layers": 6, "encoder_layers": 6}, "base")])
def test_checkpoint_config_names(tmp_path, cfg, name):
    import json
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    assert TR._infer_name(str(tmp_path)) == name


def _fallback_model(avg_lp_at):
    """A fake engine whose window quality depends on the decoding temperature: avg_lp_at(T) -> avg_logprob."""
    m = make_model(window)

    def context(beam_size, language_token, task, word_timestamps, **kw):
        t = kw.get("temperature", 0.0)
        m.log.append({"context": (beam_size, language_token, task, word_timestamps, kw)})
        return FakeCtx(m.log, (beam_size, language_token, task, t),
                       lambda s, i: window(s, i, avg_lp=avg_lp_at(t)))

    m.context = context
    return m


def test_temperature_fallback_stops_at_the_first_passing_temperature():
    """faster-whisper generate_with_fallback: T = 0 beam search, then best_of sampling at each higher T until
    avg_logprob >= log_prob_threshold (and the compression ratio passes)."""
    m = _fallback_model(lambda t: -1.5 if t < 0.4 else -0.5)
    list(m.transcribe(np.zeros(16000 * 5, np.float32), temperature=(0.0, 0.2, 0.4, 0.6), best_of=3, beam_size=4)[0])
    ctxs = [e["context"] for e in m.log if "context" in e]
    assert [c[4]["temperature"] for c in ctxs][:4] == [0.0, 0.2, 0.4, 0.0]  # window 1, then window 2 starts at 0
    assert all(c[4]["best_of"] == 3 for c in ctxs) and all(c[0] == 4 for c in ctxs)


def test_temperature_fallback_all_fail_keeps_best_and_resets_prompt():
    """Every temperature fails: the best avg_logprob is kept, reported at the last temperature (0.6 > 0.5 =
    prompt_reset_on_temperature), so the next window's prompt is reset."""
    lp = {0.0: -1.9, 0.2: -1.2, 0.6: -1.6}
    m = _fallback_model(lambda t: lp[t])
    segs = list(m.transcribe(np.zeros(16000 * 40, np.float32), temperature=(0.0, 0.2, 0.6))[0])
    assert segs and segs[0].avg_logprob == -1.2
    prompts = [e["prompt"] for e in m.log if "prompt" in e]
    assert prompts[3] == []  # window 2 (after 3 attempts at window 1): prompt reset since window 1's tokens


def test_single_temperature_is_one_decode():
    m = _fallback_model(lambda t: -3.0)  # fails the log-prob check, but there is nothing to fall back to
    segs = list(m.transcribe(np.zeros(16000 * 5, np.float32), temperature=0.1)[0])
    ctxs = [e["context"] for e in m.log if "context" in e]
    n_win = len([e for e in m.log if "seek" in e])
    assert len(ctxs) == n_win and all(c[4]["temperature"] == 0.1 and c[4]["best_of"] == 5 for c in ctxs)


# ---- vad_filter (faster-whisper 1.2.1 vad.py semantics, restated; parity unpinned: the package is absent) ----
def _vad_track():
    return np.array([0.0] * 10 + [0.9] * 20 + [0.0] * 100 + [0.9] * 10 + [0.0] * 10, np.float32)


def test_speech_timestamps_from_window_probabilities():
    from wmx import vad
    got = vad.get_speech_timestamps(_vad_track(), 150 * 512)
    # start at window 10 (5120), silence from window 30 lasts >= 2 s -> end 15360; the second run is open at the
    # end of the buffer; 400 ms padding, clipped to the buffer
    assert got == [{"start": 0, "end": 21760}, {"start": 60160, "end": 76800}]
    assert vad.get_speech_timestamps(_vad_track(), 150 * 512, min_speech_duration_ms=1000) == []  # both 640 ms runs dropped
    with pytest.raises(TypeError):
        vad.get_speech_timestamps(_vad_track(), 150 * 512, window_size_samples=1024)


def test_speech_timestamps_map():
    from wmx import vad
    chunks = [{"start": 0, "end": 21760}, {"start": 60160, "end": 76800}]
    m = vad.SpeechTimestampsMap(chunks, 16000)
    assert m.chunk_end_sample == [21760, 38400] and m.total_silence_before == [0.0, 2.4]
    assert m.get_original_time(1.0) == 1.0 and m.get_original_time(1.5) == 3.9
    assert m.get_original_time(21760 / 16000, is_end=True) == 1.36  # a chunk's own end stays in that chunk


def test_vad_filter_transcribes_speech_only_and_restores_times():
    class FakeEngine:
        max_windows = 64

        def reset(self, slot):
            self.pos = 0

        def process(self, chunk):
            (slot, x), = chunk.items()
            k = len(x) // 512
            p = _vad_track()[self.pos:self.pos + k]
            self.pos += k
            return {slot: p}

    m = make_model(window)
    m._vad = FakeEngine()
    m.vad_engine = lambda: m._vad
    segs, info = m.transcribe(np.zeros(150 * 512, np.float32), vad_filter=True, word_timestamps=False)
    segs = list(segs)
    assert info.duration == 4.8 and info.duration_after_vad == 2.4
    assert (segs[0].start, segs[0].end) == (0.0, 1.0) and (segs[1].start, segs[1].end) == (1.0, 4.4)


def test_batched_call_isolates_a_non_finite_window():
    """One stream's non-finite decode fails that stream only: the engine names the window in its
    WMX_ERR_NUMERIC error, transcribe_batch puts that error on the stream and re-runs the batch without it; the other
    streams get their segments (as they would from separate calls, the reference's per-stream processing)."""
    from wmx._lib import WMX_ERR_NUMERIC, WmxError

    class NaNCtx(FakeCtx):
        def transcribe(self, audios, prompts=None, seek=None):
            self.log.append({"n": len(audios)})
            for k, a in enumerate(audios):
                if np.isnan(a).any():
                    raise WmxError(f"non-finite decoder logits at decode step 3 (slot 5), row {5 * k + 1} "
                                   f"(window {k})", WMX_ERR_NUMERIC)
            return [window(0, i) for i in range(len(audios))]

    m = make_model(window, max_batch=4)
    m.context = lambda *a, **kw: NaNCtx(m.log, None, window)
    audios = [np.zeros(16000 * 3, np.float32) for _ in range(4)]
    audios[2][100] = np.nan
    out = m.transcribe_batch(audios, [""] * 4, word_timestamps=False)
    assert isinstance(out[2], WmxError) and out[2].status == WMX_ERR_NUMERIC
    for i in (0, 1, 3):
        assert isinstance(out[i], list) and out[i], i
    assert [e["n"] for e in m.log if "n" in e] == [4, 3]  # the batch, then the batch without the failed stream
