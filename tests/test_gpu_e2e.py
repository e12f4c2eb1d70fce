"""GPU end-to-end: the drop-in MI355XWhisperASR (reference CustomFasterWhisperASR surface) driven by the
streaming processors, single stream and batched multi-stream, on a small synthetic model."""
import numpy as np
import pytest

from wmx import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def asr():
    from wmx.asr import MI355XWhisperASR
    return MI355XWhisperASR(lan="auto", modelsize="micro", device="cuda", compute_type="float16",
                            transcribe_kwargs={"beam_size": 5}, max_new_tokens=24)


def test_asr_surface(asr):
    audio = synth.speech_like(3, 16000 * 6)
    segs = asr.transcribe(audio, init_prompt="t12 t99")
    words = asr.ts_words(segs)
    ends = asr.segments_end_ts(segs)
    assert asr.sep == ""
    assert len(ends) == len(segs)
    for s, e, w in words:
        assert 0.0 <= s <= e <= 6.5 and isinstance(w, str)
    for seg in segs:
        assert seg.start <= seg.end and 0.0 <= seg.no_speech_prob <= 1.0
    asr.set_translate_task()
    assert asr.transcribe_kargs["task"] == "translate"
    segs2 = asr.transcribe(audio)
    assert isinstance(segs2, list)
    del asr.transcribe_kargs["task"]


def test_streaming_processor_on_gpu(asr):
    from wmx.online import EnhancedOnlineASRProcessor
    p = EnhancedOnlineASRProcessor(asr, buffer_trimming=("segment", 15), agreement_n=2)
    audio = synth.speech_like(4, 16000 * 8)
    outs = []
    for i in range(0, len(audio), 8000):  # 0.5 s cadence (reference 一键.py:1510)
        p.insert_audio_chunk(audio[i: i + 8000])
        outs.append(p.process_iter())
    outs.append(p.finish())
    for beg, end, text in outs:
        if beg is not None:
            assert beg <= end


def test_stream_batcher_matches_single_stream_calls(asr):
    """B streams through one batched launch give the same words as B separate calls."""
    from wmx.online import StreamBatcher
    model = asr.model
    audios = [synth.speech_like(20 + i, 16000 * (4 + i)) for i in range(3)]
    model.max_batch = 3
    model._ctx.clear()
    batched = model.transcribe_batch(audios, ["", "t5 t6", ""])
    model.max_batch = 1
    model._ctx.clear()
    single = [model.transcribe_batch([a], [p])[0] for a, p in zip(audios, ["", "t5 t6", ""])]
    for b, s in zip(batched, single):
        assert [seg.tokens for seg in b] == [seg.tokens for seg in s]
    assert StreamBatcher(model, asr) is not None


def test_stream_batcher_two_groups_in_step_match_single_stream_calls(asr):
    """WhisperModel.groups = 2 (bench.py's stream_load): a batch of 4 streams split over two contexts decoding
    concurrently in step (wmx_ctx_set_lockstep) gives the same words as 4 separate calls, twice in a row."""
    model = asr.model
    audios = [synth.speech_like(40 + i, 16000 * (3 + i)) for i in range(4)]
    prompts = ["", "t5 t6", "", "t9"]
    model.max_batch = 1
    model._ctx.clear()
    single = [model.transcribe_batch([a], [p])[0] for a, p in zip(audios, prompts)]
    model.max_batch = 4
    model._ctx.clear()
    model.groups = 2
    try:
        for rep in range(2):
            grouped = model.transcribe_batch(audios, prompts)
            for b, s_ in zip(grouped, single):
                assert not isinstance(b, Exception), b
                assert [seg.tokens for seg in b] == [seg.tokens for seg in s_], rep
        assert sum(1 for k in model._ctx if len(k) == 14) == 2  # the two group contexts (options + (g, n))
    finally:
        model.groups = 1
        model._ctx.clear()


@pytest.mark.parametrize("kind,n", [("zeros", 32000), ("noise", 16000), ("speech", 8000), ("speech", 16000 * 31),
                                    ("speech", 116800), ("empty", 0)])
def test_asr_controls_and_lengths(asr, kind, n):
    """SURVEY §8d controls: all-zeros, white noise, 0.5 s / 7.3 s / 31 s (> one 30 s window: the seek loop moves
    to a second window) and empty input; every word lies inside the audio and segments are time-ordered."""
    audio = {"zeros": lambda: np.zeros(n, np.float32), "noise": lambda: synth.white_noise(5, n),
             "speech": lambda: synth.speech_like(6, n), "empty": lambda: np.zeros(0, np.float32)}[kind]()
    segs = asr.transcribe(audio)
    dur = n / 16000.0
    if n == 0:
        assert segs == []
        return
    prev = 0.0
    for seg in segs:
        assert prev - 1e-6 <= seg.start <= seg.end <= dur + 0.02, (seg.start, seg.end, dur)
        prev = seg.start
    for s, e, w in asr.ts_words(segs):
        assert 0.0 <= s <= e <= dur + 0.02


def test_config2_base_fp16_streaming_vac_1s_chunks():
    """BASELINE config 2 plumbing: Whisper base fp16 (PRNG weights of the base architecture) behind the drop-in
    ASR, driven through DynamicVACOnlineASRProcessor (reference asr_components.py:81-179) with 1 s online
    chunks fed at the 640-sample VAC cadence (一键.py:1286) and a scripted VAD track (Silero is not available
    offline).  Every ASR call sees a growing buffer; committed words are time-ordered and inside the audio."""
    import time
    from wmx.asr import MI355XWhisperASR
    from wmx.online import DynamicVACOnlineASRProcessor, ScriptedVAD
    asr = MI355XWhisperASR(lan="auto", modelsize="base", device="cuda", compute_type="float16",
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=16)
    calls = []
    inner = asr.transcribe

    def timed(audio, init_prompt=""):
        t0 = time.perf_counter()
        out = inner(audio, init_prompt=init_prompt)
        calls.append((len(audio), time.perf_counter() - t0))
        return out

    asr.transcribe = timed
    secs = 12
    n_win = secs * 16000 // 512
    probs = [0.0] * 30 + [0.95] * (n_win - 60) + [0.0] * 30  # silence, speech, silence
    vac = DynamicVACOnlineASRProcessor(1.0, asr, vad_model=ScriptedVAD(probs))
    audio = synth.speech_like(8, secs * 16000)
    committed = []
    for i in range(0, len(audio), 640):
        vac.insert_audio_chunk(audio[i: i + 640])
        beg, end, text = vac.process_iter()
        if beg is not None:
            committed.append((beg, end, text))
    beg, end, text = vac.finish()
    if beg is not None:
        committed.append((beg, end, text))
    assert calls, "voiced audio must reach the ASR"
    assert all(n > 0 for n, _ in calls)
    prev = 0.0
    for b, e, _ in committed:
        assert prev - 1e-6 <= b <= e <= secs + 0.05
        prev = b
    lat = sorted(t for _, t in calls)
    print(f"config 2: {len(calls)} ASR calls, p50 latency {1000 * lat[len(lat) // 2]:.1f} ms, "
          f"{len(committed)} commits")


def test_nonfinite_decode_is_an_error_not_a_short_transcript():
    """A NaN anywhere upstream of the logits (here one LayerNorm gain of decoder layer 0) must surface as an error, not
    as an EOT that silently shortens the transcript (csrc/wmx_decode.hip logits_select_b sets the per-call guard word,
    wmx_runtime.hip transcribe turns it into WMX_ERR_NUMERIC naming the step and row).  Through the drop-in adapter it
    raises WmxError; through EnhancedOnlineASRProcessor.process_iter it takes the reference's recovery path
    (enhanced_asr_processor.py:369-381: log, re-init the buffers at the same offset, return (None, None, "")).  With
    the gain restored the next call succeeds (the guard word is per call)."""
    import io
    from wmx.asr import MI355XWhisperASR
    from wmx._lib import WMX_ERR_NUMERIC, WmxError
    from wmx.online import EnhancedOnlineASRProcessor
    asr = MI355XWhisperASR(lan="auto", modelsize="micro", device="cuda", compute_type="bfloat16",
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=16)
    eng = asr.model.model
    audio = synth.speech_like(5, 16000 * 4)
    assert isinstance(asr.transcribe(audio), list)
    name = "decoder.layers.0.encoder_attn_layer_norm.weight"
    g = eng.get_tensor(name, (eng.dims.n_text_state,))
    bad = g.copy()
    bad[3] = np.nan
    eng.set_tensor(name, bad)
    with pytest.raises(WmxError) as ei:
        asr.transcribe(audio)
    assert ei.value.status == WMX_ERR_NUMERIC and "non-finite" in str(ei.value), str(ei.value)
    print(ei.value)
    log = io.StringIO()
    p = EnhancedOnlineASRProcessor(asr, buffer_trimming=("segment", 15), agreement_n=2, logfile=log)
    p.insert_audio_chunk(audio[:32000])
    assert p.process_iter() == (None, None, "")
    assert len(p.audio_buffer) == 0 and "non-finite" in log.getvalue(), log.getvalue()
    eng.set_tensor(name, g)
    assert isinstance(asr.transcribe(audio), list)


@pytest.mark.parametrize("ct", ["bfloat16", "float8"])
def test_nonfinite_in_a_graph_replayed_decode_step_is_an_error(ct):
    """The decode loop's own guard: a fixed language (lan="en": no language detection to catch
    the NaN first) and a NaN in the decoder's positional embedding row of slot 5 only, so the prompt prefill and the
    first selection (slot 2) are clean and the first non-finite logits come from the third graph-replayed step
    (wmx_runtime.hip transcribe: the per-chunk hipGraph of the step, logits_select_b's guard word).  The call must
    fail with WMX_ERR_NUMERIC naming that decode step, its slot and a row; with the row restored the next call on
    the same (cached) context and graphs succeeds -- for the bf16 model and the float8 model (8-bit decode)."""
    from wmx.asr import MI355XWhisperASR
    from wmx._lib import WMX_ERR_NUMERIC, WmxError
    asr = MI355XWhisperASR(lan="en", modelsize="micro", device="cuda", compute_type=ct,
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=16)
    eng = asr.model.model
    audio = synth.speech_like(15, 16000 * 4)
    ok = asr.transcribe(audio)
    assert isinstance(ok, list)
    name = "decoder.embed_positions.weight"
    shape = (eng.dims.n_text_ctx, eng.dims.n_text_state)
    pos = eng.get_tensor(name, shape)
    bad = pos.copy()
    bad[5, 7] = np.nan
    eng.set_tensor(name, bad)
    with pytest.raises(WmxError) as ei:
        asr.transcribe(audio)
    msg = str(ei.value)
    print(ct, msg)
    assert ei.value.status == WMX_ERR_NUMERIC, msg
    assert "decode step 3 (slot 5)" in msg and "row " in msg and "window 0" in msg, msg
    eng.set_tensor(name, pos)
    again = asr.transcribe(audio)
    assert [s.tokens for s in again] == [s.tokens for s in ok]


def test_streamload_rank_local_path_matches_per_stream_runs(asr):
    """Config 4's rank-local streaming path (wmx.streamload.run_shard: a DynamicVACOnlineASRProcessor per mic stream at
    the reference cadence, one batched transcribe per tick through StreamBatcher) on the GPU at world 1: three streams
    batched give the same committed words as each stream run alone, and every stream commits time-ordered words."""
    from wmx import streamload as SL
    model = asr.model
    model.max_batch = 3
    model._ctx.clear()
    together = SL.run_shard(model, asr, [0, 1, 2], 5.0)
    model.max_batch = 1
    model._ctx.clear()
    alone = [SL.run_shard(model, asr, [s], 5.0) for s in (0, 1, 2)]
    by = lambda recs: sorted((s, k, round(b, 4), round(e, 4), t) for s, k, b, e, t in recs)  # noqa: E731
    assert together["records"], "the streams must commit words"
    assert by(together["records"]) == by([r for a in alone for r in a["records"]])
    assert max(c[0] for c in together["calls"]) >= 2  # due streams shared a batched call
    summ = SL.summarize([together])
    print("rank-local streams:", summ)
    assert summ["p50_ms"] > 0 and 0 < summ["stream_iters"] <= len(together["lat"])
