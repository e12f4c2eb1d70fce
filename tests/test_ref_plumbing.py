"""The drop-in adapter and the streaming caller against traces of the REFERENCE's own code
(tests/golden/ref_plumbing.json, made by tests/golden/make_ref_plumbing.py from /root/reference's
asr_components.py and enhanced_asr_processor.py with the stubs of tests/ref_stubs.py).

Pinned here:
  * a1  CustomFasterWhisperASR -> the keyword arguments faster-whisper's WhisperModel(...) and .transcribe(...)
        receive, for auto / fixed language, translate, use_vad, adaptive kwargs, defaults (asr_components.py:195-309);
  * a10 ts_words / segments_end_ts / sep (asr_components.py:291-301);
  * a12 DynamicVADIterator event merging with silence changes, DynamicVACOnlineASRProcessor gating
        (asr_components.py:12-179);
  * a11 EnhancedOnlineASRProcessor LocalAgreement-2/3/4, the 300-char prompt, dynamic trimming, reset-on-error,
        and the EnhancedVACOnlineASRProcessor stack (enhanced_asr_processor.py:32-502).
Exact equality throughout (the traces are integers, strings and floats from identical arithmetic).
"""
import json
import os

import numpy as np
import pytest

import ref_stubs as S
from wmx import asr as A
from wmx import online as OL

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_plumbing.json")))


def jr(x):
    """Normalise tuples / numpy scalars exactly as the fixture's JSON encoding did."""
    return json.loads(json.dumps(x, ensure_ascii=False, default=float))


class Adaptive:
    def __init__(self, kw):
        self.kw = kw

    def get_transcribe_kwargs(self):
        return dict(self.kw)


# keys of the WhisperModel(...) call the reference makes (asr_components.py:244-262); the adapter adds its own
# engine keys (seed, beam_size, max_new_tokens), which faster-whisper does not have
FW_CTOR_KEYS = ("device", "compute_type", "download_root", "num_workers", "device_index")


@pytest.mark.parametrize("case", FX["asr"], ids=[c["name"] for c in FX["asr"]])
def test_asr_adapter_kwargs_match_reference(case, monkeypatch):
    monkeypatch.setattr(A, "WhisperModel", S.RecordingWhisperModel)
    S.CALLS.clear()
    ctor = dict(case["ctor"])
    if case["adaptive"] is not None:
        ctor["adaptive_params"] = Adaptive(case["adaptive"])
    audio = S.audio_stream(11, 3 * 16000)
    if case.get("error"):
        with pytest.raises(ValueError):
            A.MI355XWhisperASR(**ctor)
        return
    if ctor.get("device") == "cpu":
        # documented divergence: the MI355X adapter has no CPU/int8 engine and says so
        with pytest.raises(ValueError, match="GPU"):
            A.MI355XWhisperASR(**ctor)
        return
    asr = A.MI355XWhisperASR(**ctor)
    assert asr.sep == case["sep"]
    assert asr.original_language == case["original_language"]
    results = []
    for op in case["ops"]:
        if op[0] == "transcribe":
            segs = asr.transcribe(audio, init_prompt=op[1])
            results.append({"ts_words": [list(t) for t in asr.ts_words(segs)],
                            "segments_end_ts": asr.segments_end_ts(segs)})
        else:
            getattr(asr, op[0])()
    assert jr(results) == case["results"]
    assert jr(asr.transcribe_kargs) == case["transcribe_kargs"]
    got = jr(S.CALLS)
    ref = case["calls"]
    assert len(got) == len(ref)
    # constructor: the reference's faster-whisper kwargs, exactly
    assert got[0][0] == ref[0][0] == "WhisperModel" and got[0][1] == ref[0][1]
    assert {k: got[0][2].get(k) for k in ref[0][2]} == ref[0][2]
    assert set(got[0][2]) >= set(ref[0][2]) and "device_index" in ref[0][2]
    for g, r in zip(got[1:], ref[1:]):
        assert g == r  # transcribe: audio signature + every keyword argument identical


@pytest.mark.parametrize("case", FX["vad"], ids=lambda c: f"return_seconds={c['return_seconds']}")
def test_dynamic_vad_iterator_matches_reference(case):
    it = OL.DynamicVADIterator(S.ScriptedSilero(S.vad_track(3)), initial_silence_ms=500, min_silence_ms=200,
                               max_silence_ms=1000, threshold=0.5)
    audio = S.audio_stream(5)
    sets = {40: 260, 200: 5000, 201: 980, 230: 300}
    ev, pos = [], 0
    for k, n in enumerate(S.chunk_sizes(4)):
        if k in sets:
            ev.append(["set", sets[k], it.set_silence_duration(sets[k])])
        ev.append([k, it(audio[pos:pos + n], return_seconds=case["return_seconds"])])
        pos += n
    assert jr(ev) == case["events"]
    assert sum(1 for e in ev if isinstance(e[1], dict)) >= 7  # the track exercises starts and ends


@pytest.mark.parametrize("case", FX["vac"], ids=lambda c: f"chunk={c['online_chunk_size']}")
def test_dynamic_vac_gate_matches_reference(case):
    S.CALLS.clear()
    vac = OL.DynamicVACOnlineASRProcessor(case["online_chunk_size"], asr=None, initial_silence_ms=500,
                                          min_silence_ms=200, max_silence_ms=1000, vad_threshold=0.5,
                                          vad_model=S.ScriptedSilero(S.vad_track(7)), online=S.RecordingOnline())
    audio = S.audio_stream(8)
    rets, pos = [], 0
    for k, n in enumerate(S.chunk_sizes(9)):
        vac.insert_audio_chunk(audio[pos:pos + n])
        pos += n
        if k == 60:
            vac.set_silence_duration(300)
        rets.append(list(vac.process_iter()))
    assert jr(rets) == case["returns"]
    assert jr(S.CALLS) == case["calls"]
    assert sum(1 for r in rets if r[2]) >= 5


@pytest.mark.parametrize("case", FX["enhanced"],
                         ids=lambda c: f"n{c['agreement_n']}-jit{int(c['jitter'])}-fail{len(c['fail_on'])}")
def test_enhanced_online_processor_matches_reference(case):
    asr = S.FakeASR(jitter=case["jitter"], fail_on=case["fail_on"])
    p = OL.EnhancedOnlineASRProcessor(asr, buffer_trimming=("segment", case["trim"]),
                                      agreement_n=case["agreement_n"], logfile=open(os.devnull, "w"))
    audio = S.audio_stream(12, 40 * 16000)
    rets, prompts = [], []
    for i in range(0, len(audio), 8000):
        p.insert_audio_chunk(audio[i:i + 8000])
        if (i // 8000) % 2 == 1:
            prompts.append(list(p.prompt()))
            rets.append(list(p.process_iter()))
            if i // 8000 == 41:
                p.set_agreement_n(case["agreement_n"] + 1)
    rets.append(list(p.finish()))
    assert jr(prompts) == case["prompts"]
    assert jr(rets) == case["returns"]
    assert jr(asr.calls) == case["asr_calls"]
    assert p.buffer_trimming_sec == case["trimming_sec"]
    assert round(p.buffer_time_offset, 6) == case["final_offset"]


@pytest.mark.parametrize("case", FX["enhanced_vac"], ids=lambda c: f"n{c['agreement_n']}")
def test_enhanced_vac_stack_matches_reference(case):
    asr = S.FakeASR(jitter=True)
    v = OL.EnhancedVACOnlineASRProcessor(0.5, asr, logfile=open(os.devnull, "w"), agreement_n=case["agreement_n"],
                                         vad_model=S.ScriptedSilero(S.vad_track(13, 1200)))
    audio = S.audio_stream(14, 1200 * 512)
    rets, pos = [], 0
    for n in S.chunk_sizes(15, 1200 * 512):
        v.insert_audio_chunk(audio[pos:pos + n])
        pos += n
        rets.append(list(v.process_iter()))
    assert jr(rets) == case["returns"]
    assert jr(asr.calls) == case["asr_calls"]
    assert sum(1 for r in rets if r[2]) >= 10


def test_fixture_is_data_only():
    """The fixture holds traces (numbers and strings), never reference source text."""
    raw = open(os.path.join(os.path.dirname(__file__), "golden", "ref_plumbing.json"), encoding="utf-8").read()
    for needle in ("def ", "class ", "import ", "self."):
        assert needle not in raw
    assert np.isfinite(len(raw))
