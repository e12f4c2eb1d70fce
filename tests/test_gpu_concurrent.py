"""Correctness of the configuration bench.py times: context groups decoding CONCURRENTLY on one shared model.

bench.py splits its 8 windows over 2 decoding contexts (each its own HIP stream and captured decode graph, both on
one read-only wmx_model) and runs them from two host threads at once (bench.py step(); ctypes drops the GIL inside
libwmx).  Here the same shape runs at large-v3 width (d 1280, 20 heads, vocab 51866, 2 decoder layers): 2 contexts x
4 windows x beam 5, language auto-detect, word timestamps on, the hipGraph decode and the in-situ probes on, started
from two threads together, several times:
  * every result (tokens, sum_logprob, no_speech_prob, language, jump_times, token probabilities) must equal, bit for
    bit, the result of the same context run alone (the kernels are deterministic: fixed-order reductions);
  * with the search recorder on (both contexts, concurrently), oracle.search_replay must choose exactly the device's
    selection at every step of both groups, and oracle.rank_final its final sequence.
"""
import threading

import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

WIDE2 = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)
EPS_TIE = 1e-3


def _edims(d):
    from wmx import engine as E
    return E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                       d.n_text_head, d.n_text_layer)


def _run_concurrently(ctxs, batches):
    out, err = [None] * len(ctxs), []
    go = threading.Barrier(len(ctxs))

    def work(i):
        try:
            go.wait()
            out[i] = ctxs[i].transcribe(batches[i])
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(ctxs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return out


def _same(a, b, tag):
    assert a.tokens == b.tokens, (tag, a.tokens, b.tokens)
    assert a.sum_logprob == b.sum_logprob and a.no_speech_prob == b.no_speech_prob, tag
    assert a.language == b.language and a.language_prob == b.language_prob, tag
    np.testing.assert_array_equal(a.jump_times, b.jump_times, err_msg=tag)
    np.testing.assert_array_equal(a.text_token_probs, b.text_token_probs, err_msg=tag)


@pytest.mark.parametrize("ct", ["bfloat16", "float8", "int8_float16", "int8_bfloat16"])
def test_two_groups_concurrent_equal_sequential_and_replay(ct):
    """bfloat16 (the default bench line), float8 (config 5's line: MX-fp8 encoder, 8-bit decoder weights and fp8
    cross-K/V images) and the reference's CTranslate2 int8 modes (int8 decoder / logits weights with CT2 row scales,
    the separate cross-q launch, 16-bit cross-K/V images; f16 and bf16 activations: ADVICE r05)."""
    from wmx import engine as E
    m = E.Model(_edims(WIDE2), 0, ct).init_synthetic(5)
    sp = O.special_tokens(WIDE2.n_vocab)
    K, n_new = 5, 40
    ctxs = [E.Context(m, max_batch=4, beam_size=K, max_new_tokens=n_new, language=None, word_timestamps=True,
                      use_graph=True) for _ in range(2)]
    for c in ctxs:
        c.set_probe(True, 1)  # as bench.py: probes captured into the step graphs
    audios = [synth.speech_like(900 + i, 480000) for i in range(8)]
    batches = [audios[:4], audios[4:]]
    alone = [ctxs[g].transcribe(batches[g]) for g in range(2)]
    for r in alone[0] + alone[1]:
        assert len(r.tokens) == n_new and r.jump_times is not None
    for rep in range(3):
        both = _run_concurrently(ctxs, batches)
        for g in range(2):
            for b in range(4):
                _same(both[g][b], alone[g][b], f"rep {rep} group {g} window {b}")
    # search replay of both groups' recorded steps, the groups again running concurrently
    for c in ctxs:
        c.record(n_new)
    both = _run_concurrently(ctxs, batches)
    opt_langs = []
    for g in range(2):
        res = both[g]
        for b in range(4):
            _same(res[b], alone[g][b], f"recorded group {g} window {b}")
        lg, sel = ctxs[g].recorded()
        assert lg.shape[:2] == (n_new, 4 * K)
        langs = {r.language for r in res}
        opt_langs.append(sorted(langs))
        # the replay needs one language per window: windows share the options unless their detected language
        # differs, in which case each window is replayed with its own
        for b in range(4):
            opt = O.DecodeOptions(language=res[b].language, beam_size=K, max_new_tokens=n_new)
            rows = slice(b * K, (b + 1) * K)
            info = O.search_replay(lg[:, rows], sel[:, rows] - np.array([b * K, 0], np.int32) * (sel[:, rows] >= 0),
                                   K, sp, opt, eps=EPS_TIE)[0]
            assert info["mismatch"] is None, (g, b, info["mismatch"])
            if not info["ties"]:
                assert info["steps"] >= 16, (g, b, info["steps"])
                toks, sc, margin = O.rank_final(info["finished"], info["alive"], K)
                if margin > EPS_TIE:
                    assert res[b].tokens == toks, (g, b)
                    assert abs(res[b].sum_logprob - sc) <= 1e-3 * max(1.0, abs(sc)), (g, b, res[b].sum_logprob, sc)
            print(f"group {g} window {b}: replayed {info['steps']} steps, tie {info['ties']}")
    print("detected languages per group", opt_langs)
    for c in ctxs:
        c.record(0)


def test_lockstep_groups_equal_alone_and_a_lone_member_proceeds():
    """wmx_ctx_set_lockstep (bench.py's default for its two groups): the groups' decode loops meet at a host barrier.
    Results stay bit-identical to each context run alone, and a member transcribing without its partner proceeds
    after the barrier's timeout instead of hanging."""
    import time

    from wmx import engine as E
    m = E.Model(_edims(WIDE2), 0, "bfloat16").init_synthetic(6)
    n_new = 24
    ctxs = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=n_new, language=None, word_timestamps=True,
                      use_graph=True) for _ in range(2)]
    audios = [synth.speech_like(950 + i, 480000) for i in range(4)]
    batches = [audios[:2], audios[2:]]
    alone = [ctxs[g].transcribe(batches[g]) for g in range(2)]
    for c in ctxs:
        c.set_lockstep(11, 2)
    for rep in range(2):
        both = _run_concurrently(ctxs, batches)
        for g in range(2):
            for b in range(2):
                _same(both[g][b], alone[g][b], f"lockstep rep {rep} group {g} window {b}")
    t = time.perf_counter()
    lone = ctxs[0].transcribe(batches[0])  # partner absent: one 5 ms barrier timeout, then the decode
    dt = time.perf_counter() - t
    for b in range(2):
        _same(lone[b], alone[0][b], f"lone member window {b}")
    both = _run_concurrently(ctxs, batches)  # the group recovers on the next concurrent call
    for g in range(2):
        for b in range(2):
            _same(both[g][b], alone[g][b], f"after the lone call, group {g} window {b}")
    for c in ctxs:
        c.set_lockstep(0, 0)
    print(f"lone member call {1e3 * dt:.1f} ms")


def test_lockstep_member_with_a_shorter_decode_leaves_the_chunk_barrier():
    """two lockstep contexts whose decode loops have different lengths (8 and 40 steps, word timestamps
    on, so the short member goes on to the alignment forward and the host DTW while the long one still decodes).  The
    short member leaves the chunk barrier when its decode loop ends, so the long member meets no chunk-barrier
    timeout (wmx_ctx_lockstep_timeouts), and both results equal each context run alone."""
    from wmx import engine as E
    m = E.Model(_edims(WIDE2), 0, "bfloat16").init_synthetic(8)
    ctxs = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=n, language=None, word_timestamps=True,
                      use_graph=True) for n in (8, 40)]
    audios = [synth.speech_like(970 + i, 480000) for i in range(4)]
    batches = [audios[:2], audios[2:]]
    alone = [ctxs[g].transcribe(batches[g]) for g in range(2)]
    for c in ctxs:
        c.set_lockstep(12, 2)
    before = [c.lockstep_timeouts for c in ctxs]
    for rep in range(2):
        both = _run_concurrently(ctxs, batches)
        for g in range(2):
            for b in range(2):
                _same(both[g][b], alone[g][b], f"uneven lockstep rep {rep} group {g} window {b}")
    after = [c.lockstep_timeouts for c in ctxs]
    for c in ctxs:
        c.set_lockstep(0, 0)
    print("chunk-barrier timeouts before / after", before, after, "steps", [c.last_steps() for c in ctxs])
    assert after == before, (before, after)
