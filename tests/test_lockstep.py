"""The lockstep barriers of concurrently decoding context groups (wmx_ctx_set_lockstep; bench.py starts its two groups'
decode loops together through them and re-aligns them before every 8-step chunk, DESIGN.md §7 "The slow decode
mode"), exercised alone through the host-only entry point wmx_debug_lockstep_arrive: no GPU needed.

  * n members arriving from n threads all pass, without waiting out the timeout;
  * a lone member waits the timeout, reports it, and leaves the group clean: the next full round passes at once;
  * the chunk barrier waits only for the members still decoding: a member that leaves releases the others;
  * a key keeps its member count."""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))

from wmx import _lib  # noqa: E402

lib = _lib.lib


def _arrive(key, n, timeout_us, op=0):
    ok = C.c_int(-1)
    st = lib.wmx_debug_lockstep_arrive(key, n, op, timeout_us, C.byref(ok))
    assert st == 0, lib.wmx_last_error()
    return ok.value


def _round(key, n, timeout_us, stagger_s=0.0, op=0):
    out = [None] * n

    def work(i):
        time.sleep(i * stagger_s)
        out[i] = _arrive(key, n, timeout_us, op)

    th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out, time.perf_counter() - t0


def test_full_group_passes_without_the_timeout():
    for n in (2, 4):
        out, dt = _round(9100 + n, n, 2_000_000, stagger_s=0.01)  # 2 s timeout, members 10 ms apart
        assert out == [1] * n
        assert dt < 1.0, dt  # released when the last member arrived, not at the timeout


def test_lone_member_times_out_and_the_group_recovers():
    key = 9200
    t0 = time.perf_counter()
    assert _arrive(key, 2, 50_000) == 0  # alone: the 50 ms timeout
    assert time.perf_counter() - t0 >= 0.045
    for _ in range(3):  # the next rounds start clean (the lone member left the count)
        out, dt = _round(key, 2, 2_000_000)
        assert out == [1, 1] and dt < 1.0


def test_member_count_is_fixed_per_key():
    key = 9300
    out, _ = _round(key, 2, 2_000_000)
    assert out == [1, 1]
    ok = C.c_int(-1)
    assert lib.wmx_debug_lockstep_arrive(key, 3, 0, 1000, C.byref(ok)) != 0
    assert b"member count" in lib.wmx_last_error()


def test_chunk_barrier_waits_only_for_members_still_decoding():
    key, n = 9400, 2
    out, _ = _round(key, n, 2_000_000)  # the start barrier: both in this call's decode loop
    assert out == [1, 1]
    res = {}

    def b_chunks():  # member B: two more chunks
        res["b"] = [_arrive(key, n, 2_000_000, op=1) for _ in range(2)]

    t = threading.Thread(target=b_chunks)
    t0 = time.perf_counter()
    t.start()
    assert _arrive(key, n, 2_000_000, op=1) == 1  # A's next chunk meets B's first
    time.sleep(0.05)
    assert _arrive(key, n, 0, op=2) == 1  # A's decode loop ends: B's second chunk is released
    t.join()
    assert res["b"] == [1, 1] and time.perf_counter() - t0 < 1.0
    _arrive(key, n, 0, op=2)  # B leaves too
    out, dt = _round(key, n, 2_000_000)  # the next call's start barrier: a full group again
    assert out == [1, 1] and dt < 1.0
    out, dt = _round(key, n, 2_000_000, stagger_s=0.01, op=1)  # and its chunk barrier waits for both
    assert out == [1, 1] and dt < 1.0
