"""Silero VAD on device: wall time per wmx_vad_process call (bench.py's "vad" leg) for one VAC tick of 8 streams and
a 16-window backlog of 64 streams.  Usage: python tools/vad_bench.py  (under rocprofv3 for per-kernel times)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "realtime-whisper-asr_amd")]

import bench  # noqa: E402

print(json.dumps(bench.vad_bench(8)))
