"""bench.py refuses to print a line under a timing-only or removed WMX_* switch, and records the WMX_* environment of
a line it does print.  CPU only: the check runs before anything touches torch or the GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(env_extra, *args):
    env = {k: v for k, v in os.environ.items() if not k.startswith("WMX_")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=120)


def test_bench_refuses_under_the_ablation_switch():
    r = _bench({"WMX_ABLATE": "1"}, "--dry-run")
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr[-2000:])
    assert r.stdout.strip() == ""  # no JSON line
    assert "WMX_ABLATE" in r.stderr


def test_bench_refuses_under_removed_experiment_switches():
    for var in ("WMX_PHASE_PROBE", "WMX_MLP_FUSED", "WMX_REDLN_FUSED", "WMX_FOLD", "WMX_XATTN_PAIRS"):
        r = _bench({var: "1"}, "--dry-run")
        assert r.returncode == 2 and r.stdout.strip() == "", (var, r.returncode, r.stdout)


def test_check_env_records_documented_knobs(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    for k in list(os.environ):
        if k.startswith("WMX_"):
            monkeypatch.delenv(k)
    monkeypatch.setenv("WMX_LOCKSTEP", "1")
    monkeypatch.setenv("WMX_DEC_MIXED", "0")
    assert bench.check_env() == {"WMX_DEC_MIXED": "0", "WMX_LOCKSTEP": "1"}
    json.dumps(bench.BENCH_ENV_KNOBS)  # (the documented list is plain data)
