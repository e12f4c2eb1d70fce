#!/bin/bash
# round 3, GPU call 1: smoke, the whole -m gpu suite on the product library, the guarded-load diagnostic variant on the
# micro decode tests (once), a default bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?
tail -30 $O/gputest.log
if [ $rc -ne 0 ] && grep -q "Fatal\|core dumped\|HSA_STATUS_ERROR\|Memory access fault" $O/gputest.log; then echo "GPU fault: stopping"; exit 1; fi
WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_guarded.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_step.py -k "micro" tests/test_gpu_parity.py > $O/guarded_variant.log 2>&1
grc=$?
echo "guarded variant rc $grc; OOB reports: $(grep -c 'WMX_PACKED_GUARDED OOB' $O/guarded_variant.log)"
tail -5 $O/guarded_variant.log
if [ $grc -ne 0 ] && grep -q "Fatal\|core dumped\|HSA_STATUS_ERROR\|Memory access fault" $O/guarded_variant.log; then echo "GPU fault in variant: stopping"; exit 1; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc $?"; cat $O/bench.json | head -c 600; echo
exit $rc
