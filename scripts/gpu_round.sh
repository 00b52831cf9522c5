#!/bin/bash
# One GPU call: the -m gpu suite (failures reported, not fatal), then the default bench.
# Stops at the first fault / abort / timeout (exit codes other than 0 or 1 from pytest).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -v -rf --timeout 300 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
tail -c 3000 gpurun_out/bench.json
echo "pytest rc=$rc bench rc=$brc"
exit $brc
