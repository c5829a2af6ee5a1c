#!/bin/bash
# One GPU-box pass: the GPU tests (or a -k selection), then bench.py with the driver's arguments.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-1} -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} \
  > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.json; tail -n 5 gpurun_out/bench_$TAG.err
exit $rc
