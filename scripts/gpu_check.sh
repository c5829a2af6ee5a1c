#!/bin/bash
# One GPU-box session: gpu tests -> bench -> rocprofv3 kernel stats.
# Stops at the first step that ends in a fault/abort/timeout (rc >= 124 or 134/139).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r01}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] ; }

timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu_$TAG.log
ok $rc || exit $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0

timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -n 5 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_PROF:-0}" = 1 ] && exit 0

export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 1000 --warmup 50 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/prof_bench_$TAG.json" 2> "$R/gpurun_out/prof_bench_$TAG.err"
rc=$?; echo "rocprof rc=$rc"
find "$R/gpurun_out/prof_$TAG" -name "*stats*" | head
exit $rc
