#!/bin/bash
# Round-4 GPU check of the in-tree library: GPU suite, smoke, the driver's bench command, counter list.
#   bash scripts/archive/r04_check.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > "$O/pytest_gpu_$TAG.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu_$TAG.log"
[ $rc -eq 0 ] || { echo "gpu suite failed ($rc)"; exit $rc; }
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke_$TAG.log"; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --detail "$O/bench_detail_driver_args_$TAG.json" \
  > "$O/bench_driver_args_$TAG.json" 2> "$O/bench_driver_args_$TAG.err" || { echo "bench failed"; tail -5 "$O/bench_driver_args_$TAG.err"; exit 1; }
wc -c "$O/bench_driver_args_$TAG.json"
