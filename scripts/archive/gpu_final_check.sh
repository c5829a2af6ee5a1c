#!/bin/bash
# One GPU-box pass over a library build: the GPU suite, smoke(), the roofline evidence of every bench entry
# (headline sizes, the large-N sweep, the streamed rollouts), the bench with the driver's arguments and with no
# flags, and rocprofv3 --stats of the driver-argument command.  Every GPU step has its own time limit; the
# script stops at the first failure.
#   bash scripts/archive/gpu_final_check.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1; shift; local lim=$1; shift
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 "$OUT/$name.out" "$OUT/$name.err"; exit $rc; }; }
step pytest 500 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider
tail -n 2 "$OUT/pytest.out"
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
bash scripts/gpu_roofline_evidence.sh "$TAG" \
  rollout:LeeLanded:4096 step:LeeLanded:4096 rollout:QuadTracking:4096 step:QuadTracking:4096 \
  rollout:QuadFault:8192 step:QuadFault:8192 rollout:QuadMixed:4096 step:QuadMixed:4096 > "$OUT/evidence_headline.log" 2>&1 \
  || { tail -n 20 "$OUT/evidence_headline.log"; exit 1; }
echo "evidence headline ok"
bash scripts/gpu_roofline_evidence.sh "$TAG" > "$OUT/evidence_large.log" 2>&1 || { tail -n 20 "$OUT/evidence_large.log"; exit 1; }
echo "evidence large-N ok"
# the bench prices traffic from profiles/: stage this run's summaries there for the bench lines below
mkdir -p profiles/r03/roofline
for f in gpurun_out/pmc_${TAG}_*_summary.json; do
  b=$(basename "$f" _summary.json)
  cp "$f" profiles/r03/roofline/ && cp "gpurun_out/${b}_STATS/run_kernel_stats.csv" "profiles/r03/roofline/${b}_kernel_stats.csv"
done
step bench_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python -u bench.py
export TMPDIR=/tmp
step prof_driver 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/$OUT/prof" -o run -- \
  python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs
tail -c 400 "$OUT/bench_driver.out"; echo
tail -c 400 "$OUT/bench_default.out"; echo
