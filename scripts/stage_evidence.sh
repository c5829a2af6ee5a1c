#!/bin/bash
# Stage one evidence part's outputs (scripts/gpu_evidence_r06.sh TAG h|a|b, merged back into gpurun_out/) into the
# tracked profiles/RND/: PMC summaries + their rocprofv3 --stats CSVs, VALU summaries, bench lines and the
# driver-command rocprof summary.   bash scripts/stage_evidence.sh TAG [RND (default r06)]
set -eu
TAG=$1
RND=${2:-r06}
mkdir -p profiles/$RND/roofline profiles/$RND/valu profiles/$RND/bench profiles/$RND/cls_large
for f in gpurun_out/pmc_${TAG}_*_summary.json gpurun_out/pmc_${TAG}k[0-9]*_summary.json; do
  [ -e "$f" ] || continue
  b=$(basename "$f" _summary.json)
  cp "$f" profiles/$RND/roofline/
  cp "gpurun_out/${b}_STATS/run_kernel_stats.csv" "profiles/$RND/roofline/${b}_kernel_stats.csv"
done
for f in gpurun_out/valu_${TAG}_*_summary.json gpurun_out/valu_${TAG}k[0-9]*_summary.json; do [ -e "$f" ] && cp "$f" profiles/$RND/valu/; done
for f in gpurun_out/pmc_${TAG}cls_*_summary.json gpurun_out/valu_${TAG}cls_*_summary.json; do
  [ -e "$f" ] || continue
  cp "$f" profiles/$RND/cls_large/
  b=$(basename "$f" _summary.json)
  [ -e "gpurun_out/${b}_STATS/run_kernel_stats.csv" ] && cp "gpurun_out/${b}_STATS/run_kernel_stats.csv" "profiles/$RND/cls_large/${b}_kernel_stats.csv"
done
O=gpurun_out/$TAG
if [ -e "$O/bench_driver.out" ]; then
  tail -n 1 "$O/bench_driver.out" > "profiles/$RND/bench/bench_driver_${TAG}.jsonl"
  cp "$O/bench_detail_driver.json" "profiles/$RND/bench/bench_detail_driver_${TAG}.json"
  cp "$O/prof/run_kernel_stats.csv" "profiles/$RND/bench/rocprof_driver_cmd_${TAG}_kernel_stats.csv"
fi
if [ -e "$O/bench_default.out" ]; then
  tail -n 1 "$O/bench_default.out" > "profiles/$RND/bench/bench_default_${TAG}.jsonl"
  cp "$O/bench_detail_default.json" "profiles/$RND/bench/bench_detail_default_${TAG}.json"
fi
ls profiles/$RND/roofline/*${TAG}* profiles/$RND/valu/*${TAG}* profiles/$RND/bench/*${TAG}* 2>/dev/null | wc -l
