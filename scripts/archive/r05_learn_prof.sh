#!/bin/bash
# The learner update under rocprofv3 --kernel-trace --stats (config D: QuadFault 8192 envs, RPO-LSTM; VERDICT r04
# item 5).  Keeps the --stats summaries, drops the (large) per-dispatch trace.   bash scripts/archive/r05_learn_prof.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
O="$R/gpurun_out/learn_$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 --warmup 3 \
  > "$O/bench_plain.json" 2> "$O/bench_plain.err" || { echo "learner bench failed"; tail -5 "$O/bench_plain.err"; exit 1; }
cat "$O/bench_plain.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o learn -- \
  python3 scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 8 --warmup 2 > "$O/learn.out" 2> "$O/learn.err" \
  || { echo "learner profile failed"; tail -5 "$O/learn.err"; exit 1; }
tail -1 "$O/learn.out"
for f in $(find "$O/prof" -name "*_stats.csv"); do cp "$f" "$O/"; done
rm -rf "$O/prof"
ls -la "$O"
head -25 "$O"/*kernel_stats.csv
