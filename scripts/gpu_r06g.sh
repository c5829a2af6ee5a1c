# round-6 learner evidence on the final library: learning curves (30 M env-steps each), config D throughput and its
# rocprofv3 kernel statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06learn bash scripts/learn_curves.sh > gpurun_out/learn_curves_r06.log 2>&1 || { tail -20 gpurun_out/learn_curves_r06.log; exit 1; }
tail -40 gpurun_out/learn_curves_r06.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r06learn/prof -o run -- \
  python3 -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 > gpurun_out/r06learn/prof.log 2>&1 || exit 1
tail -1 gpurun_out/r06learn/prof.log
