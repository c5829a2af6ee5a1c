#!/bin/bash
# RPO-LSTM training runs on the HIP env for a fixed env-step budget (the reference's total_steps default is
# 30M, RPO-LSTM/main.py:22): the learners' default env (Landing), config D's consumer (QuadFault, 8192 envs)
# and Ouzelum hover.  Writes the per-iteration CSVs (PPO/main.py:102-116 scalars) under gpurun_out/$TAG/,
# then the learner throughput on config D.  Each run has its own time limit; stops at the first failure.
set -u
TAG=${TAG:-learn}
OUT=gpurun_out/$TAG
STEPS=${STEPS:-30000000}
mkdir -p $OUT
for spec in ${RUNS:-Landing:4096 QuadFault:8192 Ouzelum:4096}; do
  env=${spec%%:*}; n=${spec##*:}
  timeout -k 10 ${RUN_TIMEOUT:-240} python -u -m ouzelum_amd.learners.train --env $env --num_envs $n \
    --total_steps $STEPS --seed 0 --logdir $OUT/${env}_$n --no_checkpoints --quiet > $OUT/${env}_$n.log 2>&1
  rc=$?; echo "$env $n rc=$rc"; tail -n 3 $OUT/${env}_$n.log
  [ $rc -eq 0 ] || exit $rc
  f=$(ls $OUT/${env}_$n/*.csv); python - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
k = max(1, len(rows) // 8)
for r in rows[::k] + [rows[-1]]:
    print(f"  {int(r['global_step']):>10d}  avg_rew {float(r['average_reward']):9.4f}  ep_ret {float(r['episodic_return']):10.3f}"
          f"  ep_len {float(r['episodic_length']):7.1f}  {float(r['env_steps_per_s'])/1e6:6.2f} M/s")
EOF
done
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 200 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 20 > $OUT/bench_learner_QuadFault_8192.json 2>&1
rc=$?; echo "bench_learner rc=$rc"; tail -c 800 $OUT/bench_learner_QuadFault_8192.json
exit $rc
