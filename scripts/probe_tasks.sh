# Per-launch GPU time (spin-held) and host issue rate of the single-step kernel at 4096 envs, per task.
set -u
for t in ${TASKS:-LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed}; do
  timeout -k 10 120 python scripts/launch_probe.py $t 2>&1 | grep -E "^(A|C|H)" | sed "s/^/$t /" || exit 1
done
