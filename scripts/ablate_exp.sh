# Ablation probe: per-step GPU time of the LeeLanded step with parts of env_core compiled out
# (OUZ_PROBE_SKIP bits: 1 controller, 2 integrator, 4 reward).  Not a parity build.
set -u
for v in 0 1 2 4 7; do
  OUZ_EXTRA_FLAGS="-DOUZ_PROBE_SKIP=$v" python -m ouzelum_amd.build --force > /dev/null 2>&1 || exit 1
  timeout -k 10 120 python scripts/launch_probe.py ${TASK:-LeeLanded} 2>&1 | grep -E "^(A|C|H)" | sed "s/^/skip$v /" || exit 1
done
python -m ouzelum_amd.build --force > /dev/null 2>&1
