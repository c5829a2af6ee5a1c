set -u
for v in base nocore; do
  if [ $v = nocore ]; then OUZ_EXTRA_FLAGS=-DOUZ_PROBE_NOCORE python -m ouzelum_amd.build --force > /dev/null 2>&1 || exit 1; fi
  for t in LeeLanded EKFLeeLanded; do
    timeout -k 10 120 python scripts/launch_probe.py $t 2>&1 | grep -E "^(A|H|I)" | sed "s/^/$v $t /"
  done
done
