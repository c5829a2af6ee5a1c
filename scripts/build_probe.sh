#!/bin/bash
# Probe build of the library with per-wave s_memtime stamps (scripts/stamp_probe.py, scripts/stamp_rollout.py),
# same flags as the product build plus -DOUZ_STAMPS; loaded through OUZ_LIB, never the product default.
set -eu
cd "$(dirname "$0")/.."
OUZ_EXTRA_FLAGS="-DOUZ_STAMPS ${OUZ_EXTRA_FLAGS:-}" OUZ_BUILD_OUT=$PWD/ouzelum_amd/libouzelum_probe.so \
  python -c "from ouzelum_amd import build; build.build(force=True, verbose=False)"
