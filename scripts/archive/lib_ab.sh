#!/bin/bash
# A/B of two in-tree library builds on the large-N step kernel: scripts/exp/pipe_ab.py under the product
# library and under OUZ_LIB=$1, alternating twice.  Usage: bash scripts/archive/lib_ab.sh <variant.so> TASKS SIZES TILES
set -eu
cd "$(dirname "$0")/../.."
V=$1; T=$2; S=$3; P=${4:-1}
for r in 1 2; do
  echo "# product build (round $r)"
  timeout -k 10 300 python -u scripts/exp/pipe_ab.py "$T" "$S" "$P"
  echo "# $V (round $r)"
  OUZ_LIB=$PWD/$V timeout -k 10 300 python -u scripts/exp/pipe_ab.py "$T" "$S" "$P"
done
