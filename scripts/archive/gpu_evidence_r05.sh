#!/bin/bash
# Round-5 evidence of ONE library build, in gpurun calls each under the 20-minute limit:
#   bash scripts/archive/gpu_evidence_r05.sh TAG h   the headline alone (when boxes are scarce): roofline + VALU evidence of
#                                            config B's two kernels, staged, then smoke(), the driver-argument bench
#                                            line and rocprofv3 --stats of the driver's command
#   bash scripts/archive/gpu_evidence_r05.sh TAG t   GPU suite and smoke()
#   bash scripts/archive/gpu_evidence_r05.sh TAG a   (after h) roofline evidence (rocprofv3 --stats + FETCH_SIZE /
#                                            WRITE_SIZE passes) of the headline-size entries, VALU / issue passes
#                                            of every entry that is not HBM-bound
#   bash scripts/archive/gpu_evidence_r05.sh TAG b   roofline evidence of the large-N sweep, then the bench lines (driver
#                                            arguments, no flags) and rocprofv3 --stats of the driver's command
# Summaries land in gpurun_out/ (copied into profiles/r05/ by hand between the calls; part b stages its own into
# profiles/r05/roofline on the box so that its bench lines price traffic from them).  Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; PART=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1; shift; local lim=$1; shift
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 "$OUT/$name.out" "$OUT/$name.err"; exit $rc; }; }
stage() {   # summaries of this build into profiles/r05 on the box, so that its bench lines price from them
  mkdir -p profiles/r05/roofline profiles/r05/valu
  for f in gpurun_out/pmc_${TAG}_*_summary.json; do
    [ -e "$f" ] || continue
    b=$(basename "$f" _summary.json)
    cp "$f" profiles/r05/roofline/ && cp "gpurun_out/${b}_STATS/run_kernel_stats.csv" "profiles/r05/roofline/${b}_kernel_stats.csv"
  done
  for f in gpurun_out/valu_${TAG}_*_summary.json; do [ -e "$f" ] && cp "$f" profiles/r05/valu/; done
  return 0; }
driver_bench() {
  step bench_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --detail "$OUT/bench_detail_driver.json"
  export TMPDIR=/tmp
  step prof_driver 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/$OUT/prof" -o run -- \
    python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs --detail "$OUT/bench_detail_prof.json"
  tail -c 300 "$OUT/bench_driver.out"; echo; }
if [ "$PART" = h ]; then
  bash scripts/gpu_roofline_evidence.sh "$TAG" rollout:LeeLanded:4096 step:LeeLanded:4096 > "$OUT/evidence_h.log" 2>&1 \
    || { tail -n 20 "$OUT/evidence_h.log"; exit 1; }
  bash scripts/gpu_valu.sh "$TAG" rollout:LeeLanded:4096 step:LeeLanded:4096 > "$OUT/valu_h.log" 2>&1 \
    || { tail -n 20 "$OUT/valu_h.log"; exit 1; }
  echo "headline evidence ok"
  stage
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
  driver_bench
elif [ "$PART" = t ]; then
  step pytest 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider
  tail -n 2 "$OUT/pytest.out"
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
elif [ "$PART" = a ]; then
  bash scripts/gpu_roofline_evidence.sh "$TAG" \
    rollout:QuadTracking:4096 step:QuadTracking:4096 rollout:QuadFault:8192 step:QuadFault:8192 rollout:QuadMixed:4096 step:QuadMixed:4096 > "$OUT/evidence_headline.log" 2>&1 \
    || { tail -n 20 "$OUT/evidence_headline.log"; exit 1; }
  echo "evidence headline ok"
  bash scripts/gpu_valu.sh "$TAG" rollout:QuadTracking:4096 step:QuadTracking:4096 rollout:QuadFault:8192 step:QuadFault:8192 rollout:QuadMixed:4096 step:QuadMixed:4096 \
    rollout:QuadTracking:4194304 rollout:QuadMixed:4194304 rollout:QuadTracking:16777216 rollout:QuadMixed:16777216 \
    > "$OUT/valu.log" 2>&1 || { tail -n 20 "$OUT/valu.log"; exit 1; }
  echo "valu ok"
  # the opt-in trigger-class layout above the latency regime (OUZ_CLS_LARGE=1): its VALU / issue view beside the
  # identity layout's, tagged apart (TAGcls, staged by hand into profiles/r05/cls_large, never
  # into roofline/) so the bench never prices from it
  OUZ_CLS_LARGE=1 bash scripts/gpu_valu.sh "${TAG}cls" rollout:QuadTracking:4194304 rollout:QuadMixed:4194304 \
    > "$OUT/valu_cls.log" 2>&1 || { tail -n 20 "$OUT/valu_cls.log"; exit 1; }
  OUZ_CLS_LARGE=1 bash scripts/gpu_roofline_evidence.sh "${TAG}cls" rollout:QuadTracking:4194304 rollout:QuadMixed:4194304 \
    > "$OUT/evidence_cls.log" 2>&1 || { tail -n 20 "$OUT/evidence_cls.log"; exit 1; }
  echo "cls valu / traffic ok"
else
  bash scripts/gpu_roofline_evidence.sh "$TAG" > "$OUT/evidence_large.log" 2>&1 || { tail -n 20 "$OUT/evidence_large.log"; exit 1; }
  echo "evidence large-N ok"
  stage
  step bench_default 500 python -u bench.py --detail "$OUT/bench_detail_default.json"
  driver_bench
  tail -c 300 "$OUT/bench_default.out"; echo
fi
