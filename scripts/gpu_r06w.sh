#!/bin/bash
# Round 6, VERDICT r05 item 2(a) measured: the large-N estimator rollout without its scratch spill.  A variant build of
# the same sources with -DOUZ_EST_ROLLOUT_WPE=1 (register budget for one wave per SIMD: 256 VGPR + 104 AGPR, no
# scratch; build: OUZ_BUILD_OUT=ouzelum_amd/libouzelum_hip_wpe1.so OUZ_EXTRA_FLAGS=-DOUZ_EST_ROLLOUT_WPE=1
# python -c "from ouzelum_amd import build; build.build(force=True)") against the shipped WPE = 2 build (two waves per
# SIMD, 111 VGPRs spilled), same box, interleaved: rocprofv3 --stats + FETCH_SIZE / WRITE_SIZE passes and the two VALU
# passes of QuadTracking and QuadMixed rollouts at 4 M envs (16-step launches), tags r06w1 (variant) / r06w2 (shipped).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
E="rollout:QuadTracking:4194304 rollout:QuadMixed:4194304"
for round in 1 2; do
  OUZ_LIB=$R/ouzelum_amd/libouzelum_hip_wpe1.so bash scripts/gpu_roofline_evidence.sh r06w1r$round $E > gpurun_out/r06w1_$round.log 2>&1 || exit 1
  bash scripts/gpu_roofline_evidence.sh r06w2r$round $E > gpurun_out/r06w2_$round.log 2>&1 || exit 1
done
OUZ_LIB=$R/ouzelum_amd/libouzelum_hip_wpe1.so bash scripts/gpu_valu.sh r06w1 $E > gpurun_out/r06w1_valu.log 2>&1 || exit 1
bash scripts/gpu_valu.sh r06w2 $E > gpurun_out/r06w2_valu.log 2>&1 || exit 1
echo ok
