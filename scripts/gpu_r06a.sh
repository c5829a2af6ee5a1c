# round-6 check of the new tests on the current library: large-N oracle pins, mixed split with a shard offset,
# output-wave cases, gravity DR, TunableOp default; then the driver's bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06a
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_timed_kernels.py -k "large_n or mixed_split" tests/test_gpu_env.py::test_output_wave_rollout_matches_one_wave \
  tests/test_dr_physical.py -m gpu "tests/test_gpu_learner.py::test_shipped_gemm_tuning_applies_on_this_box" \
  > gpurun_out/r06a/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/r06a/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep \
  --detail gpurun_out/r06a/bench_detail.json > gpurun_out/r06a/bench.out 2> gpurun_out/r06a/bench.err
rc=$?; tail -c 1500 gpurun_out/r06a/bench.out; exit $rc
