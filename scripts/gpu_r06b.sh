# round-6: the gravity DR / output-wave / TunableOp GPU tests (r06a's -k filter deselected them)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  \
  "tests/test_gpu_learner.py::test_shipped_gemm_tuning_applies_on_this_box" "tests/test_gpu_learner.py::test_training_loop_runs" \
  -m gpu > gpurun_out/r06b/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/r06b/pytest.log; exit $rc
