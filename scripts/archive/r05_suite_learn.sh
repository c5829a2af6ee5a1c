#!/bin/bash
# Round 5: the class-layout GPU tests, smoke(), the skinny weight-gradient A/B and the learner bench (config D).
set -u
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_kernels.py -m gpu -q -x -k cls_large --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r05x/pytest_cls.out 2>&1 || { tail -30 gpurun_out/r05x/pytest_cls.out; exit 1; }
tail -2 gpurun_out/r05x/pytest_cls.out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05x/smoke.out 2>&1 || { tail -20 gpurun_out/r05x/smoke.out; exit 1; }
echo smoke ok
timeout -k 10 300 python -u scripts/exp/skinny_wgrad_ab.py > gpurun_out/r05x/skinny.jsonl 2> gpurun_out/r05x/skinny.err || { tail -5 gpurun_out/r05x/skinny.err; exit 1; }
echo skinny ok
timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 --warmup 3 > gpurun_out/r05x/bench_learner.json 2> gpurun_out/r05x/bench_learner.err || { tail -5 gpurun_out/r05x/bench_learner.err; exit 1; }
cat gpurun_out/r05x/bench_learner.json
