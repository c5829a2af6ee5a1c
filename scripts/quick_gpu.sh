# GPU tests, then the launch probe and a short bench per task.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for t in ${TASKS:-LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed}; do
  timeout -k 10 300 python bench.py --task $t --steps 1000 --warmup 50 --no-cpu-baseline ${BENCH_FLAGS:---no-sweep} > gpurun_out/q_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/q_$t.json'));f=d.get('fused_rollout',{});print('$t', 'value %.3g k_us %.2f fused %.3g'%(d['value'],d['roofline']['kernel_us'],f.get('value',0)), ' '.join('N=%d k_us %.1f frac %.3f'%(s['num_envs'],s['kernel_us'],s['frac']) for s in d.get('roofline_sweep',[])))"
done
