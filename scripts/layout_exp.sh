# Tiled-layout check: GPU tests, then a sweep per task at HBM-resident sizes.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for t in LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed; do
  timeout -k 10 300 python bench.py --task $t --steps 300 --warmup 20 --no-cpu-baseline --no-fused > gpurun_out/lay_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lay_$t.json'));print('$t', 'bench k_us %.2f value %.3g'%(d['roofline']['kernel_us'],d['value']), ' '.join('N=%d k_us %.1f frac %.3f'%(s['num_envs'],s['kernel_us'],s['frac']) for s in d['roofline_sweep']))"
done
