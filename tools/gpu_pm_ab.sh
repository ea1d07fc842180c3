# fused 18-channel block forward: brick geometry A/B (parity with the default, then timing of both)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_mid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pm_tests.log 2>&1 || { tail -30 gpurun_out/pm_tests.log; exit 1; }
tail -1 gpurun_out/pm_tests.log
for b in 8 16; do
  VQ3D_PM_BRICK=$b timeout -k 10 120 python -c "
import sys, json, torch; sys.path.insert(0, '3d-vq-vae-2_amd'); import bench
r = bench.dominant_kernel_roofline('bf16', torch.device('cuda:0'))
print('brick $b', round(r['avg_launch_us'], 2), 'us', round(r['frac'], 4))" 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pm_bench.json 2> gpurun_out/pm_bench.err || { tail -20 gpurun_out/pm_bench.err; exit 1; }
cut -c1-200 gpurun_out/pm_bench.json
