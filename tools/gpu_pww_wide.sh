# wide register-path pointwise weight gradient (9 <-> 18 channels) vs the slab kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_engines.py -k pointwise -x -q --timeout 120 --timeout-method thread > gpurun_out/pww.log 2>&1 || { tail -30 gpurun_out/pww.log; exit 1; }
tail -1 gpurun_out/pww.log
: > gpurun_out/pww_wide.log
for a in "9 18 128 128 32 1 1 0 0" "18 9 128 128 32 1 1 0 0"; do
  timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed "s/^/wide /" >> gpurun_out/pww_wide.log || exit 1
  VQ3D_PWW_NO_WIDE=1 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed "s/^/slab /" >> gpurun_out/pww_wide.log || exit 1
done
cat gpurun_out/pww_wide.log
