# tiny-channel engine: tests vs torch, A/B micro timings against the MFMA engines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_tc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1 || { tail -40 gpurun_out/tc.log; exit 1; }
tail -1 gpurun_out/tc.log
: > gpurun_out/tc_ab.log
for a in "2 2 512 512 128 3 1 1 1" "1 1 128 128 32 3 1 1 1"; do
for m in fwd dgrad wgrad; do
  timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 2>/dev/null | sed 's/^/tc   /' >> gpurun_out/tc_ab.log || exit 1
  VQ3D_NO_TC=1 timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 2>/dev/null | sed 's/^/old  /' >> gpurun_out/tc_ab.log || exit 1
done; done
cat gpurun_out/tc_ab.log
