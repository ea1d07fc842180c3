# pointwise weight gradient: lines MFMA engine (k = 1) vs the slab kernel; tests with lines forced
set -o pipefail
mkdir -p gpurun_out
VQ3D_PW_LINES_WGRAD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_engines.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pwwg.log 2>&1 || { tail -40 gpurun_out/pwwg.log; exit 1; }
tail -1 gpurun_out/pwwg.log
: > gpurun_out/pwwg_ab.log
for a in "9 18 128 128 32 1 1 0 0" "18 9 128 128 32 1 1 0 0" "72 36 32 32 8 1 1 0 0" "36 72 32 32 8 1 1 0 0" "2 4 512 512 128 1 1 0 0" "4 2 256 256 64 1 1 0 0" "16 32 64 64 16 1 1 0 0"; do
  VQ3D_PW_LINES_WGRAD=1 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed 's/^/lines /' >> gpurun_out/pwwg_ab.log || exit 1
  VQ3D_PW_LINES_WGRAD=0 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed 's/^/slab  /' >> gpurun_out/pwwg_ab.log || exit 1
done
cat gpurun_out/pwwg_ab.log
