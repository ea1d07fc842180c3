# k^3 weight gradient engines: tests with the lines engine forced, A/B micro timings, bench
set -o pipefail
mkdir -p gpurun_out
VQ3D_LINES_WGRAD=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_engines.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng.log 2>&1 || { tail -40 gpurun_out/eng.log; exit 1; }
tail -1 gpurun_out/eng.log
: > gpurun_out/wg_ab.log
for a in "9 9 128 128 32 3 1 1 1" "1 1 128 128 32 3 1 1 1" "2 2 512 512 128 3 1 1 1" "4 4 256 256 64 4 2 1 1" "4 4 512 512 128 4 2 1 1" "36 36 32 32 8 3 1 1 1" "4 4 256 256 64 3 1 1 1" "16 16 64 64 16 3 1 1 1" "8 8 128 128 32 3 1 1 1"; do
  VQ3D_LINES_WGRAD=1 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed 's/^/lines  /' >> gpurun_out/wg_ab.log || exit 1
  VQ3D_LINES_WGRAD=0 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed 's/^/direct /' >> gpurun_out/wg_ab.log || exit 1
done
cat gpurun_out/wg_ab.log
