# lines weight gradient for C % 4 != 0: engine tests, A/B micro timings, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_engines.py tests/test_gpu_conv_small.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng.log 2>&1 || { tail -40 gpurun_out/eng.log; exit 1; }
tail -2 gpurun_out/eng.log
: > gpurun_out/wg_ab.log
for a in "9 9 128 128 32 3 1 1 1" "1 1 128 128 32 3 1 1 1" "2 2 128 128 32 3 1 1 1" "2 2 512 512 128 3 1 1 1" "4 4 256 256 64 4 2 1 1" "4 4 512 512 128 4 2 1 1" "36 36 32 32 8 3 1 1 1" "4 4 256 256 64 3 1 1 1" "16 16 64 64 16 3 1 1 1"; do
  timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 >> gpurun_out/wg_ab.log 2>&1 || exit 1
  VQ3D_DISABLE_LINES_WGRAD=1 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 | sed 's/^/  old /' >> gpurun_out/wg_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/wg_ab.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
