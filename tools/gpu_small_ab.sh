# small-grid conv engine: tests, A/B micro timings vs the previous engines, then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_small.py tests/test_gpu_tiny_block.py -x -q --timeout 120 --timeout-method thread > gpurun_out/small.log 2>&1 || { tail -40 gpurun_out/small.log; exit 1; }
tail -2 gpurun_out/small.log
: > gpurun_out/small_ab.log
for a in "128 128 8 8 2 3 1 1 1" "128 128 16 16 4 4 2 1 1" "64 64 16 16 4 3 1 1 1" "64 64 32 32 8 3 1 1 1" "36 36 16 16 4 3 1 1 1"; do
  for m in fwd dgrad; do
    timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 >> gpurun_out/small_ab.log 2>&1 || exit 1
    VQ3D_NO_SMALL=1 timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 | sed 's/^/  old /' >> gpurun_out/small_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/small_ab.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
