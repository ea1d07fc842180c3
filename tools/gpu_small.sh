# fused few-channel PreAct blocks: parity tests, then the bench step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_small.py -x -v --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -40 gpurun_out/small_tests.log; exit 1; }
tail -3 gpurun_out/small_tests.log
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/small_bench.json 2> gpurun_out/small_bench.err || { tail -20 gpurun_out/small_bench.err; exit 1; }
cat gpurun_out/small_bench.json
