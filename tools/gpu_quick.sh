set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_conv_engines.py -x -q > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
for m in fwd dgrad; do for a in "9 9 128 128 32 3 1 1 1" "4 4 512 512 128 3 1 1 1" "2 2 512 512 128 3 1 1 1" "16 16 64 64 16 3 1 1 1" "8 8 256 256 64 4 2 1 1"; do
  timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 >> gpurun_out/q_micro.log 2>&1
done; done
