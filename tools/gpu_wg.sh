set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_conv_engines.py -x -q > gpurun_out/wg_tests.log 2>&1
for a in "9 9 128 128 32 3 1 1 1" "4 4 512 512 128 3 1 1 1" "16 16 64 64 16 3 1 1 1" "36 36 32 32 8 3 1 1 1" "4 4 512 512 128 4 2 1 1" "9 9 256 256 64 4 2 1 1"; do
  timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 >> gpurun_out/wg_micro.log 2>&1
done
for m in fwd dgrad; do for a in "9 9 128 128 32 3 1 1 1" "4 4 512 512 128 3 1 1 1" "18 9 128 128 32 1 1 0 0" "9 18 128 128 32 1 1 0 0" "4 2 512 512 128 1 1 0 0" "2 4 512 512 128 1 1 0 0"; do
  timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 >> gpurun_out/pw_micro.log 2>&1
done; done
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/parity.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/hiptr -o run -- python bench.py --config 2l_dflt --size 128 128 32 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/hiptr.log 2>&1
