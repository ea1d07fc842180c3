set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
echo done
