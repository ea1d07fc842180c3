# one GPU iteration: full GPU test suite, then per-call timing of the 3L published step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 400 python tools/call_timing.py --top 150 > gpurun_out/calls.txt 2>&1 || { tail -30 gpurun_out/calls.txt; exit 1; }
head -3 gpurun_out/calls.txt
