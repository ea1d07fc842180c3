# full GPU suite, bench line, and a kernel-trace profile of the bench (serial wgrad)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof7
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof7 -o run -- python3 bench.py --steps 3 --warmup 3 --serial-wgrad > gpurun_out/prof7.log 2>&1 || { tail -20 gpurun_out/prof7.log; exit 1; }
