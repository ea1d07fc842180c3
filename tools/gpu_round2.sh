# round measurement: GPU tests, PMC HBM traffic of the dominant kernel (two separate counter
# passes), kernel-trace --stats of the bench, then the bench line itself
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/stats
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- python3 tools/dominant_kernel.py > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- python3 tools/dominant_kernel.py > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w > gpurun_out/pmc_dominant.json || exit 1
cp gpurun_out/pmc_dominant.json profiles/pmc_dominant.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stats.log 2>&1 || { tail -20 gpurun_out/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_step -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline --serial-wgrad > gpurun_out/prof_step.log 2>&1 || { tail -20 gpurun_out/prof_step.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
