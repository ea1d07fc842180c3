# dominant kernel iteration: its parity tests, PMC HBM traffic (two passes), bench with roofline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_mid.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dom_tests.log 2>&1 || { tail -30 gpurun_out/dom_tests.log; exit 1; }
tail -1 gpurun_out/dom_tests.log
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- python3 tools/dominant_kernel.py > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- python3 tools/dominant_kernel.py > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w > gpurun_out/pmc_dominant.json || exit 1
grep -E "fetch|write_size|hbm" gpurun_out/pmc_dominant.json
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dom_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/dom_bench.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
