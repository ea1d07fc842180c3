set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/ah.log 2>&1; rc=$?
tail -1 gpurun_out/ah.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/ah.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bah.json 2> gpurun_out/bah.err || { tail -5 gpurun_out/bah.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('prior', round(d['ms_per_step'],3), 'ms')" gpurun_out/bah.json
bash tools/gpu_prior_trace.sh | head -40
