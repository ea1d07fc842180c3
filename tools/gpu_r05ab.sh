set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q -s --timeout 300 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/ab.log 2>&1; rc=$?
grep -E "rel|passed|failed|^E " gpurun_out/ab.log | head -30; echo "rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bab.json 2> gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],3), 'ms', d['config']['final_loss'])" gpurun_out/bab.json
