set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 100 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/ap.log 2>&1; rc=$?
tail -1 gpurun_out/ap.log; [ $rc -eq 0 ] || grep -E "^E " gpurun_out/ap.log | cut -c1-200 | head -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --prior > gpurun_out/bap.json 2> gpurun_out/bap.err || { tail -5 gpurun_out/bap.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); a=d['attention_kernel']; print('prior', round(d['ms_per_step'],3), 'ms', round(d['value'],2), 'attn fwd', round(a['fwd_ms'],3), 'bwd', round(a['bwd_ms'],3), 'cpu', d.get('cpu_baseline',{}).get('value'))" gpurun_out/bap.json
