set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 100 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/am.log 2>&1; rc=$?
tail -1 gpurun_out/am.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Timeout" gpurun_out/am.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --prior --no-cpu-baseline > gpurun_out/bam.json 2> gpurun_out/bam.err || { tail -5 gpurun_out/bam.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); a=d['attention_kernel']; print('prior', round(d['ms_per_step'],3), 'ms attn fwd', round(a['fwd_ms'],3), 'bwd', round(a['bwd_ms'],3))" gpurun_out/bam.json
