set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 600 python -u -m pytest -m gpu -q -s --timeout 300 --timeout-method thread tests/test_gpu_determinism.py tests/test_gpu_library.py tests/test_gpu_upsample.py > gpurun_out/lib.log 2>&1; rc=$?
grep -E "differ|passed|failed|^E |  " gpurun_out/lib.log | head -60; echo "rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/gpu_env_ab.sh "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=1"
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k batched > gpurun_out/benc.log 2>&1; rc=$?; tail -1 gpurun_out/benc.log; [ $rc -le 1 ] || exit $rc
for b in 1 2 4 8; do
  timeout -k 10 300 python3 bench.py --encode-only --encode-batch $b --no-cpu-baseline --no-roofline > gpurun_out/enc_$b.json 2> gpurun_out/enc_$b.err || { tail -5 gpurun_out/enc_$b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('encode batch', sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value'],2), d['unit'])" gpurun_out/enc_$b.json $b
done
bash tools/gpu_mfma.sh r05
