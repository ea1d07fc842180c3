# fused few-channel blocks: parity, bench at the default fused-backward size limit and with the
# fused backward on every grid
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_small.py -x -q --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -40 gpurun_out/small_tests.log; exit 1; }
tail -1 gpurun_out/small_tests.log
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline"
timeout -k 10 240 $B 2>/dev/null | python -c "import json,sys; print('default', json.loads(sys.stdin.readlines()[-1])['ms_per_step'])" || exit 1
VQ3D_SMALL_BWD_MAX_VOX=1000000000 timeout -k 10 240 $B 2>/dev/null | python -c "import json,sys; print('all-fused', json.loads(sys.stdin.readlines()[-1])['ms_per_step'])" || exit 1
