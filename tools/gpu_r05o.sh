# r05o: determinism + kernel tests on the current build, bench a (round start of this change) vs c,
# then a kernel trace of c.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 500 python -u -m pytest -m gpu -q -s --timeout 300 --timeout-method thread tests/test_gpu_determinism.py > gpurun_out/det.log 2>&1; rc=$?
grep -E "differ|entries|passed|failed" gpurun_out/det.log | head -60; echo "det rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_upsample.py tests/test_gpu_conv_engines.py tests/test_gpu_conv_small.py tests/test_gpu_conv_tc.py tests/test_gpu_wgrad_windowed.py tests/test_gpu_parity.py > gpurun_out/kt.log 2>&1; rc=$?
tail -2 gpurun_out/kt.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/kt.log | head -30
[ $rc -le 1 ] || exit $rc
for v in a c a c; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 3 > gpurun_out/bn_$v.json 2> gpurun_out/bn_$v.err || { tail -5 gpurun_out/bn_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value'],2), d['unit'])" gpurun_out/bn_$v.json $v
done
bash tools/gpu_trace_libs.sh o c
