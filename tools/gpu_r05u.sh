set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_conv_engines.py tests/test_gpu_determinism.py > gpurun_out/u.log 2>&1; rc=$?
tail -2 gpurun_out/u.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/u.log | head -20
[ $rc -le 1 ] || exit $rc
for v in c d c d; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > gpurun_out/bn_$v.json 2> gpurun_out/bn_$v.err || { tail -5 gpurun_out/bn_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" gpurun_out/bn_$v.json $v
done
bash tools/gpu_trace_libs.sh u d
grep -E "wgrad_tiled|gen_reduce" gpurun_out/tl_u_d.txt | head
