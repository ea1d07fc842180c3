set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 700 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_conv_engines.py tests/test_gpu_pixelsnail.py tests/test_gpu_determinism.py tests/test_gpu_parity.py > gpurun_out/ac.log 2>&1; rc=$?
tail -1 gpurun_out/ac.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/ac.log | head -20
[ $rc -le 1 ] || exit $rc
for v in j k; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 400 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bac.json 2> gpurun_out/bac.err || { tail -5 gpurun_out/bac.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'prior', round(d['ms_per_step'],3), 'ms')" gpurun_out/bac.json $v
done
for v in j k j k; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > gpurun_out/bn_$v.json 2> gpurun_out/bn_$v.err || { tail -5 gpurun_out/bn_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" gpurun_out/bn_$v.json $v
done
