set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
VQ3D_LIB=$L/libvq3d_i.so timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/z.log 2>&1; rc=$?
tail -1 gpurun_out/z.log; [ $rc -le 1 ] || exit $rc
for v in h i; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 400 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bz.json 2> gpurun_out/bz.err || { tail -5 gpurun_out/bz.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', 'fwd', round(d['attention_kernel']['fwd_ms'],4), 'bwd', round(d['attention_kernel']['bwd_ms'],4))" gpurun_out/bz.json $v
done
