set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/w.log 2>&1; rc=$?
tail -2 gpurun_out/w.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/w.log | head -20
[ $rc -le 1 ] || exit $rc
for v in f g; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 400 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bp_$v.json 2> gpurun_out/bp_$v.err || { tail -5 gpurun_out/bp_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', {k: v for k, v in d.items() if 'attn' in k})" gpurun_out/bp_$v.json $v
done
