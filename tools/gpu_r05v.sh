set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
VQ3D_LIB=$L/libvq3d_e.so timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_preact_col.py tests/test_gpu_preact_small.py > gpurun_out/v.log 2>&1; rc=$?
tail -2 gpurun_out/v.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/v.log | head -20
[ $rc -le 1 ] || exit $rc
for v in d e f; do echo "== $v"; VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 200 python3 tools/probe_time.py "k_col_fwd<4_2" "k_col_bwd<4_2" "k_col_fwd<8_4" "k_col_bwd<8_4" "k_col_fwd<2_1" "k_col_bwd<2_1" 2>&1 | grep -v amdgpu.ids; done
for v in d e f d e f; do
  VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > gpurun_out/bn_$v.json 2> gpurun_out/bn_$v.err || { tail -5 gpurun_out/bn_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" gpurun_out/bn_$v.json $v
done
