cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_upsample.py tests/test_gpu_parity.py tests/test_gpu_pixelsnail.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_up.log 2>&1; rc=$?; tail -3 gpurun_out/t_up.log; [ $rc -eq 0 ] || exit 1
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
for v in a b; do echo "== $v"; VQ3D_LIB=$L/libvq3d_$v.so timeout -k 10 200 python3 tools/up_ab.py 2>&1 | grep -v amdgpu.ids; done
timeout -k 10 300 python3 bench.py --prior --no-cpu-baseline > gpurun_out/bench_prior.json 2> gpurun_out/bench_prior.err || { tail -5 gpurun_out/bench_prior.err; exit 1; }; cut -c1-400 gpurun_out/bench_prior.json
