# upsample tests + launch-time A/B of every library variant 3d-vq-vae-2_amd/lib/libvq3d_{a,b,c,...}.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_upsample.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_up.log 2>&1; rc=$?; tail -3 gpurun_out/t_up.log; [ $rc -eq 0 ] || exit 1
for f in "$GRAFT_REPO_ROOT"/3d-vq-vae-2_amd/lib/libvq3d_?.so; do
  echo "== $(basename $f)"; VQ3D_LIB=$f timeout -k 10 200 python3 tools/up_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
