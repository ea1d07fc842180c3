# block_micro over the experiment variants lib/libvq3d_exp*.so:  gpurun -- bash tools/gpu_exp_col.sh C BR H W D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "product:"; timeout -k 10 60 python3 tools/block_micro.py "$@" 2>&1 | grep -v "amdgpu.ids\|^copy" || exit 1
for f in 3d-vq-vae-2_amd/lib/libvq3d_exp*.so; do
  echo "$f:"; VQ3D_LIB=$GRAFT_REPO_ROOT/$f timeout -k 10 60 python3 tools/block_micro.py "$@" 2>&1 | grep -v "amdgpu.ids\|^copy" || exit 1
done
