cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
echo base; VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_a.so timeout -k 10 200 python3 tools/probe_time.py "$@" 2>&1 | grep -v amdgpu.ids
echo variant; VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_b.so timeout -k 10 200 python3 tools/probe_time.py "$@" 2>&1 | grep -v amdgpu.ids
