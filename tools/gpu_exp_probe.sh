# Time bench.py kernel probes under several builds of the library (timing-experiment variants
# lib/libvq3d_expN.so from `make exp EXP=N`, or any VQ3D_LIB):
#   gpurun -- bash tools/gpu_exp_probe.sh "PROBE [PROBE ...]" LIB [LIB ...]      (LIB relative to 3d-vq-vae-2_amd/lib)
set -o pipefail
probes=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for lib in "$@"; do
    echo "== $lib"
    VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/$lib timeout -k 10 200 python3 tools/probe_time.py $probes 2>&1 \
        | grep -v amdgpu.ids || exit 1
done
