# kernel-trace A/B of library builds: per build (3d-vq-vae-2_amd/lib/libvq3d_<v>.so) one rocprofv3
# --kernel-trace run of a short bench and the last step's ranking (tools/step_profile.py).
#   gpurun -- bash tools/gpu_trace_libs.sh TAG v1 v2 ...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in "$@"; do
    rm -rf gpurun_out/tl_${tag}_$v
    VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_${tag}_$v -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/tl_${tag}_$v.log 2>&1 \
        || { tail -20 gpurun_out/tl_${tag}_$v.log; exit 1; }
    python3 tools/step_profile.py gpurun_out/tl_${tag}_$v 2000 > gpurun_out/tl_${tag}_$v.txt
    echo "== $v $(head -1 gpurun_out/tl_${tag}_$v.txt)"
done
