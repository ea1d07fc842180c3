# Mid-level engine check: its GPU tests, then bench.py probe timings under one or more library
# builds (LIB relative to 3d-vq-vae-2_amd/lib; the first is the product build).
#   gpurun -- bash tools/gpu_mid.sh "PROBE [PROBE ...]" LIB [LIB ...]
set -o pipefail
probes=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_mid.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/mid_tests.log 2>&1 || { tail -30 gpurun_out/mid_tests.log; exit 1; }
tail -2 gpurun_out/mid_tests.log
for lib in "$@"; do
    echo "== $lib"
    VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/$lib timeout -k 10 200 python3 tools/probe_time.py $probes 2>&1 \
        | grep -v amdgpu.ids || exit 1
done
