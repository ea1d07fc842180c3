set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib
timeout -k 10 600 python -u -m pytest -m gpu -q -s --timeout 300 --timeout-method thread tests/test_gpu_determinism.py tests/test_gpu_library.py tests/test_gpu_upsample.py > gpurun_out/lib.log 2>&1; rc=$?
grep -E "differ|passed|failed|^E |  " gpurun_out/lib.log | head -60; echo "rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/gpu_env_ab.sh "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=1"
