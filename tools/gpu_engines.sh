# The fused-block engine tests (after an engine change): stack / wide / mid / col / small / tiny.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_preact_stack.py \
    tests/test_gpu_preact_wide.py tests/test_gpu_preact_mid.py tests/test_gpu_preact_col.py tests/test_gpu_preact_small.py \
    tests/test_gpu_tiny_block.py tests/test_gpu_stale_lds.py "$@" > gpurun_out/pytest_engines.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_engines.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_engines.log | head -20; exit $rc; }
