set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests/test_gpu_fullsize_golden.py > gpurun_out/pytest_r05d.log 2>&1
grep -E "vs the reference|passed|failed|Error" gpurun_out/pytest_r05d.log | head -8
