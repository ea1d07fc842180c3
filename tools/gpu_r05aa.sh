set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_pixelsnail.py -k "matrix_core or mid_level or prior" > gpurun_out/aa.log 2>&1; rc=$?
tail -3 gpurun_out/aa.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" gpurun_out/aa.log | head -20
