set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 100 --timeout-method thread tests/test_gpu_pixelsnail.py > gpurun_out/an.log 2>&1; rc=$?
grep -E "^E " gpurun_out/an.log | cut -c1-300 | head -8; tail -1 gpurun_out/an.log
exit $rc
