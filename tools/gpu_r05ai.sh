set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ai.log 2>&1; rc=$?
tail -2 gpurun_out/ai.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/ai.log | head -30
exit $rc
