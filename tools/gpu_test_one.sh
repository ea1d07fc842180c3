set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/one.log 2>&1
rc=$?
tail -30 gpurun_out/one.log
exit $rc
