set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  timeout -k 10 120 python -u -m pytest -m gpu -q -rxX --timeout 100 --timeout-method thread tests/test_gpu_pixelsnail.py -k lanes > gpurun_out/aq.log 2>&1; rc=$?
  echo "run $r rc=$rc $(tail -1 gpurun_out/aq.log)"
  [ $rc -le 1 ] || exit $rc
done
