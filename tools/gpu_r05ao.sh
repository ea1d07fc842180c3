set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for env in "TORCH_BLAS_PREFER_HIPBLASLT=0" "X=1"; do
  for r in 1 2 3; do
    env $env timeout -k 10 120 python -u -m pytest -m gpu -q --timeout 100 --timeout-method thread tests/test_gpu_pixelsnail.py -k lanes > gpurun_out/ao.log 2>&1; rc=$?
    echo "$env run $r rc=$rc $(tail -1 gpurun_out/ao.log)"
    [ $rc -le 1 ] || exit $rc
  done
done
