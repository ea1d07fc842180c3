set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_conv_engines.py tests/test_gpu_parity.py tests/test_gpu_bf16_model.py tests/test_gpu_fullsize_golden.py tests/test_gpu_stale_lds.py > gpurun_out/pytest_r05h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r05h.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r05h.log | head; exit $rc; }
bash tools/gpu_ab.sh bench --steps 20 --warmup 3
