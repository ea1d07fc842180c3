set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_preact_col.py tests/test_gpu_preact_small.py > gpurun_out/pytest_r05i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r05i.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_r05i.log | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16_model.py tests/test_gpu_fullsize_golden.py tests/test_gpu_library.py > gpurun_out/pytest_r05i2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r05i2.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_r05i2.log | head -20; exit $rc; }
bash tools/gpu_ab_flags.sh r05i "--no-small-chain" "" "--no-small-chain" ""
