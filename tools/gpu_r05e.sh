set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_library.py tests/test_gpu_bf16_model.py tests/test_gpu_fullsize_golden.py tests/test_gpu_multistep_oracle.py > gpurun_out/pytest_r05e.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r05e.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r05e.log | head -20; exit $rc; }
bash tools/gpu_ab_flags.sh r05e "--no-overlap-levels" "" "--no-overlap-levels" ""
