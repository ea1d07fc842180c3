set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_level_overlap_matches_serial_3l" > gpurun_out/pytest_r05c.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/pytest_r05c.log | head -20; [ $rc -eq 0 ] || exit $rc
VQ3D_STACK_VALU=1 timeout -k 10 300 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread "tests/test_gpu_fullsize_golden.py::test_published_model_fullsize_vs_reference[bf16]" > gpurun_out/pytest_r05c2.log 2>&1
grep -E "vs the reference|passed|failed" gpurun_out/pytest_r05c2.log | head -5
bash tools/gpu_ab_flags.sh r05c "--no-overlap-levels" "" "--no-overlap-levels" ""
VQ3D_STACK_VALU=1 bash tools/gpu_ab_flags.sh r05cv ""
