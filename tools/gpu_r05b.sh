set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread "tests/test_gpu_fullsize_golden.py::test_published_model_fullsize_vs_reference[fp16]" "tests/test_gpu_parity.py::test_level_overlap_matches_serial_3l" "tests/test_gpu_parity.py::test_concurrent_wgrad_and_graph_replay_match_serial" > gpurun_out/pytest_r05b.log 2>&1
rc=$?; grep -E "vs the reference|passed|failed|Error|assert" gpurun_out/pytest_r05b.log | head -20; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_flags.sh r05b "--no-overlap-levels" "" "--no-overlap-levels" ""
