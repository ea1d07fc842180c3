set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_conv_engines.py -k "dgrad_s2" > gpurun_out/pytest_r05g.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r05g.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r05g.log | head; exit $rc; }
bash tools/gpu_ab.sh conv "4,4,512,512,128,4,2,1,1,dgrad" "8,8,256,256,64,4,2,1,1,dgrad" "4,8,512,512,128,2,2,0,0,dgrad" "8,16,256,256,64,2,2,0,0,dgrad"

