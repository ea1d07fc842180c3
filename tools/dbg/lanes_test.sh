# The lanes test itself (tests/test_gpu_pixelsnail.py -k lanes_match), first with the HIP API log
# (AMD_LOG_LEVEL=3: capture / stream / event calls kept), then without it; stops at the first failure.
#   gpurun -- bash tools/dbg/lanes_test.sh TAG [pytest -k expression]
set -o pipefail
tag=${1:-dbg}
k=${2:-lanes_match}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider"
AMD_LOG_LEVEL=3 timeout -k 10 240 $PYT -s tests/test_gpu_pixelsnail.py -k "$k" > gpurun_out/${tag}_raw.log 2>&1; rc=$?
echo "logged rc=$rc"
grep -E "PASSED|FAILED|Fatal|Segmentation|hipStreamBeginCapture|hipStreamEndCapture|hipStreamWaitEvent|hipEventRecord|hipGraph|error|Error" \
    gpurun_out/${tag}_raw.log | grep -v "hipGetLastError" | tail -6000 > gpurun_out/${tag}_cap.log
tail -c 300000 gpurun_out/${tag}_raw.log > gpurun_out/${tag}_tail.log
rm -f gpurun_out/${tag}_raw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 $PYT tests/test_gpu_pixelsnail.py -k "$k" > gpurun_out/${tag}_plain.log 2>&1; rc=$?
echo "plain rc=$rc"; tail -3 gpurun_out/${tag}_plain.log
exit $rc
