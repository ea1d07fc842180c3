# PixelSNAIL lanes capture: the HIP stream / event / capture API calls of a small model's capture
# (AMD_LOG_LEVEL=3), forward-only first, then forward + backward; stops at the first failure.
#   gpurun -- bash tools/dbg/lanes.sh TAG [num_blocks layers]
set -o pipefail
tag=${1:-dbg}
nb=${2:-1}
nl=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in fwd bwd; do
  AMD_LOG_LEVEL=3 timeout -k 10 120 python3 -u tools/dbg/lanes_capture.py $m $nb $nl > gpurun_out/${tag}_raw_$m.log 2>&1; rc=$?
  echo "$m rc=$rc"
  grep -E "eager ok|capture stream|step issued|captured|replayed|Fatal|Segmentation|hipStreamBeginCapture|hipStreamEndCapture|hipStreamWaitEvent|hipEventRecord|hipEventCreate|hipEventDestroy|hipStreamIsCapturing|hipStreamGetCaptureInfo|hipGraph|hipStreamCreate|error|Error" \
      gpurun_out/${tag}_raw_$m.log | grep -v "hipGetLastError" | tail -4000 > gpurun_out/${tag}_cap_$m.log
  tail -c 200000 gpurun_out/${tag}_raw_$m.log > gpurun_out/${tag}_tail_$m.log
  rm -f gpurun_out/${tag}_raw_$m.log
  [ $rc -eq 0 ] || exit $rc
done
