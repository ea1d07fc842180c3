set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in bwd_noflush full; do
  AMD_LOG_LEVEL=1 timeout -k 10 120 python3 -u tools/dbg/lanes_capture.py $m > gpurun_out/dbg_$m.log 2>&1; rc=$?
  echo "$m rc=$rc"; grep -E "hipGraph|Capture|capture|Fatal|backward|eager|hipStreamCreate|hipStreamWaitEvent \(|hipEventRecord \(" gpurun_out/dbg_$m.log > gpurun_out/dbg_cap.log; rm -f gpurun_out/dbg_$m.log
  [ $rc -eq 0 ] || exit $rc
done
