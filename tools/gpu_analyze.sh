# Where the step's time goes: per-call-site GPU time of one eager step (tools/call_timing.py) and
# SQ counter passes over the named kernel probes (tools/gpu_pmc_probe.sh):
#   gpurun -- bash tools/gpu_analyze.sh TAG [PROBE ...]
set -o pipefail
tag=${1:-an}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/call_timing.py 3l_pub --top 90 > gpurun_out/calls_$tag.txt 2>&1 || { tail -20 gpurun_out/calls_$tag.txt; exit 1; }
head -40 gpurun_out/calls_$tag.txt
[ $# -gt 0 ] && bash tools/gpu_pmc_probe.sh $tag "$@"
exit 0
