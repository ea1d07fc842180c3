# Round-end check: smoke(), then the bench line + kernel trace + PMC of the dominant kernel
#   gpurun -- bash tools/gpu_final.sh TAG
set -o pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -2 gpurun_out/smoke_$tag.log
bash tools/gpu_bench.sh $tag
