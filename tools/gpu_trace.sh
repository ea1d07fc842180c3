# Kernel-trace step breakdown of the bench step only:  gpurun -- bash tools/gpu_trace.sh TAG [bench args]
set -o pipefail
tag=${1:-t}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-roofline --serial-wgrad "$@" > gpurun_out/trace_$tag.log 2>&1 \
    || { tail -20 gpurun_out/trace_$tag.log; exit 1; }
python3 tools/step_profile.py gpurun_out/trace_$tag 80 --json gpurun_out/step_top_$tag.json > gpurun_out/step_$tag.txt
head -60 gpurun_out/step_$tag.txt
