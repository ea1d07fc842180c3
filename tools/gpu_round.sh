# GPU round check: parity tests, the bench line, and a kernel-trace profile of the bench step.
#   gpurun -- bash tools/gpu_round.sh [TAG] [bench args...]
set -o pipefail
tag=${1:-r02}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
rm -rf gpurun_out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-roofline "$@" > gpurun_out/trace_$tag.log 2>&1 \
    || { tail -20 gpurun_out/trace_$tag.log; exit 1; }
python3 tools/step_profile.py gpurun_out/trace_$tag 60 --json gpurun_out/step_top_$tag.json > gpurun_out/step_$tag.txt
head -30 gpurun_out/step_$tag.txt
