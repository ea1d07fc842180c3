# Bench line + kernel-trace step breakdown + PMC traffic of the dominant kernel (no tests):
#   gpurun -- bash tools/gpu_bench.sh TAG [bench args]
# The trace is of the bench command itself (roofline probes included, CPU baseline off), so the
# --stats summary holds both the step's launches and the probe's launches of the dominant kernel.
set -o pipefail
tag=${1:-r02}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
rm -rf gpurun_out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --serial-wgrad "$@" > gpurun_out/trace_$tag.log 2>&1 \
    || { tail -20 gpurun_out/trace_$tag.log; exit 1; }
python3 tools/step_profile.py gpurun_out/trace_$tag 60 --json gpurun_out/step_top_$tag.json > gpurun_out/step_$tag.txt
head -25 gpurun_out/step_$tag.txt
dom=${DOM:-$(python3 -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import dominant_kernel as d; print(d.dominant())")}
rm -rf gpurun_out/pmc_f_$tag gpurun_out/pmc_w_$tag
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_f_$tag -o run --output-format csv -- \
    python3 tools/dominant_kernel.py $dom > gpurun_out/pmc_f_$tag.log 2>&1 || { tail -5 gpurun_out/pmc_f_$tag.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_w_$tag -o run --output-format csv -- \
    python3 tools/dominant_kernel.py $dom > gpurun_out/pmc_w_$tag.log 2>&1 || { tail -5 gpurun_out/pmc_w_$tag.log; exit 1; }
python3 tools/pmc_traffic.py $dom gpurun_out/pmc_f_$tag gpurun_out/pmc_w_$tag > gpurun_out/pmc_$tag.json && cat gpurun_out/pmc_$tag.json
