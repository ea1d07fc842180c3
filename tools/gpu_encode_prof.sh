# encode-only bench line + its kernel statistics (cfg4): gpurun -- bash tools/gpu_encode_prof.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-enc}
timeout -k 10 300 python3 bench.py --encode-only > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -5 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
rm -rf gpurun_out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 bench.py --encode-only --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_$tag.log 2>&1 \
    || { tail -20 gpurun_out/trace_$tag.log; exit 1; }
