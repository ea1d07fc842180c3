# kernel trace of bench.py with extra flags: gpurun -- bash tools/gpu_trace_flags.sh TAG [bench flags]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
rm -rf gpurun_out/tf_$tag
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tf_$tag -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline "$@" > gpurun_out/tf_$tag.log 2>&1 \
    || { tail -20 gpurun_out/tf_$tag.log; exit 1; }
python3 tools/step_profile.py gpurun_out/tf_$tag 60 > gpurun_out/tf_$tag.txt
head -1 gpurun_out/tf_$tag.txt
