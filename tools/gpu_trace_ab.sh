# kernel-trace A/B of bench.py flag variants: per variant one rocprofv3 --kernel-trace run of a
# short bench and the last step's ranking (tools/step_profile.py), filtered by a kernel pattern.
#   gpurun -- bash tools/gpu_trace_ab.sh TAG PATTERN "flags A" "flags B" ...
set -o pipefail
tag=$1; pat=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
i=0
for flags in "$@"; do
    i=$((i+1))
    rm -rf gpurun_out/tab_${tag}_$i
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tab_${tag}_$i -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline $flags > gpurun_out/tab_${tag}_$i.log 2>&1 \
        || { tail -20 gpurun_out/tab_${tag}_$i.log; exit 1; }
    python3 tools/step_profile.py gpurun_out/tab_${tag}_$i 400 > gpurun_out/tab_${tag}_$i.txt
    echo "== [$flags] $(head -1 gpurun_out/tab_${tag}_$i.txt)"
    grep -E "$pat" gpurun_out/tab_${tag}_$i.txt | head -30
done
