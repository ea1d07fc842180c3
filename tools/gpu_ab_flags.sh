# A/B of bench.py command-line variants on one box (same library): each variant's bench line.
#   gpurun -- bash tools/gpu_ab_flags.sh TAG "flags A" "flags B" ...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
i=0
for flags in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $flags \
        > gpurun_out/ab_${tag}_$i.json 2> gpurun_out/ab_${tag}_$i.err || { tail -20 gpurun_out/ab_${tag}_$i.err; exit 1; }
    echo "[$flags] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${tag}_$i.json')); print(round(d['ms_per_step'],3), 'ms', round(d['config'].get('final_loss',0),6))")"
done
