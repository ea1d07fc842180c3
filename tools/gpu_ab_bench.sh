# bench.py variants back to back on one box (A/B of launch / stream options), one JSON line each:
#   gpurun -- bash tools/gpu_ab_bench.sh TAG "ARGS1" "ARGS2" ...
# Each variant: bench.py --no-cpu-baseline --no-roofline ARGSi -> gpurun_out/TAG_abI.json; stops at
# the first failing run.
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
i=0
for args in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/${tag}_ab$i.log 2>&1 || { tail -5 gpurun_out/${tag}_ab$i.log; exit 1; }
  tail -1 gpurun_out/${tag}_ab$i.log > gpurun_out/${tag}_ab$i.json
  echo "[$args] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/${tag}_ab$i.json')); print(round(d['ms_per_step'],3), 'ms', d['launch'])")"
done
