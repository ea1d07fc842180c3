# A/B bench variants (+ optional focused tests) in one GPU call:
#   gpurun -- bash tools/gpu_ab.sh TAG "PYTEST_ARGS|-" "BENCH_ARGS_A" "BENCH_ARGS_B" ...
set -o pipefail
tag=$1; shift; tests=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$tests" != "-" ]; then
    timeout -k 10 600 python -u -m pytest $tests -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
    rc=$?; tail -5 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for v in "$@"; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline $v > gpurun_out/ab_${tag}_$i.json 2> gpurun_out/ab_${tag}_$i.err \
        || { tail -20 gpurun_out/ab_${tag}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), d.get('launch'))" gpurun_out/ab_${tag}_$i.json "[$v]"
    i=$((i+1))
done
