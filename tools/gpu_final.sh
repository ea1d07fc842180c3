# Round-end measurement set: GPU tests, the bench step's kernel trace (the step ranking bench.py
# reads), PMC HBM traffic of the top kernels, then the bench line and the other configurations.
#   gpurun -- bash tools/gpu_final.sh TAG
set -o pipefail
tag=${1:-r05x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/pytest_$tag.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -2 gpurun_out/smoke_$tag.log
rm -rf gpurun_out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/trace_$tag.log 2>&1 \
    || { tail -20 gpurun_out/trace_$tag.log; exit 1; }
python3 tools/step_profile.py gpurun_out/trace_$tag 60 --json gpurun_out/step_top_$tag.json > gpurun_out/step_$tag.txt || exit 1
head -12 gpurun_out/step_$tag.txt
cp gpurun_out/step_top_$tag.json profiles/r05_step_top.json
bash tools/gpu_traffic.sh $tag "k_pm_bwd2:k_pm_bwd2<true k_pm_fwd:k_pm_fwd<true k_pm_w2grad k_pm_w13grad k_col_bwd<4_2 k_col_fwd<4_2 k_stackm_bwd k_stackm_fwd" || exit 1
for f in gpurun_out/${tag}_pmc_*.json; do b=$(basename $f); cp $f profiles/r05_pmc_${b#${tag}_pmc_}; done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cut -c1-400 gpurun_out/bench_$tag.json
for cfg in "--config 2l_pub" "--encode-only" "--encode-only --encode-batch 8" "--prior"; do
  n=$(echo $cfg | tr -d ' -'); timeout -k 10 400 python3 bench.py $cfg --no-cpu-baseline > gpurun_out/bench_${tag}_$n.json 2> gpurun_out/bench_${tag}_$n.err || { tail -5 gpurun_out/bench_${tag}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value'],2), d['unit'])" gpurun_out/bench_${tag}_$n.json "$cfg"
done
