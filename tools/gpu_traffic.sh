# HBM bytes per launch (PMC FETCH_SIZE / WRITE_SIZE, one counter per pass; MI355X_MICROARCH.md §HBM
# corrections in pmc_traffic.py) of bench.py kernel probes, into gpurun_out/TAG_pmc_<probe>.json:
#   gpurun -- bash tools/gpu_traffic.sh TAG "PROBE[:KERNEL_SUBSTRING] ..."
# KERNEL_SUBSTRING picks the probe's dominant kernel in the trace (default: the probe name; ", " in
# template arguments written as "_", e.g. k_pm_fwd:k_pm_fwd<true or k_col_bwd<4_2).
set -o pipefail
tag=$1; items=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for it in $items; do
  probe=${it%%:*}; kern=${it#*:}
  [ "$kern" = "$it" ] && kern=$probe
  d=gpurun_out/tr_${tag}_${probe//[<>]/_}
  rm -rf ${d}_f ${d}_w
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${d}_f -o run --output-format csv -- \
      python3 tools/dominant_kernel.py "$probe" 6 > ${d}_f.log 2>&1 || { tail -5 ${d}_f.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d ${d}_w -o run --output-format csv -- \
      python3 tools/dominant_kernel.py "$probe" 6 > ${d}_w.log 2>&1 || { tail -5 ${d}_w.log; exit 1; }
  python3 tools/pmc_traffic.py "$kern" ${d}_f ${d}_w > gpurun_out/${tag}_pmc_${probe}.json || exit 1
  echo "$probe: $(cat gpurun_out/${tag}_pmc_${probe}.json | tr -d '\n' | cut -c1-300)"
done
