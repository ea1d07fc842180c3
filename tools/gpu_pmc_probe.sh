# SQ counter passes (one set per run) over one of bench.py's kernel probes:
#   gpurun -- bash tools/gpu_pmc_probe.sh TAG PROBE [PROBE ...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for probe in "$@"; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAIT_INST_LDS" "SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    rm -rf gpurun_out/pmc_${tag}_${probe}_$i
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${tag}_${probe}_$i -o run -- python3 tools/dominant_kernel.py $probe 3 > gpurun_out/pmc_${tag}_${probe}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${tag}_${probe}_$i.log; exit 1; }
  done
  python3 tools/pmc_kernels.py "gpurun_out/pmc_${tag}_${probe}_*" $probe
done
