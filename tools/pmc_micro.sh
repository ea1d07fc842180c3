# usage: bash tools/pmc_micro.sh TAG <conv_micro args...>   (three separate --pmc passes)
set -e -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAIT_INST_LDS" "SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- python tools/conv_micro.py "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1
done
