# PMC passes (one counter set per run) over tools/block_micro.py:  gpurun -- bash tools/gpu_pmc_block.sh TAG [block args]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/block_micro.py "$@" || exit 1
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${tag}_$i
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- python3 tools/block_micro.py "$@" 5 > gpurun_out/pmc_${tag}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
rm -rf gpurun_out/tr_$tag
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$tag -o run --output-format csv -- python3 tools/block_micro.py "$@" > gpurun_out/tr_$tag.log 2>&1 || exit 1
python3 tools/pmc_kernels.py "gpurun_out/pmc_${tag}_*" ${FILT:-k_}
cut -d, -f1-8 gpurun_out/tr_$tag/*kernel_stats.csv | head -30
