# SQ stall breakdown of the dominant kernel (one counter pass)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/sq1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES -d gpurun_out/sq1 -o run --output-format csv -- python3 tools/dominant_kernel.py 5 > gpurun_out/sq1.log 2>&1 || { tail -20 gpurun_out/sq1.log; exit 1; }
rm -rf gpurun_out/sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/sq2 -o run --output-format csv -- python3 tools/dominant_kernel.py 5 > gpurun_out/sq2.log 2>&1 || { tail -20 gpurun_out/sq2.log; exit 1; }
echo ok
