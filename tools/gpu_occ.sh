set -e -o pipefail
mkdir -p gpurun_out
for bpc in 0 2 4 8 16; do for m in fwd dgrad; do
  VQ3D_VERBOSE=1 VQ3D_MFMA_BLOCKS_PER_CU=$bpc timeout -k 10 120 python tools/conv_micro.py 4 4 512 512 128 3 1 1 1 $m bf16 20 >> gpurun_out/occ.log 2>&1
  VQ3D_MFMA_BLOCKS_PER_CU=$bpc timeout -k 10 120 python tools/conv_micro.py 9 9 128 128 32 3 1 1 1 $m bf16 20 >> gpurun_out/occ.log 2>&1
done; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python tools/conv_micro.py 4 4 512 512 128 3 1 1 1 fwd bf16 3 > gpurun_out/pmc1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc2 -o run -- python tools/conv_micro.py 4 4 512 512 128 3 1 1 1 fwd bf16 3 > gpurun_out/pmc2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc3 -o run -- python tools/conv_micro.py 4 4 512 512 128 3 1 1 1 fwd bf16 3 > gpurun_out/pmc3.log 2>&1
