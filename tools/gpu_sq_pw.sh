# SQ counters for the pointwise kernels at 128x128x32
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in fwd wgrad; do
rm -rf gpurun_out/sqp_$m
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/sqp_$m -o run --output-format csv -- python3 tools/pw_kernel.py 9 18 128 128 32 $m 5 > gpurun_out/sqp_$m.log 2>&1 || { tail -20 gpurun_out/sqp_$m.log; exit 1; }
rm -rf gpurun_out/trp_$m
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trp_$m -o run -- python3 tools/pw_kernel.py 9 18 128 128 32 $m 5 > gpurun_out/trp_$m.log 2>&1 || { tail -20 gpurun_out/trp_$m.log; exit 1; }
done
echo ok
