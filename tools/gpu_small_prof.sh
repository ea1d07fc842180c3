# fused few-channel PreAct blocks: bench with the per-conv backward, kernel trace of the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline"
VQ3D_SMALL_BWD=0 timeout -k 10 240 $B > gpurun_out/small_b0.json 2>/dev/null || exit 1
tail -c 300 gpurun_out/small_b0.json
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_small -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/prof_small.log 2>&1 || { tail -20 gpurun_out/prof_small.log; exit 1; }
echo ok
