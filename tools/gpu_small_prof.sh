# kernel trace of the bench step with the fused few-channel backward on every grid
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_small
VQ3D_SMALL_BWD_MAX_VOX=1000000000 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_small -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/prof_small.log 2>&1 || { tail -20 gpurun_out/prof_small.log; exit 1; }
echo ok
