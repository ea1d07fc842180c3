# time the lines engine with phases skipped (VQ3D_LINES_DBG bits: 1 staging, 2 MFMA, 4 stores)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/phase.log
for a in "9 9 128 128 32 3 1 1 1" "2 2 512 512 128 3 1 1 1" "36 36 32 32 8 3 1 1 1"; do
for dbg in 0 1 2 4 3 6 5 7; do
  echo "dbg=$dbg" >> gpurun_out/phase.log
  VQ3D_LINES_DBG=$dbg timeout -k 10 120 python tools/conv_micro.py $a fwd bf16 20 2>&1 | grep -v amdgpu.ids >> gpurun_out/phase.log || exit 1
done; done
cat gpurun_out/phase.log
