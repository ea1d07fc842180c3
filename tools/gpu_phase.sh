# time the lines engine with phases skipped (VQ3D_LINES_DBG bits: 1 staging, 2 MFMA, 4 stores),
# with in-kernel vs pre-packed weight images
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/phase.log
for a in "9 9 128 128 32 3 1 1 1" "1 1 128 128 32 3 1 1 1"; do
for pp in 0 1; do
for dbg in 0 1 2 4 7; do
  echo "prepack=$pp dbg=$dbg" >> gpurun_out/phase.log
  VQ3D_LINES_PREPACK=$pp VQ3D_LINES_DBG=$dbg timeout -k 10 120 python tools/conv_micro.py $a fwd bf16 20 2>&1 | grep -v amdgpu.ids >> gpurun_out/phase.log || exit 1
done; done; done
cat gpurun_out/phase.log
