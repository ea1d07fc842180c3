# k^3 MFMA weight gradient: workgroup-count sweep (VQ3D_WGM_NBX) vs the lines engine
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/wgm.log
for a in "9 9 128 128 32 3 1 1 1" "4 4 256 256 64 3 1 1 1" "8 8 256 256 64 3 1 1 1" "4 4 32 32 8 3 1 1 1"; do
  VQ3D_LINES_WGRAD=1 timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed "s/^/lines   /" >> gpurun_out/wgm.log || exit 1
  for cap in 100000 768 512 384 256; do
    VQ3D_WGM_NBX=$cap timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed "s/^/cap$cap /" >> gpurun_out/wgm.log || exit 1
  done
done
cat gpurun_out/wgm.log
