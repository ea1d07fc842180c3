# pointwise weight gradient on mid-size grids: workgroup cap sweep (direct atomics at <= 16)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pww_mid.log
for a in "72 36 32 32 8 1 1 0 0" "36 72 32 32 8 1 1 0 0" "8 4 32 32 8 1 1 0 0" "64 32 16 16 4 1 1 0 0"; do
for cap in 0 8 16 32; do
  VQ3D_PWW_MID_NBX=$cap timeout -k 10 120 python tools/conv_micro.py $a wgrad bf16 20 2>/dev/null | sed "s/^/cap$cap /" >> gpurun_out/pww_mid.log || exit 1
done; done
cat gpurun_out/pww_mid.log
