# slab pointwise kernel: workgroup cap sweep on the 128x128x32 shapes
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pwcap.log
for a in "18 9 128 128 32" "9 18 128 128 32"; do
for cap in 2048 1024 512; do
  VQ3D_PW_SG=0 VQ3D_PW_SLAB_BLOCKS=$cap timeout -k 10 120 python tools/pw_micro.py $a 20 2>/dev/null | sed "s/^/cap$cap /" >> gpurun_out/pwcap.log || exit 1
done; done
cat gpurun_out/pwcap.log
