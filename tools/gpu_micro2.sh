# k^3 lines-engine micro timings (graph replay): fwd and dgrad of the chain shapes
set -o pipefail
for m in fwd dgrad; do
for a in "9 9 128 128 32 3 1 1 1" "1 1 128 128 32 3 1 1 1" "2 2 512 512 128 3 1 1 1" "36 36 32 32 8 3 1 1 1" "16 16 8 8 2 3 1 1 1" "4 4 32 32 8 3 1 1 1" "4 4 256 256 64 3 1 1 1"; do
  timeout -k 10 120 python tools/conv_micro.py $a $m bf16 20 2>&1 | grep -v amdgpu.ids || exit 1
done; done
