# fused 18-channel block forward: time with phases skipped (VQ3D_PM_DBG bits) per brick geometry
set -o pipefail
mkdir -p gpurun_out
for b in 16; do for d in 0 1 2 4 7; do
  VQ3D_PM_BRICK=$b VQ3D_PM_DBG=$d timeout -k 10 120 python -c "
import sys, torch; sys.path.insert(0, '3d-vq-vae-2_amd'); import bench
r = bench.dominant_kernel_roofline('bf16', torch.device('cuda:0'))
print('brick $b dbg $d', round(r['avg_launch_us'], 2), 'us')" 2>/dev/null || exit 1
done; done
