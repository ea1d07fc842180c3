# kernel-trace stats of tools/conv_ab.py shapes with library b:  gpurun -- bash tools/gpu_prof_conv.sh SHAPE ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_b.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pwg -o run --output-format csv -- python3 tools/conv_ab.py "$@" > gpurun_out/pwg.log 2>&1 || { tail gpurun_out/pwg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pwg.log | grep " us " || true
f=$(find gpurun_out/pwg -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -14
