# wgrad_ds tests + A/B of the weight-gradient shapes it covers (libvq3d_a.so = before, _b = after)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_engines.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wg.log 2>&1; rc=$?; tail -3 gpurun_out/t_wg.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh conv 4,4,512,512,128,3,1,1,1,wgrad 4,4,512,512,128,4,2,1,1,wgrad 8,8,256,256,64,4,2,1,1,wgrad 16,16,128,128,32,4,2,1,1,wgrad 4,8,512,512,128,2,2,0,0,wgrad 8,16,256,256,64,2,2,0,0,wgrad
