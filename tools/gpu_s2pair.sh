cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_ab_probe.sh "k_dgrad_s2<4_4" || exit 1
rm -f 3d-vq-vae-2_amd/lib/libvq3d_a.so 3d-vq-vae-2_amd/lib/libvq3d_b.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pr_t.log 2>&1; rc=$?; tail -2 gpurun_out/pr_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline | python3 -c "import json,sys; print(json.load(sys.stdin)['ms_per_step'])"
