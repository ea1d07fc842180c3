# PixelSNAIL prior: attention + model GPU tests, then the cfg5 bench step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pixelsnail.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prior_t.log 2>&1; rc=$?; tail -2 gpurun_out/prior_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --prior --no-cpu-baseline --no-roofline | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'])"
