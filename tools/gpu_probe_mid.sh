cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_preact_mid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 tools/probe_time.py k_pm_fwd k_pm_bwd2 k_pm_w2grad k_pm_w13grad k_pm_t2 k_pm_bwd1 2>&1 | grep -v Warn
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline | python3 -c "import json,sys; print(json.load(sys.stdin)['ms_per_step'])"
