# The GPU test suite (optionally a subset: extra pytest args), then bench.py probe timings.
#   gpurun -- bash tools/gpu_tests.sh TAG "PROBES" [pytest args...]
set -o pipefail
tag=$1; probes=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$probes" ]; then timeout -k 10 200 python3 tools/probe_time.py $probes 2>&1 | grep -v amdgpu.ids; fi
