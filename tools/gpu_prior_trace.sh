set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
rm -rf gpurun_out/tp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/tp -o run --output-format csv -- python3 bench.py --prior --steps 3 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/tp.log 2>&1 || { tail -20 gpurun_out/tp.log; exit 1; }
python3 tools/step_profile.py gpurun_out/tp 50 > gpurun_out/tp.txt; head -50 gpurun_out/tp.txt
