# Round-5 checks: selected GPU tests, then the N=2 data-parallel bench path rehearsed on one GPU
# (two gloo ranks sharing device 0: VQ3D_RANKS_SHARE_GPU=1), then a short N=1 bench.
#   gpurun -- bash tools/gpu_rehearse.sh TAG [pytest files...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
VQ3D_RANKS_SHARE_GPU=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline \
    --no-roofline > gpurun_out/bench2_$tag.json 2> gpurun_out/bench2_$tag.err || { tail -30 gpurun_out/bench2_$tag.err; exit 1; }
cat gpurun_out/bench2_$tag.json
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/bench1_$tag.json \
    2> gpurun_out/bench1_$tag.err || { tail -30 gpurun_out/bench1_$tag.err; exit 1; }
cat gpurun_out/bench1_$tag.json
