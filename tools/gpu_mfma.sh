# MFMA utilisation pass over one eager bench step:  gpurun -- bash tools/gpu_mfma.sh TAG
set -o pipefail
tag=${1:-m}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
rm -rf gpurun_out/pmc_mfma_$tag
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_mfma_$tag -o run --output-format csv -- \
    python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/pmc_mfma_$tag.log 2>&1 \
    || { tail -20 gpurun_out/pmc_mfma_$tag.log; exit 1; }
python3 tools/mfma_util.py gpurun_out/pmc_mfma_$tag --md gpurun_out/mfma_util_$tag.md | head -40
