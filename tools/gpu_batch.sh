# One GPU call for a round's check-in: the model-level fp16/bf16 parity test (printed numbers), the
# rest of the GPU suite, kernel probe timings, phase-skip experiment libraries, SQ counter passes.
#   gpurun --timeout 1200 -- bash tools/gpu_batch.sh TAG "PROBES" "EXP_PROBES" "EXP_LIBS" "PMC_PROBES"
set -o pipefail
tag=$1; probes=$2; xprobes=$3; xlibs=$4; pmc=$5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_model.py -q -s --timeout 300 --timeout-method thread \
    > gpurun_out/model_$tag.log 2>&1
rc=$?
grep -E "3L-pub|passed|failed" gpurun_out/model_$tag.log
[ $rc -le 1 ] || exit $rc   # 1 = a parity bound missed (read the log); anything else: stop
bash tools/gpu_tests.sh $tag "$probes" --deselect tests/test_gpu_bf16_model.py || exit 1
if [ -n "$xlibs" ]; then bash tools/gpu_exp_probe.sh "$xprobes" $xlibs || exit 1; fi
if [ -n "$pmc" ]; then bash tools/gpu_pmc_probe.sh $tag $pmc > gpurun_out/pmc_$tag.txt 2>&1 || exit 1; fi
echo batch done
