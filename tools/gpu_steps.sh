#!/bin/bash
# One parameterised GPU-box launcher (replaces the round-5 one-off gpu_r05*.sh scripts):
#   gpurun -- bash tools/gpu_steps.sh TAG STEP [STEP ...]
# Each STEP runs under its own time limit, writes gpurun_out/TAG_<name>.log, and the script stops
# at the first failing step (no GPU work after a fault, abort or timeout).  STEPs:
#   gputests            the whole `pytest -m gpu` suite (what the driver runs at round end)
#   tests:<k-expr>      pytest -m gpu -k <k-expr> over tests/ ("_or_" stands for " or ")
#   file:<test file>    pytest -m gpu on one test file
#   smoke               __graft_entry__.smoke()
#   race                tools/dbg/lanes_race.py (PixelSNAIL lanes replays at the published size)
#   bench               bench.py (the headline line) -> gpurun_out/TAG_bench.json
#   eager               bench.py --eager (no HIP graph) -> gpurun_out/TAG_eager.json
#   prior|cfg2|cfg4|cfg4b8   bench.py --prior / --config 2l_pub / --encode-only [--encode-batch 8]
#   prof                rocprofv3 kernel trace + stats of the bench step -> gpurun_out/TAG_prof/, the
#                       step ranking gpurun_out/TAG_step.txt / TAG_step_top.json (tools/step_profile.py)
#   profprior           the same trace for --prior
#   pmc:<probe>         PMC FETCH_SIZE / WRITE_SIZE passes over one bench probe (tools/gpu_traffic.sh)
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider"
run() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "[gpu_steps] $TAG $name: $*"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "[gpu_steps] $TAG $name rc=$rc: $(tail -1 "gpurun_out/${TAG}_${name}.log")"
    return $rc
}
for s in "$@"; do
    case $s in
        gputests) run gputests 1100 $PYT tests || exit $? ;;
        tests:*) k="${s#tests:}"; k="${k//_or_/ or }"  # tests:a_or_b -> -k "a or b"
                 run "tests_$(echo "${s#tests:}" | tr -c 'a-zA-Z0-9_' '_')" 900 $PYT tests -k "$k" || exit $? ;;
        file:*) run "file_$(basename "${s#file:}" .py)" 900 $PYT "${s#file:}" || exit $? ;;
        smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        race) run race 600 python -u tools/dbg/lanes_race.py 3 4 || exit $? ;;
        bench) run bench 600 python -u bench.py || exit $?
               tail -1 "gpurun_out/${TAG}_bench.log" > "gpurun_out/${TAG}_bench.json" ;;
        eager) run eager 600 python -u bench.py --eager --no-cpu-baseline || exit $?
               tail -1 "gpurun_out/${TAG}_eager.log" > "gpurun_out/${TAG}_eager.json" ;;
        prior) run prior 600 python -u bench.py --prior || exit $?
               tail -1 "gpurun_out/${TAG}_prior.log" > "gpurun_out/${TAG}_prior.json" ;;
        cfg2) run cfg2 600 python -u bench.py --config 2l_pub || exit $?
              tail -1 "gpurun_out/${TAG}_cfg2.log" > "gpurun_out/${TAG}_cfg2.json" ;;
        cfg4) run cfg4 600 python -u bench.py --encode-only || exit $?
              tail -1 "gpurun_out/${TAG}_cfg4.log" > "gpurun_out/${TAG}_cfg4.json" ;;
        cfg4b8) run cfg4b8 600 python -u bench.py --encode-only --encode-batch 8 || exit $?
                tail -1 "gpurun_out/${TAG}_cfg4b8.log" > "gpurun_out/${TAG}_cfg4b8.json" ;;
        prof) rm -rf "gpurun_out/${TAG}_prof"
              run prof 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof" -o run --output-format csv -- \
                  python3 -u bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-roofline || exit $?
              python3 tools/step_profile.py "gpurun_out/${TAG}_prof" 60 --json "gpurun_out/${TAG}_step_top.json" \
                  > "gpurun_out/${TAG}_step.txt" || exit $? ;;
        profprior) rm -rf "gpurun_out/${TAG}_profprior"
                   run profprior 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_profprior" -o run \
                       --output-format csv -- python3 -u bench.py --prior --steps 4 --warmup 3 --no-cpu-baseline || exit $? ;;
        pmc:*) bash tools/gpu_traffic.sh "$TAG" "${s#pmc:}" > "gpurun_out/${TAG}_pmc.log" 2>&1 || exit $? ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "[gpu_steps] $TAG done"
