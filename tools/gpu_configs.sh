# The other BASELINE configurations and the eager (no HIP graph) step, one GPU call:
#   gpurun -- bash tools/gpu_configs.sh TAG
set -o pipefail
tag=${1:-cfg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-roofline "$@" > gpurun_out/bench_${tag}_$n.json 2> gpurun_out/bench_${tag}_$n.err \
    || { tail -5 gpurun_out/bench_${tag}_$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'ms', d.get('launch'))" gpurun_out/bench_${tag}_$n.json $n
}
run eager --eager --no-cpu-baseline && run cfg4 --encode-only --no-cpu-baseline && run cfg2 --config 2l_pub --no-cpu-baseline && run cfg5 --prior
