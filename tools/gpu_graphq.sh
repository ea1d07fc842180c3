# HIP-graph branch concurrency A/B: side-stream weight gradients vs serial, graph queue knobs
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/graphq.log
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline"
run() { echo "== $1" >> gpurun_out/graphq.log; shift; timeout -k 10 240 env "$@" 2>>gpurun_out/graphq.err | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'])" >> gpurun_out/graphq.log; }
run default X=1 $B || exit 1
run serial X=1 $B --serial-wgrad || exit 1
run queues2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B || exit 1
run queues4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B || exit 1
run nopacket DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B || exit 1
cat gpurun_out/graphq.log
