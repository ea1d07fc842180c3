# bench.py step time under environment settings, each run twice in alternation:
#   gpurun -- bash tools/gpu_env_ab.sh "" "VQ3D_SMALL_MMA_MAX=4096" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for set in "$@"; do
    i=$((i + 1))
    env $set timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > gpurun_out/eab_$i.json 2> gpurun_out/eab_$i.err || { tail -5 gpurun_out/eab_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), round(d['ms_per_step'],3), 'ms')" gpurun_out/eab_$i.json "$set"
  done
done
