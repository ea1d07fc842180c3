set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/host_time.py 2>&1 | grep -v amdgpu.ids
for rep in 1 2; do
for set in "" "VQ3D_MID_SIDE=1"; do
  for fl in "" "--eager"; do
    env $set timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline $fl > gpurun_out/r_$rep.json 2> gpurun_out/r_$rep.err || { tail -5 gpurun_out/r_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), round(d['ms_per_step'],3), 'ms')" gpurun_out/r_$rep.json "$set $fl"
  done
done
done
