# A/B of two library builds (3d-vq-vae-2_amd/lib/libvq3d_a.so vs _b.so, selected with VQ3D_LIB):
#   gpurun -- bash tools/gpu_ab.sh conv [SHAPE ...]     conv launch times (tools/conv_ab.py)
#   gpurun -- bash tools/gpu_ab.sh probe PROBE ...      bench.py kernel probes (tools/probe_time.py)
#   gpurun -- bash tools/gpu_ab.sh bench [BENCH ARGS]   bench.py step time (a, b, a, b)
mode=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ "$mode" = bench ]; then
  for v in a b a b; do
    VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline "$@" > gpurun_out/bab_$v.json 2> gpurun_out/bab_$v.err || { tail -5 gpurun_out/bab_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value'],2), d['unit'])" gpurun_out/bab_$v.json $v
  done
  exit 0
fi
tool=tools/conv_ab.py; [ "$mode" = probe ] && tool=tools/probe_time.py
for v in a b; do
  echo "== $v"
  VQ3D_LIB=$GRAFT_REPO_ROOT/3d-vq-vae-2_amd/lib/libvq3d_$v.so timeout -k 10 300 python3 $tool "$@" > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$v.log
done
