# scalar-weight pointwise kernel: GPU tests, then A/B graph-replay timings against the slab kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
: > gpurun_out/pw_ab.log
for a in "72 36 32 32 8" "36 72 32 32 8" "8 4 32 32 8" "64 32 16 16 4" "18 9 128 128 32" "9 18 128 128 32"; do
  VQ3D_PW_SG=1 timeout -k 10 120 python tools/pw_micro.py $a 20 2>/dev/null | sed 's/^/sg   /' >> gpurun_out/pw_ab.log || exit 1
  VQ3D_PW_SG=0 timeout -k 10 120 python tools/pw_micro.py $a 20 2>/dev/null | sed 's/^/slab /' >> gpurun_out/pw_ab.log || exit 1
done
cat gpurun_out/pw_ab.log
