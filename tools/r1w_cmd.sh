export TMPDIR=/tmp
mkdir -p gpurun_out/r1w
for d in 0 1 2 3; do
  DRO_CONV_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r1w/d$d -o run -- python tools/bench_conv.py --iters 5 > gpurun_out/r1w/d$d.log 2>&1 || exit 1
done
echo done
