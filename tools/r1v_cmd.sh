set -e
bash tools/gpu_session.sh r1y t:tests/test_conv_engine.py
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r1y/bc -o run -- python tools/bench_conv.py --iters 10 > gpurun_out/r1y/bench_conv.log 2>&1
echo done
