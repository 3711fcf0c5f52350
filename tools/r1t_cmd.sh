set -e
bash tools/gpu_session.sh r1t t:tests/test_conv_engine.py tests
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1t/bc -o run -- python tools/bench_conv.py --iters 10 > gpurun_out/r1t/bench_conv.log 2>&1
python tools/prof_configs.py gpurun_out/r1t/bc/run_kernel_trace.csv dconv igemm wgrad finish > gpurun_out/r1t/bc_configs.txt 2>&1 || true
bash tools/gpu_session.sh r1t benchq
