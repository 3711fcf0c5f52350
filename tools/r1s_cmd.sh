export TMPDIR=/tmp
mkdir -p gpurun_out/r1s
timeout -k 10 120 rocprofv3 -L > gpurun_out/r1s/counters.txt 2>&1
timeout -k 10 300 python tools/bench_conv.py --iters 30 > gpurun_out/r1s/bench_conv.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/r1s/pmc1 -o run --output-format csv -- python tools/bench_conv.py --iters 5 > gpurun_out/r1s/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/r1s/pmc2 -o run --output-format csv -- python tools/bench_conv.py --iters 5 > gpurun_out/r1s/pmc2.log 2>&1
cat gpurun_out/r1s/bench_conv.log
