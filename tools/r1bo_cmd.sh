set -u
bash tools/gpu_session.sh r1bo t:tests/test_conv_engine.py t:tests/test_hip_parity.py benchab prof && \
timeout -k 10 120 python tools/prof_summary.py gpurun_out/r1bo/prof/run_kernel_trace.csv --top 60 > gpurun_out/r1bo/prof_summary.txt
