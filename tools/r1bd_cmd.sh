set -u
bash tools/gpu_session.sh r1bd pmc roof && \
STAMP_DBG=0 bash tools/gpu_session.sh r1bd stampdbg prof && \
timeout -k 10 120 python tools/prof_summary.py gpurun_out/r1bd/prof/run_kernel_trace.csv --top 45 > gpurun_out/r1bd/prof_summary.txt
