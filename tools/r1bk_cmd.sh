set -u
bash tools/gpu_session.sh r1bk t:tests/test_conv_engine.py t:tests/test_hip_parity.py t:tests/test_graph_step.py benchab && \
DRO_CONV_NO_THIN=1 bash tools/gpu_session.sh r1bk_nothin benchab
