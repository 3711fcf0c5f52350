set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for v in 1 2; do
cp dro-sfm_amd/ab_occ$v.so dro-sfm_amd/libdro_amd.so
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abprof$v -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/abprof$v.log 2>&1
done
