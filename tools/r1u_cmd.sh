export TMPDIR=/tmp
O=gpurun_out/r1u; mkdir -p $O
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $O/p1 -o run -- python tools/bench_conv.py --iters 3 > $O/p1.log 2>&1 || exit 1
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_IFETCH SQ_LDS_BANK_CONFLICT -d $O/p2 -o run -- python tools/bench_conv.py --iters 3 > $O/p2.log 2>&1 || exit 1
$P --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE -d $O/p3 -o run -- python tools/bench_conv.py --iters 3 > $O/p3.log 2>&1 || exit 1
echo done
