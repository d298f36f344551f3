#!/bin/bash
# SQ counters of the C3 step kernels (policy + env step), two --pmc passes.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/sqp
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --horizon 0 --no-cpu-baseline --two-ply-batches 0 --c2-steps 0"
RX="k_policy_act|k_step"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_F16 --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python bench.py $ARGS > $OUT/p1.log 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python bench.py $ARGS > $OUT/p2.log 2>&1 || true
SQ_MIN_WAVES=100 python tools/sq_summary.py $OUT/p1 $OUT/p2
