#!/bin/bash
# SQ counters of the env-step kernels on the C3 step alone (two --pmc passes, each its own run).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/sqs
mkdir -p $OUT
ARGS="--steps 100 --warmup 5 --two-ply-batches 0 --horizon 0 --no-cpu-baseline --c2-steps 0"
RX="k_step|k_policy"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python bench.py $ARGS > $OUT/p2.log 2>&1
SQ_MIN_WAVES=100 python tools/sq_summary.py $OUT/p1 $OUT/p2
