#!/bin/bash
# SQ instruction-mix counters, two separate --pmc passes (run on the GPU box).
# Usage: tools/sq.sh TAG [bench args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $OUT/p1 -o run -- python bench.py "$@" > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o run -- python bench.py "$@" > $OUT/p2.log 2>&1
python tools/sq_summary.py $OUT > $OUT/sq.txt
