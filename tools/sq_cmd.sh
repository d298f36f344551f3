#!/bin/bash
# SQ counters for any python script (two --pmc passes).  Usage: tools/sq_cmd.sh TAG script.py [args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $OUT/p1 -o run -- python "$@" > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU --output-format csv -d $OUT/p2 -o run -- python "$@" > $OUT/p2.log 2>&1
python tools/sq_summary.py $OUT > $OUT/sq.txt
