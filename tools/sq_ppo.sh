#!/bin/bash
# SQ counters of the fused PPO head kernels over one tools/ppo_time.py run (two --pmc
# passes, each its own run).  Usage: tools/sq_ppo.sh TAG
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
RX="k_ppo_rows|k_ppo_gw2"
N=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_BRANCH --kernel-include-regex "$RX" --output-format csv -d $OUT/p1 -o run -- python tools/ppo_time.py > $OUT/p1.log 2>&1
N=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$RX" --output-format csv -d $OUT/p2 -o run -- python tools/ppo_time.py > $OUT/p2.log 2>&1
SQ_MIN_WAVES=100 python tools/sq_summary.py $OUT/p1 $OUT/p2
