#!/bin/bash
# Run on the GPU box (via gpurun).  Pass 1: --kernel-trace --stats of the bench
# command as given (the committed per-kernel summary).  Passes 2-3: FETCH_SIZE and
# WRITE_SIZE counters, each in its own run, of the C3 step alone (the extras --
# 2-ply, PPO update, CPU baseline -- do not change the env-step kernels and make
# counter collection, which serializes every dispatch, too slow), restricted to
# the env-step kernels.  Summary -> gpurun_out/$TAG/summary.json.
# Usage: tools/profile.sh TAG [bench args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
PMC_ARGS="--two-ply-batches 0 --horizon 0 --no-cpu-baseline --c2-steps 0"
REGEX='k_step|k_order|k_movegen_over'
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py "$@" > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/fetch -o run -- python bench.py $PMC_ARGS > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/write -o run -- python bench.py $PMC_ARGS > $OUT/write.log 2>&1
# 2-ply evaluator: MFMA busy cycles and HBM bytes of k_eval (one C4 batch), each its own pass
EVAL_ARGS="--steps 2 --warmup 1 --burn-in 150 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0"
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_eval" --output-format csv -d $OUT/mfma -o run -- python bench.py $EVAL_ARGS > $OUT/mfma.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_eval" --output-format csv -d $OUT/efetch -o run -- python bench.py $EVAL_ARGS > $OUT/efetch.log 2>&1
python tools/summarize_profile.py $OUT "$*" "$PMC_ARGS"
cp $OUT/summary.json gpurun_out/$TAG.summary.json
cp $OUT/trace/run_kernel_stats.csv gpurun_out/$TAG.kernel_stats.csv
