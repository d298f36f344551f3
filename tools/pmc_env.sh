#!/bin/bash
# GPU box: C3 bench line + FETCH_SIZE / WRITE_SIZE passes (each its own run) of
# the env-step kernels, then the per-kernel HBM bytes.  Usage: tools/pmc_env.sh TAG [bench args]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--two-ply-batches 0 --horizon 0 --no-cpu-baseline --c2-steps 0 $*"
REGEX='k_step|k_order|k_movegen_over'
timeout -k 10 200 python bench.py $ARGS > $OUT/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/fetch -o run -- python bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/write -o run -- python bench.py $ARGS > $OUT/write.log 2>&1
python tools/summarize_profile.py $OUT "$ARGS" "$ARGS" > /dev/null || true
