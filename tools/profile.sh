#!/bin/bash
# Run on the GPU box (via gpurun): kernel-trace/stats pass + two separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) of the same bench command, then summarize
# into gpurun_out/$TAG/summary.json.  Usage: tools/profile.sh TAG [bench args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py "$@" > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python bench.py "$@" > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python bench.py "$@" > $OUT/write.log 2>&1
python tools/summarize_profile.py $OUT "$*"
cp $OUT/summary.json gpurun_out/$TAG.summary.json
cp $OUT/trace/run_kernel_stats.csv gpurun_out/$TAG.kernel_stats.csv
