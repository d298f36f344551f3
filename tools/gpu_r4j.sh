#!/bin/bash
# C3 on the device clock: a 200-step run (cadence early vs late) and a 20-step run with
# the HIP API trace (hipGraphLaunch host cost), tools/c3_window.py.
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
B="--warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t200 -o run -- python bench.py --steps 200 $B > $O/b200.log 2>&1 || exit 1
python tools/c3_window.py $O/t200/run_kernel_trace.csv $O/b200.log 200 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/th -o run -- python bench.py --steps 20 $B > $O/bh.log 2>&1 || exit 1
python tools/c3_window.py $O/th/run_kernel_trace.csv $O/bh.log 20 || exit 1
ls $O/th
