#!/bin/bash
# Round-4 measurement pass at HEAD: the C3 step-time series against game age (1,600 steps
# from reset), then tools/profile.sh (kernel trace of the default bench command, env-step
# HBM / SQ passes, evaluator, policy-kernel and enumerator counter passes).
O=gpurun_out/r4p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/step_series.py --steps 1600 --window 20 > $O/series.json 2> $O/series.err || { tail -5 $O/series.err; exit 1; }
bash tools/profile.sh r4p > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -40 $O/profile.log
# keep what comes back under gpurun's 64 MiB: the big raw CSVs compressed
find gpurun_out/r4p -name '*.csv' -size +1M -exec gzip -9 {} \;
du -sh gpurun_out/r4p
