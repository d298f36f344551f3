#!/bin/bash
# Round-4 first GPU pass: the -m gpu suite (incl. the one-rank RCCL + capture-failure tests),
# the C3 step-time series against game age, then the default bench line.
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/step_series.py --steps 1600 --window 20 > $O/series.json 2> $O/series.err || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
exit 0
