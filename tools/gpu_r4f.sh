#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite, smoke(), the default bench line.
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python tools/c4_ab.py $O/bench.log
exit 0
