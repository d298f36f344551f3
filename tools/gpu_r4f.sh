#!/bin/bash
# Round-4 re-entry pass: the whole -m gpu suite, smoke(), the default bench line, then the
# staged register-weight evaluators (BGX_EVAL_FORM=r): parity and a C4 A/B against the
# LDS-weight form.
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
BGX_EVAL_FORM=r timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > $O/tests_search_r.log 2>&1 || { tail -30 $O/tests_search_r.log; exit 1; }
A="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 2 --c2-steps 0 --mirror-steps 0"
BGX_EVAL_FORM=r timeout -k 10 200 python bench.py $A > $O/eval_r.log 2>&1 || exit 1
timeout -k 10 200 python bench.py $A > $O/eval_lds.log 2>&1 || exit 1
exit 0
