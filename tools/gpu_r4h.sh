#!/bin/bash
# Round-4: the factored 2-ply evaluator -- search parity tests, then a C4 A/B:
# factored (default) / full 13-k-block form (BGX_2PLY_UNFACTORED) / the narrow
# evaluator at 2 waves per SIMD (variants/libbgx_wpe2.so).
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 200 --timeout-method thread > $O/tests_search.log 2>&1 || { tail -40 $O/tests_search.log; exit 1; }
tail -2 $O/tests_search.log
A="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 3 --c2-steps 0 --mirror-steps 0"
timeout -k 10 200 python bench.py $A > $O/fact.log 2>&1 || exit 1
BGX_2PLY_UNFACTORED=1 timeout -k 10 200 python bench.py $A > $O/full.log 2>&1 || exit 1
BGX_LIB=$PWD/variants/libbgx_wpe2.so timeout -k 10 200 python bench.py $A > $O/fact_wpe2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py $A > $O/fact2.log 2>&1 || exit 1
python - <<'PY'
import json
for f in ["fact", "full", "fact_wpe2", "fact2"]:
    l = json.loads([x for x in open(f"gpurun_out/r4h/{f}.log").read().splitlines() if x.startswith("{")][-1])
    print(f, *[f"{k}: {l[k]['root_decisions_per_s']/1e6:.3f}M enum {l[k]['enumeration_ms_per_batch']:.2f} eval {l[k]['evaluation_ms_per_batch']:.2f}" for k in ("two_ply", "two_ply_h128")])
PY
