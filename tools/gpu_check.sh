#!/bin/bash
# One GPU round trip: the -m gpu suite, smoke(), the default bench line, then
# optional C4 evaluator A/B variants (tools/ab_eval.sh NAME...).  Usage:
#   tools/gpu_check.sh TAG [AB_VARIANTS...]     (outputs under gpurun_out/TAG/)
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc         # 1 = test failures (keep going), else a crash / time limit
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python - $O/bench.log <<'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1])
print("C3", round(l["value"] / 1e6, 1), "M  C4", round(l["two_ply"]["root_decisions_per_s"] / 1e6, 3),
      round(l["two_ply_h128"]["root_decisions_per_s"] / 1e6, 3), "C2", round(l["one_ply_selfplay"]["env_steps_per_s"] / 1e6, 1),
      "PPO", round(l["ppo_iteration"]["env_steps_per_s_incl_update"] / 1e6, 1))
PY
[ $# -gt 0 ] && bash tools/ab_eval.sh "$@"
exit 0
