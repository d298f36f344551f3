#!/bin/bash
# Round-4: PPO update fixes (tests + kernel trace of an update) and the bench line.
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo_fused.py tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
bash tools/prof_update.sh r4d_upd > $O/update.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
exit 0
