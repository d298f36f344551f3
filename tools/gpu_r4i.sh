#!/bin/bash
# Round-4: the new gW1 kernel and argmax reductions (tests), the update trace, and C3 at
# the driver's 20 steps for graph lengths 2 / 4 / 10.
O=gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_train.py tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/prof_update.sh r4i_upd > $O/update.txt 2>&1 || exit 1
head -8 $O/update.txt
B="--warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
for G in 2 4 10; do for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --graph-steps $G $B > $O/g$G.$r.log 2>&1 || exit 1
  python -c "import json; l=[x for x in open('$O/g$G.$r.log') if x.startswith('{')][-1]; d=json.loads(l); print('G=$G steps=20', round(d['value']/1e6,1))"
done; done
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --horizon 32 --no-cpu-baseline --two-ply-batches 2 --mirror-steps 0 > $O/legs.log 2>&1 || exit 1
python tools/c4_ab.py $O/legs.log
python -c "import json; l=[x for x in open('$O/legs.log') if x.startswith('{')][-1]; d=json.loads(l); print('C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,2), 'PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1), 'upd ms', round(d['ppo_iteration']['update_s']*1e3,2))"
