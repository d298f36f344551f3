#!/bin/bash
# The optimizer step as one HIP call (bgx_adam_step): train tests, the update trace, the PPO leg.
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo_fused.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/prof_update.sh r4q_upd > $O/update.txt 2>&1 || exit 1
head -12 $O/update.txt
B="--steps 20 --warmup 5 --horizon 32 --two-ply-batches 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
for r in 1 2; do
timeout -k 10 200 python bench.py $B > $O/ppo$r.log 2>&1 || exit 1
python -c "import json; l=[x for x in open('$O/ppo$r.log') if x.startswith('{')][-1]; d=json.loads(l)['ppo_iteration']; print('PPO', round(d['env_steps_per_s_incl_update']/1e6,1), 'rollout ms', round(d['rollout_s']*1e3,2), 'upd', round(d['update_s']*1e3,2))"
done
