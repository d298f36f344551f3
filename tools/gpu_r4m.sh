#!/bin/bash
# PPO leg: trainer shards 2/4, forked vs linear steps; then the default bench line (4 linear C3 shards).
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
B="--steps 2 --warmup 1 --horizon 32 --two-ply-batches 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)['ppo_iteration']; print('$1', round(d['env_steps_per_s_incl_update']/1e6,1), 'rollout ms', round(d['rollout_s']*1e3,2), 'upd', round(d['update_s']*1e3,2))"; }
timeout -k 10 200 python bench.py $B > $O/s2f.log 2>&1 && v $O/s2f.log || exit 1
BGX_TR_LINEAR=1 timeout -k 10 200 python bench.py $B > $O/s2l.log 2>&1 && v $O/s2l.log || exit 1
BGX_TR_SHARDS=4 BGX_TR_LINEAR=1 timeout -k 10 200 python bench.py $B > $O/s4l.log 2>&1 && v $O/s4l.log || exit 1
BGX_TR_SHARDS=4 timeout -k 10 200 python bench.py $B > $O/s4f.log 2>&1 && v $O/s4f.log || exit 1
timeout -k 10 120 python -u -m pytest tests/test_gpu_graph.py -q --timeout 100 --timeout-method thread > $O/graph.log 2>&1 || { tail -20 $O/graph.log; exit 1; }
tail -1 $O/graph.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python -c "
import json; l=[x for x in open('$O/bench.log') if x.startswith('{')][-1]; d=json.loads(l)
print('C3', round(d['value']/1e6,1), 'mirror', round(d['host_mirror']['env_steps_per_s']/1e6,1), 'C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,1), 'C4', round(d['two_ply']['root_decisions_per_s']/1e6,3), round(d['two_ply_h128']['root_decisions_per_s']/1e6,3), 'PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1))"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -5 $O/bench20.log; exit 1; }
python -c "
import json; l=[x for x in open('$O/bench20.log') if x.startswith('{')][-1]; d=json.loads(l)
print('20-step C3', round(d['value']/1e6,1), 'mirror', round(d['host_mirror']['env_steps_per_s']/1e6,1), 'C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,1), 'C4', round(d['two_ply']['root_decisions_per_s']/1e6,3), 'PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1))"
