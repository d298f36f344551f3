set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6bench; mkdir -p $O
for i in 1 2; do timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1; grep '^{"metric"' $O/bench_$i.log | tail -1 > $O/bench_$i.json; python3 -c "
import json; d=json.load(open('$O/bench_$i.json')); print('C3', round(d['value']/1e6,1), 'mirror', round(d['host_mirror']['env_steps_per_s']/1e6,1), 'C4', round(d['two_ply']['root_decisions_per_s']/1e6,3), 'H128', round(d['two_ply_h128']['root_decisions_per_s']/1e6,3), 'PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1), 'upd', round(d['ppo_iteration']['update_s']*1e3,2), 'C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,1), 'frac', round(d['roofline']['frac'],4), 'cpu', round(d['cpu_baseline']['value']/1e3,1))"; done
