set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6verify; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for i in 1 2; do timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1; grep '^{"metric"' $O/bench_$i.log | tail -1 > $O/bench_$i.json; python3 -c "
import json; d=json.load(open('$O/bench_$i.json')); print('C3', round(d['value']/1e6,1), 'C4', round(d['two_ply']['root_decisions_per_s']/1e6,3), 'H128', round(d['two_ply_h128']['root_decisions_per_s']/1e6,3), 'PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1), 'upd', round(d['ppo_iteration']['update_s']*1e3,2), 'C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,1), 'io', d['two_ply']['roofline'].get('issued_over_algorithmic'))"; done
