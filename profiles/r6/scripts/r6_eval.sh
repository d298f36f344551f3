# usage: bash scratch/r6_eval.sh TAG [tests]
set -o pipefail
tag=$1; mode=${2:-tests}
out=gpurun_out/r6/$tag; mkdir -p $out
if [ "$mode" = tests ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
  tail -1 $out/gpu_tests.log
fi
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$i.log 2>&1 || { tail -20 $out/bench_$i.log; exit 1; }
  tail -1 $out/bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('C3', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],4), 'ms | C4', round(d['two_ply']['root_decisions_per_s']/1e6,3), 'H128', round(d['two_ply_h128']['root_decisions_per_s']/1e6,3), '| C2', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,1), '| PPO', round(d['ppo_iteration']['env_steps_per_s_incl_update']/1e6,1), 'upd', round(d['ppo_iteration']['update_s']*1e3,2), 'roll', round(d['ppo_iteration']['rollout_s']*1e3,2))"
done
