mkdir -p gpurun_out/r3t
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_multirank.py tests/test_gpu_ppo_fused.py -q --timeout 300 --timeout-method thread > gpurun_out/r3t/train.log 2>&1; tail -3 gpurun_out/r3t/train.log
BGX_HEAVY_WPE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dropin.py -q --timeout 200 --timeout-method thread > gpurun_out/r3t/eng.log 2>&1; tail -2 gpurun_out/r3t/eng.log
timeout -k 10 300 python bench.py --steps 20 --two-ply-batches 0 --c2-steps 0 --no-cpu-baseline --mirror-steps 0 > gpurun_out/r3t/ppo.log 2>&1 && python -c "import json;l=json.loads([x for x in open('gpurun_out/r3t/ppo.log').read().splitlines() if x.startswith('{')][-1]);p=l['ppo_iteration'];print('PPO',round(p['env_steps_per_s_incl_update']/1e6,1),round(p['rollout_s']*1e3,2),round(p['update_s']*1e3,2))"
bash tools/ab_args.sh "--shards 2" "BGX_HEAVY_WPE=4 --shards 2"
