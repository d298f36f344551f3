#!/bin/bash
# C3 A/B over bench.py argument sets / env prefixes: tools/ab_args.sh "ENV=1 --shards 2" "--shards 4" ...
# (each set run twice, interleaved; extra args appended to a C3-only bench command)
mkdir -p gpurun_out
for rep in 1 2; do
  n=0
  for set in "$@"; do
    n=$((n + 1))
    envs=$(echo "$set" | tr ' ' '\n' | grep '=' | grep -v '^--' | tr '\n' ' ')
    args=$(echo "$set" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
    env $envs timeout -k 10 200 python bench.py --steps 400 --two-ply-batches 0 --c2-steps 0 --horizon 0 \
      --no-cpu-baseline --mirror-steps 0 $args > gpurun_out/aba_$n.log 2>&1 || { echo "[$set] failed"; tail -5 gpurun_out/aba_$n.log; exit 1; }
    python -c "import json;l=json.loads([x for x in open('gpurun_out/aba_$n.log').read().splitlines() if x.startswith('{')][-1]);print('[$set]',round(l['value']/1e6,1))"
  done
done
