set -o pipefail
out=gpurun_out/r6/caps; mkdir -p $out
ARGS="--steps 2 --warmup 1 --two-ply-batches 2 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0"
for opt in "" "BGX_2PLY_EVAL_WG=1" "BGX_2PLY_ENUM_CAP=2" "BGX_2PLY_EVAL_WG=1,BGX_2PLY_ENUM_CAP=3" ""; do
  timeout -k 10 200 python3 tools/bench_with_options.py "$opt" $ARGS > $out/run.log 2>&1 || { tail -5 $out/run.log; exit 1; }
  echo "[$opt] $(tail -1 $out/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); t=d['two_ply']; h=d['two_ply_h128']
print('C4', round(t['root_decisions_per_s']/1e6,3), 'one-engine enum', round(t['one_engine']['enumeration_ms_per_batch'],2), 'eval', round(t['one_engine']['evaluation_ms_per_batch'],2), '| H128', round(h['root_decisions_per_s']/1e6,3), 'eval', round(h['evaluation_ms_per_batch'],2), 'issued', t['roofline']['issued_over_algorithmic'])")"
done
