# usage: bash scratch/r6_c4ab.sh TAG "libA libB ..."
set -o pipefail
tag=$1; libs=$2
out=gpurun_out/r6/c4_$tag; mkdir -p $out
for r in 1 2; do
  for L in $libs; do
    lib=$L; [ "$L" = cur ] && lib=mlp-ppo-2ply-p3_amd/bgx/libbgx.so
    BGX_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --two-ply-batches 2 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > $out/${L##*/}_$r.log 2>&1 || { tail -5 $out/${L##*/}_$r.log; exit 1; }
    echo "$L round $r: $(tail -1 $out/${L##*/}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); t=d['two_ply']; h=d['two_ply_h128']
print('C4', round(t['root_decisions_per_s']/1e6,3), 'one-engine enum', round(t['one_engine']['enumeration_ms_per_batch'],2), 'eval', round(t['one_engine']['evaluation_ms_per_batch'],2), '| H128', round(h['root_decisions_per_s']/1e6,3), 'eval', round(h['evaluation_ms_per_batch'],2))")"
  done
done
