# usage: bash scratch/r6_ab.sh TAG "libA libB ..." [steps]
set -o pipefail
tag=$1; libs=$2; steps=${3:-200}
out=gpurun_out/r6/ab_$tag; mkdir -p $out
for r in 1 2 3; do
  for L in $libs; do
    lib=$L; [ "$L" = cur ] && lib=mlp-ppo-2ply-p3_amd/bgx/libbgx.so
    BGX_LIB=$lib timeout -k 10 120 python3 bench.py --steps $steps --warmup 5 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > $out/${L##*/}_$r.log 2>&1 || { tail -5 $out/${L##*/}_$r.log; exit 1; }
    echo "$L round $r: $(tail -1 $out/${L##*/}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), 'M', round(d['ms_per_step']*1e3,1), 'us')")"
  done
done
