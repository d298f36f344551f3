# A/B of env knobs on one box: tools/tf.sh VAR "v1 v2 ..."
VAR=$1; VALS=$2
for f in $VALS; do env $VAR=$f timeout -k 10 300 python bench.py --no-cpu-baseline --two-ply-batches 0 --horizon 0 > gpurun_out/tf_$f.log 2>&1 || exit 1; grep "^{" gpurun_out/tf_$f.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$VAR=$f', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],3))"; done
