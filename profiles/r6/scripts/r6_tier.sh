set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/tailfuse; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_dropin.py > $O/tests.log 2>&1
tail -3 $O/tests.log
A="--steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0"
for i in 1 2; do
  for v in prev new; do
    if [ $v = new ]; then L=mlp-ppo-2ply-p3_amd/bgx/libbgx.so; else L=scratch/lib_$v.so; fi
    BGX_LIB=$L timeout -k 10 200 python3 bench.py $A > $O/${v}_$i.log 2>&1; echo "$v 200 $(grep -o '"value": [0-9.]*' $O/${v}_$i.log | head -1)"
    BGX_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > $O/${v}_s20_$i.log 2>&1; echo "$v 20 $(grep -o '"value": [0-9.]*' $O/${v}_s20_$i.log | head -1)"
  done
done
