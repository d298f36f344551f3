set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/pol; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy.py tests/test_gpu_train.py > $O/tests.log 2>&1
tail -3 $O/tests.log
for i in 1 2; do timeout -k 10 200 python3 bench.py --steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > $O/c3_$i.log 2>&1; tail -1 $O/c3_$i.log | cut -c1-200; done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/c3trace -o c3 -- python3 bench.py --steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > $O/c3trace.log 2>&1
f=$(find $O/c3trace -name "*kernel_trace.csv" | head -1)
gzip -c "$f" > $O/c3trace.csv.gz && rm -f "$f"
