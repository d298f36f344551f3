set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6/c3trace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6/c3trace -o c3 -- python3 bench.py --steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > gpurun_out/r6/c3trace/bench.log 2>&1
f=$(find gpurun_out/r6/c3trace -name "*kernel_trace.csv" | head -1)
gzip -c "$f" > gpurun_out/r6/c3trace/trace.csv.gz && rm -f "$f"
tail -1 gpurun_out/r6/c3trace/bench.log | cut -c1-300
