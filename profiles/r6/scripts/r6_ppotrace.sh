set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/ppotrace2; mkdir -p $O
N=3 ROUNDS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/ppo_ab.py "" > $O/run.log 2>&1
f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/stats.csv
f=$(find $O -name "*kernel_trace.csv" | head -1); gzip -c "$f" > $O/trace.csv.gz; rm -f "$f"
