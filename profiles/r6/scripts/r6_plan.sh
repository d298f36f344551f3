set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/plan; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo_fused.py -k "plan or gather" > $O/tests.log 2>&1; tail -2 $O/tests.log
N=2 ROUNDS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/ppo_ab.py "" > $O/run.log 2>&1
f=$(find $O -name "*kernel_stats.csv" | head -1); grep -E "k_plan|k_gather" "$f" | cut -d, -f1-6
