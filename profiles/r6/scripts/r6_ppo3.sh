set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/ppo9; mkdir -p $O
N=6 ROUNDS=3 timeout -k 10 600 python3 tools/ppo_ab.py "FUSED_RETURNS=0" "FUSED_RETURNS=1" > $O/ab.jsonl 2>&1; cat $O/ab.jsonl | grep variant
