set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/profile.sh r6final --steps 20 --warmup 5 > gpurun_out/r6final_profile.log 2>&1
tail -5 gpurun_out/r6final_profile.log
