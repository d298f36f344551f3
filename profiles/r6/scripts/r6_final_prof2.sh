set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6verify2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6verify2/gpu_tests.log 2>&1
tail -2 gpurun_out/r6verify2/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > gpurun_out/r6verify2/smoke.log 2>&1; tail -1 gpurun_out/r6verify2/smoke.log
bash tools/profile.sh r6final2 --steps 20 --warmup 5 > gpurun_out/r6final2_profile.log 2>&1; echo "profile rc $?"
