set -o pipefail
mkdir -p gpurun_out/r6/pair_cause
for v in ${VARIANTS:-slp opsel_asm slp_nopack}; do
  BGX_LIB=scratch/lib_$v.so TRIALS=3 timeout -k 10 150 python -u tools/pair_diag.py > gpurun_out/r6/pair_cause/diag_$v.log 2>&1 || { echo "fail $v rc=$?"; exit 1; }
  tail -1 gpurun_out/r6/pair_cause/diag_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', [d[t]['bad'] for t in d])"
done
