set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6/sq2; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --burn-in 150 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0 --mirror-steps 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_eval" --output-format csv -d $OUT/p2 -o run -- python bench.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_eval" --output-format csv -d $OUT/p1 -o run -- python bench.py $ARGS > $OUT/p1.log 2>&1
SQ_MIN_WAVES=100 python tools/sq_summary.py $OUT/p1 $OUT/p2 | tee $OUT/summary.txt
