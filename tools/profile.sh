#!/bin/bash
# Run on the GPU box (via gpurun).  Pass 1: --kernel-trace --stats of the bench
# command as given (the committed per-kernel summary).  Then counter passes, each in
# its own run (rocprofv3 does not split counters over passes):
#   fetch / write  FETCH_SIZE, WRITE_SIZE of the env-step kernels on the C3 step alone
#                  (the extras -- 2-ply, PPO update, CPU baseline -- do not change the
#                  env-step kernels, and counter collection serializes every dispatch)
#   sqi / sqc      SQ instruction counts and wave-cycle split of the same kernels (the
#                  env step's issue-rate roofline)
#   mfma / efetch  the 2-ply evaluators (H 40 and H 128): MFMA busy cycles + VALU
#                  counters, and HBM read bytes
#   eval2          the evaluators' wave-time split
#   pol1 / pol2    the C3 policy kernel k_policy_act: MFMA / VALU issue, wave-time split
#   enum1 / enum2  the 2-ply reply enumerators: instruction mix, wave-time split
# Summary -> gpurun_out/$TAG/summary.json.   Usage: tools/profile.sh TAG [bench args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
PMC_ARGS="--steps 200 --warmup 10 --two-ply-batches 0 --horizon 0 --no-cpu-baseline --c2-steps 0 --mirror-steps 0"
REGEX='k_step|k_order|k_movegen_over'
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py "$@" > $OUT/trace.log 2>&1
# the C3 step alone, kernel trace only: the env-step kernels' durations over the timed window
export C3TRACE_ARGS="--steps 200 --warmup 10 --two-ply-batches 0 --horizon 0 --no-cpu-baseline --c2-steps 0 --mirror-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c3trace -o run -- python bench.py $C3TRACE_ARGS > $OUT/c3trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/fetch -o run -- python bench.py $PMC_ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/write -o run -- python bench.py $PMC_ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH --kernel-include-regex "$REGEX" --output-format csv -d $OUT/sqi -o run -- python bench.py $PMC_ARGS > $OUT/sqi.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$REGEX" --output-format csv -d $OUT/sqc -o run -- python bench.py $PMC_ARGS > $OUT/sqc.log 2>&1
EVAL_ARGS="--steps 2 --warmup 1 --burn-in 150 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0 --mirror-steps 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_eval" --output-format csv -d $OUT/mfma -o run -- python bench.py $EVAL_ARGS > $OUT/mfma.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_eval" --output-format csv -d $OUT/efetch -o run -- python bench.py $EVAL_ARGS > $OUT/efetch.log 2>&1
# the evaluators' wave-time split (round 6)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_eval" --output-format csv -d $OUT/eval2 -o run -- python bench.py $EVAL_ARGS > $OUT/eval2.log 2>&1
# the C3 policy kernel (k_policy_act, round 4): MFMA / VALU issue and the wave-time split
POL='k_policy_act'
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-include-regex "$POL" --output-format csv -d $OUT/pol1 -o run -- python bench.py $PMC_ARGS > $OUT/pol1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH --kernel-include-regex "$POL" --output-format csv -d $OUT/pol2 -o run -- python bench.py $PMC_ARGS > $OUT/pol2.log 2>&1
# the 2-ply reply enumerators (k_enum*, k_enum_tier*): instruction mix and wave-time split
ENUM='k_enum'
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-include-regex "$ENUM" --output-format csv -d $OUT/enum1 -o run -- python bench.py $EVAL_ARGS > $OUT/enum1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$ENUM" --output-format csv -d $OUT/enum2 -o run -- python bench.py $EVAL_ARGS > $OUT/enum2.log 2>&1
python tools/summarize_profile.py $OUT "$*" "$PMC_ARGS"
cp $OUT/summary.json gpurun_out/$TAG.summary.json
cp $OUT/trace/run_kernel_stats.csv gpurun_out/$TAG.kernel_stats.csv
