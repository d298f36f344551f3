#!/bin/bash
# Round-4: the staged register-weight evaluators (BGX_EVAL_FORM=r) -- parity, A/B against
# the LDS-weight form, counters; the PPO fixes (tests, update trace); the bench line.
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
BGX_EVAL_FORM=r timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > $O/tests_search_r.log 2>&1 || { tail -30 $O/tests_search_r.log; exit 1; }
A="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 2 --c2-steps 0 --mirror-steps 0"
BGX_EVAL_FORM=r timeout -k 10 200 python bench.py $A > $O/eval_r.log 2>&1 || exit 1
timeout -k 10 200 python bench.py $A > $O/eval_lds.log 2>&1 || exit 1
E="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0 --mirror-steps 0"
BGX_EVAL_FORM=r timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_eval" --output-format csv -d $O/mfma -o run -- python bench.py $E > $O/mfma.log 2>&1 || exit 1
BGX_EVAL_FORM=r timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_eval" --output-format csv -d $O/wait -o run -- python bench.py $E > $O/wait.log 2>&1 || exit 1
BGX_EVAL_FORM=r timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py $E > $O/trace.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo_fused.py -x -q --timeout 200 --timeout-method thread > $O/tests_train.log 2>&1 || { tail -30 $O/tests_train.log; exit 1; }
bash tools/prof_update.sh r4e_upd > $O/update.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
exit 0
