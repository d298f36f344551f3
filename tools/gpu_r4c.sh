#!/bin/bash
# Round-4: phase probe (GPU vs host time of short windows), evaluator A/B + counters, bench.
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/phase_probe.py > $O/phase.log 2>&1 || exit 1
A="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 2 --c2-steps 0 --mirror-steps 0"
timeout -k 10 200 python bench.py $A > $O/eval_rw.log 2>&1 || exit 1
E="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0 --mirror-steps 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_eval" --output-format csv -d $O/mfma -o run -- python bench.py $E > $O/mfma.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_eval" --output-format csv -d $O/wait -o run -- python bench.py $E > $O/wait.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py $E > $O/trace.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_train.py tests/test_gpu_ppo_fused.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
bash tools/prof_update.sh r4c_upd > $O/update.txt 2>&1 || exit 1
exit 0
