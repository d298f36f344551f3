#!/bin/bash
# Round-4 experiments: C3 shard phase probe, device->host copy bandwidth, 2-ply evaluator A/B
# (register-weight form vs the LDS-weight form) and their MFMA counters.
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/phase_probe.py > $O/phase.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/copy_probe.py > $O/copy.log 2>&1 || exit 1
A="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 2 --c2-steps 0 --mirror-steps 0"
timeout -k 10 200 python bench.py $A > $O/eval_rw.log 2>&1 || exit 1
BGX_EVAL_FORM=lds timeout -k 10 200 python bench.py $A > $O/eval_lds.log 2>&1 || exit 1
E="--steps 2 --warmup 1 --horizon 0 --no-cpu-baseline --two-ply-batches 1 --c2-steps 0 --mirror-steps 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_eval" --output-format csv -d $O/mfma -o run -- python bench.py $E > $O/mfma.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_eval" --output-format csv -d $O/wait -o run -- python bench.py $E > $O/wait.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py $E > $O/trace.log 2>&1 || exit 1
exit 0
