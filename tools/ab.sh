#!/bin/bash
# A/B the bench between the in-tree library and exp/libbgx_old.so on ONE box,
# interleaved.  Usage: tools/ab.sh ROUNDS [bench args...]
set -e
R=$1; shift
for i in $(seq 1 $R); do
  timeout -k 10 300 python bench.py "$@" > gpurun_out/ab_new_$i.log 2>&1
  BGX_LIB=exp/libbgx_old.so timeout -k 10 300 python bench.py "$@" > gpurun_out/ab_old_$i.log 2>&1
done
