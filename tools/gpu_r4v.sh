#!/bin/bash
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c4_shards.py --shards 2 --hidden 40 > $O/s2h40.json 2> $O/s2h40.err || { tail -20 $O/s2h40.err; exit 1; }
cat $O/s2h40.json
timeout -k 10 300 python -u tools/c4_shards.py --shards 4 --hidden 40 > $O/s4h40.json 2> $O/s4h40.err || { tail -20 $O/s4h40.err; exit 1; }
cat $O/s4h40.json
timeout -k 10 300 python -u tools/c4_shards.py --shards 2 --hidden 128 > $O/s2h128.json 2> $O/s2h128.err || { tail -20 $O/s2h128.err; exit 1; }
cat $O/s2h128.json
