#!/bin/bash
# A/B the standalone policy kernel timing (tools/policy_time.py): in-tree vs exp/libbgx_old.so
set -e
for i in 1 2; do
  echo new; timeout -k 10 200 python tools/policy_time.py 2>&1 | grep us
  echo old; BGX_LIB=exp/libbgx_old.so timeout -k 10 200 python tools/policy_time.py 2>&1 | grep us
done
