#!/bin/bash
# Build the library of git revision REV (default HEAD) into exp/libbgx_old.so for tools/ab.sh.
set -e
REV=${1:-HEAD}
rm -rf exp/old && mkdir -p exp/old/csrc exp/old/include
for f in bg_core.h bg_engine.h bg_engine.hip bg_mlp.hip bg_search.hip bg_ppo.hip; do git show $REV:mlp-ppo-2ply-p3_amd/csrc/$f > exp/old/csrc/$f 2>/dev/null || rm -f exp/old/csrc/$f; done
git show $REV:include/bgx.h > exp/old/include/bgx.h
cd exp/old/csrc && sed -i 's#"../../include/bgx.h"#"../include/bgx.h"#' *.hip *.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form -I../include bg_engine.hip bg_search.hip bg_mlp.hip $(ls bg_ppo.hip 2>/dev/null) -o ../../libbgx_old.so
