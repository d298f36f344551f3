#!/bin/bash
# Build an A/B variant of libbgx.so into build/libbgx_NAME.so with extra hipcc
# flags (e.g. -DBGX_PARENT_BSEARCH); run it with BGX_LIB=build/libbgx_NAME.so.
# Usage: tools/build_variant.sh NAME [FLAGS...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p build
C=mlp-ppo-2ply-p3_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form -Iinclude "$@" \
  -o build/libbgx_$NAME.so $C/bg_engine.hip $C/bg_mlp.hip $C/bg_search.hip $C/bg_ppo.hip $C/bg_ppo_fused.hip
