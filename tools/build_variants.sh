#!/bin/bash
# Tuning builds of libpatrolhip with overridden kernel constants, for A/B
# timing on the GPU box (PATROLHIP_LIB=tools/var/<name>.so python tools/exp_c2.py).
# Usage: tools/build_variants.sh "name:-DPHIP_HOT_MAX=640 -DPHIP_HOT_LDS=1024" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/var
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-value \
    -Iinclude -DPHIP_BUILD_ID='"variant-'$name'"' $defs -shared -o tools/var/$name.so patrol_amd/csrc/phip_engine.hip patrol_amd/csrc/phip_group.hip patrol_amd/csrc/phip_host.cpp patrol_amd/csrc/phip_udp.cpp patrol_amd/csrc/phip_batcher.cpp -lrccl &
done
wait
ls -la tools/var
