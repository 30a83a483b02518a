#!/bin/bash
# Build an ablation variant of libsqr: sqr_conv3.hip with -DSQR_EXP=<bits> (see its header),
# everything else as the default build.  Output: sq-recovery_amd/sqr/libsqr_exp<bits>.so
#   bash tools/build_exp.sh 128 [extra hipcc flags...]
set -euo pipefail
EXP=$1; shift
cd "$(dirname "$0")/.."
make -s -C sq-recovery_amd/csrc >/dev/null
OBJ=build/obj
mkdir -p build/exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DSQR_EXP=$EXP "$@" \
  -c sq-recovery_amd/csrc/sqr_conv3.hip -o build/exp/sqr_conv3_$EXP.o
OTHERS=$(ls $OBJ/*.o | grep -v sqr_conv3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o sq-recovery_amd/sqr/libsqr_exp$EXP.so build/exp/sqr_conv3_$EXP.o $OTHERS
echo sq-recovery_amd/sqr/libsqr_exp$EXP.so
